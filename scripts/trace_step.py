"""Dump the kernel sequence of ONE timed step from a rocprofv3 kernel-trace CSV (after bench.py's
marker kernel): index, start offset (us), duration (us), stream (or queue) id, name.  Usage: trace_step.py <csv> <steps>"""
import csv
import sys


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = max(i for i, r in enumerate(rows) if "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower())
    win = rows[idx + 1:]
    per = len(win) // steps
    step = win[per * (steps - 1):]  # the last step
    t0 = int(step[0]["Start_Timestamp"])
    for i, r in enumerate(step):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Stream_Id", r.get("Queue_Id", ""))
        print(f"{i}\t{(s - t0) / 1e3:.1f}\t{(e - s) / 1e3:.1f}\t{q}\t{r['Kernel_Name'][:110]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
