"""Summarise a rocprofv3 --stats kernel CSV into a markdown table (top-N kernels)."""
import csv
import sys


def main(path, top=30, steps=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    calls = sum(int(r["Calls"]) for r in rows)
    out = [f"Total kernel time {tot/1e6:.1f} ms over {calls} dispatches"
           + (f" ({tot/1e6/steps:.2f} ms and {calls/steps:.0f} dispatches per profiled step)" if steps else ""), "",
           "| total ms | calls | avg us | % | kernel |", "|---:|---:|---:|---:|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        out.append(f"| {float(r['TotalDurationNs'])/1e6:.2f} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                   f"{float(r['Percentage']):.2f} | `{r['Name'][:90]}` |")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30, float(sys.argv[3]) if len(sys.argv) > 3 else None)
