"""Per-kernel totals from a rocprofv3 rocpd database: python scripts/rocpd_summary.py run_results.db [top] [name-filter]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
flt = sys.argv[3] if len(sys.argv) > 3 else ""
tot = sum(r[0] for r in db.execute("select end - start from kernels")) / 1e6
print(f"total kernel time {tot:.2f} ms")
q = ("select name, grid_x, grid_y, grid_z, count(*), sum(end - start), avg(end - start) from kernels "
     "where name like ? group by name, grid_x, grid_y, grid_z order by sum(end - start) desc limit ?")
for n, gx, gy, gz, cnt, s, a in db.execute(q, (f"%{flt}%", top)):
    print(f"{s / 1e6:8.2f} ms {cnt:6d} x {a / 1e3:7.1f} us  grid ({gx},{gy},{gz})  {n[:90]}")
