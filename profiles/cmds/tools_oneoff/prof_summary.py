"""Summarise decode kernel durations from a rocprofv3 sqlite output (diagnostic)."""
import glob
import sqlite3
import sys

db = glob.glob(f"gpurun_out/{sys.argv[1]}/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select name, grid_x, duration from kernels where name like '%decode%' order by start").fetchall()
k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n = len(rows) // k
for i in range(k):
    part = rows[i * n:(i + 1) * n]
    sp = [d for nm, gx, d in part if "split" in nm]
    mg = [d for nm, gx, d in part if "split" not in nm]
    print(i, part[0][1], round(sum(sp) / len(sp) / 1e3, 2), round(sum(mg) / len(mg) / 1e3, 2))
