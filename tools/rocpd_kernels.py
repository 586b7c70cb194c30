"""Kernel durations from a rocprofv3 rocpd database (the default output
format): per (kernel, grid) in dispatch order, count / median / min in us."""
import collections
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
agg = collections.OrderedDict()
for name, start, end, gx, wx in rows:
    short = name.split("(")[0]
    agg.setdefault((short[-60:], gx // max(wx, 1)), []).append((end - start) / 1000.0)
for (n, wgs), v in agg.items():
    v = sorted(v)
    print(f"{n:60s} wgs={wgs:5d} n={len(v):4d} med={v[len(v) // 2]:9.2f} us min={v[0]:9.2f} us")
