#!/usr/bin/env python3
"""Group a rocprofv3 kernel_trace.csv of prof_small.py by spec: the vcrc
kernels in launch order, REPS (x kernels per call) per spec; prints the median
duration of each spec's launches. usage: kt_groups.py TRACE REPS spec... Tooling only."""
import csv
import sys
from statistics import median

trace, reps, specs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(trace))
               if "vcrc" in r["Kernel_Name"]))
per = len(rows) // (reps * len(specs))
for i, s in enumerate(specs):
    grp = rows[i * reps * per:(i + 1) * reps * per]
    calls = [grp[j * per:(j + 1) * per] for j in range(reps)]
    d = [(c[-1][1] - c[0][0]) / 1000 for c in calls]
    parts = " ".join(f"{c[2].split('(')[0].split('::')[-1][:18]}={median([(x[j][1] - x[j][0]) / 1000 for x in calls]):.1f}"
                     for j, c in enumerate(calls[0]))
    print(f"{s:16s} kernels/call={per} med={median(d):8.2f} us min={min(d):8.2f} us  {parts}")
