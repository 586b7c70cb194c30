#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv: per kernel name, count and the
median / min duration in microseconds, in launch order. Tooling only."""
import csv
import sys
from collections import OrderedDict
from statistics import median

rows = OrderedDict()
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        if "vcrc" not in name and "rocclr" not in name:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        rows.setdefault(name[:70], []).append(d)
for k, v in rows.items():
    print(f"{k:70s} n={len(v):4d} med={median(v):9.2f} us min={min(v):9.2f} us")
