#!/usr/bin/env python3
"""Summarise tools/pmc_mem.sh: per tag, CRC-kernel average ms and every
counter averaged per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    tags = sorted({os.path.basename(p)[2:] for p in glob.glob(os.path.join(d, "t_*")) if os.path.isdir(p)})
    for t in tags:
        ms = float("nan")
        for p in glob.glob(os.path.join(d, f"t_{t}", "*kernel_stats.csv")):
            with open(p, newline="") as f:
                for r in csv.DictReader(f):
                    if "k_frames" in r["Name"]:
                        ms = float(r["AverageNs"]) / 1e6
        vals = defaultdict(float)
        disp = defaultdict(set)
        for p in glob.glob(os.path.join(d, f"p*_{t}", "*counter_collection.csv")):
            with open(p, newline="") as f:
                for r in csv.DictReader(f):
                    if "k_frames" in r["Kernel_Name"]:
                        vals[r["Counter_Name"]] += float(r["Counter_Value"])
                        disp[r["Counter_Name"]].add((p, r["Dispatch_Id"]))
        line = " ".join(f"{k}={vals[k] / max(1, len(disp[k])):.4g}" for k in sorted(vals))
        print(f"{t}: ms={ms:.4f} {line}")


if __name__ == "__main__":
    main(sys.argv[1])
