#!/usr/bin/env python3
"""Summarise tools/pmc_ragged.sh output: per tag, the CRC kernel's average
duration and its PMC counters (summed over its dispatches / dispatch count)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def kernel_rows(path):
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if "k_frames" in r["Kernel_Name"]:
                yield r


def main(d):
    tags = sorted({os.path.basename(p)[2:] for p in glob.glob(os.path.join(d, "t_*")) if os.path.isdir(p)})
    print(f"{'tag':18s} {'ms':>7s} {'waves':>7s} {'VALU/wave':>9s} {'LDS/wave':>9s} {'conf/LDS':>9s} "
          f"{'waitany/cyc':>11s} {'waitLDS/cyc':>11s} {'VMEM/wave':>9s} {'fetch GB':>9s}")
    for t in tags:
        ms = float("nan")
        for p in glob.glob(os.path.join(d, f"t_{t}", "*kernel_stats.csv")):
            with open(p, newline="") as f:
                for r in csv.DictReader(f):
                    if "k_frames" in r["Name"]:
                        ms = float(r["AverageNs"]) / 1e6
        c = defaultdict(float)
        disp = set()
        for p in glob.glob(os.path.join(d, f"p_{t}", "*counter_collection.csv")) + \
                glob.glob(os.path.join(d, f"f_{t}", "*counter_collection.csv")):
            for r in kernel_rows(p):
                c[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add((p, r["Dispatch_Id"]))
        nd = max(1, len({x for x in disp if "/p_" in x[0]}))
        nf = max(1, len({x for x in disp if "/f_" in x[0]}))
        waves = c["SQ_WAVES"] / nd
        cyc = c["SQ_WAVE_CYCLES"] or 1.0
        print(f"{t:18s} {ms:7.3f} {waves:7.0f} {c['SQ_INSTS_VALU'] / max(1, c['SQ_WAVES']):9.0f} "
              f"{c['SQ_INSTS_LDS'] / max(1, c['SQ_WAVES']):9.0f} {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_INSTS_LDS']):9.3f} "
              f"{c['SQ_WAIT_ANY'] / cyc:11.2f} {c['SQ_WAIT_INST_LDS'] / cyc:11.2f} "
              f"{c['SQ_INSTS_VMEM_RD'] / max(1, c['SQ_WAVES']):9.0f} {c['FETCH_SIZE'] / nf * 1024 * 2 / 1e9:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcr")
