#!/usr/bin/env python3
"""Summarise gpurun_out/pmcs (tools/pmc_short.sh) per workload: per launch of
the frames kernel, instruction counts and waits per KiB of CRC input, and
L2->memory read requests by size. FETCH_SIZE is reported raw and x2 (the
gfx950 rule of MI355X_MICROARCH.md for 16 B/lane streams); the RDREQ size
split says which part of the traffic that rule fits. Tooling only.
Usage: pmc_short_summary.py [dir] > profiles/<name>.json"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcs"


def counters(path):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_frames" not in k:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = k
    if not per:
        return {}, None
    keys = sorted({c for d in per.values() for c in d})
    avg = {c: sum(d.get(c, 0.0) for d in per.values()) / len(per) for c in keys}
    return avg, sorted(set(names.values()))


def kernel_us(path):
    for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_frames" in r["Name"]:
                return float(r["AverageNs"]) / 1e3, r["Name"]
    return None, None


out = {}
for log in sorted(glob.glob(os.path.join(D, "*.trace.log"))):
    w = os.path.basename(log)[:-len(".trace.log")]
    m = re.search(r"algorithmic_bytes_per_launch (\d+)", open(log).read())
    if not m:
        continue
    alg = int(m.group(1))
    kib = alg / 1024.0
    us, kname = kernel_us(os.path.join(D, w, "trace"))
    c = {}
    for p in ("p1", "p2", "p3", "p4"):
        v, _ = counters(os.path.join(D, w, p))
        c.update(v)
    e = {"kernel": kname, "kernel_us": us, "algorithmic_bytes": alg,
         "alg_TB_s": alg / (us * 1e-6) / 1e12 if us else None}
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"):
        if k in c:
            e[k + "_per_KiB"] = c[k] / kib
    if "SQ_WAVE_CYCLES" in c:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_LDS"):
            if k in c:
                e[k + "_frac_of_wave_cycles"] = c[k] / c["SQ_WAVE_CYCLES"]
    if "TCC_EA0_RDREQ_sum" in c:
        r = c["TCC_EA0_RDREQ_sum"]
        e["RDREQ"] = r
        for s in ("32B", "64B", "128B"):
            if f"TCC_EA0_RDREQ_{s}_sum" in c:
                e[f"RDREQ_{s}_frac"] = c[f"TCC_EA0_RDREQ_{s}_sum"] / r if r else None
        b32 = c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        b64 = c.get("TCC_EA0_RDREQ_64B_sum", 0.0)
        b128 = c.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        e["bytes_by_request_size"] = 32 * b32 + 64 * b64 + 128 * b128
        e["bytes_by_request_size_over_alg"] = e["bytes_by_request_size"] / alg
    if "FETCH_SIZE" in c:
        e["FETCH_SIZE_KiB"] = c["FETCH_SIZE"]
        e["fetch_x2_over_alg"] = c["FETCH_SIZE"] * 2048.0 / alg
    for k in ("TCC_HIT_sum", "TCC_MISS_sum", "TCP_TCC_READ_REQ_sum", "TCC_EA0_RDREQ_DRAM_sum", "GRBM_GUI_ACTIVE"):
        if k in c:
            e[k] = c[k]
    out[w] = e
json.dump(out, sys.stdout, indent=1)
print()
