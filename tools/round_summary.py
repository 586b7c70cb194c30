#!/usr/bin/env python3
"""Assemble profiles/rNN_summary.json (+ pmc_<cfg>.json and the kernel-stat
CSVs) from the output of tools/gpu_round_profile.sh.
usage: round_summary.py [gpurun_out/round] [round_no]"""
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.pmc_traffic import per_launch  # noqa: E402


def bench_line(path):
    try:
        with open(path) as f:
            return json.loads(f.read().strip().splitlines()[-1])
    except Exception:
        return None


def alg_bytes(log):
    m = re.search(r"algorithmic_bytes_per_launch (\d+)", open(log).read())
    return int(m.group(1))


def traffic(o, fetch, write, cfg, out_name):
    fcsv = os.path.join(o, fetch, "p_counter_collection.csv")
    if not os.path.exists(fcsv):
        return None
    alg = alg_bytes(os.path.join(o, fetch + ".log"))
    fk, nd = per_launch(fcsv, "FETCH_SIZE")
    wk = None
    if write:
        wcsv = os.path.join(o, write, "p_counter_collection.csv")
        wk, _ = per_launch(wcsv, "WRITE_SIZE") if os.path.exists(wcsv) else (None, 0)
    rd, wr = fk * 1024 * 2, (wk or 0.0) * 1024
    d = {"config": cfg, "dispatches": nd, "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk,
         "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
         "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (rd + wr) / alg,
         "correction": "gfx950: FETCH_SIZE x1024 x2 (half-count of 16 B/lane streaming reads), WRITE_SIZE x1024"}
    prov = os.path.join(o, "provenance.json")
    if os.path.exists(prov):  # bench.py reports it as roofline.traffic_source
        d["source"] = dict(json.load(open(prov)), method="rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate "
                                                          "passes over tools/prof_target.py (3 launches)")
    with open(os.path.join(ROOT, "profiles", out_name), "w") as f:
        json.dump(d, f, indent=1)
    return d


def kernel_trace(o, sub, rnd, tag, prefer=None):
    d = os.path.join(o, sub)
    stats = os.path.join(d, "bench_kernel_stats.csv")
    if not os.path.exists(stats):
        return None
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"r{rnd:02d}_bench_{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(d, "bench_kernel_trace.csv"))))
    crc = [r for r in rows if "vcrc::" in r["Kernel_Name"]]
    with open(os.path.join(ROOT, "profiles", f"r{rnd:02d}_bench_{tag}_crc_dispatches.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "duration_ns"])
        for r in crc:
            w.writerow([r["Dispatch_Id"], r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])])
    kstats = list(csv.DictReader(open(stats)))
    pick = [r for r in kstats if prefer and prefer in r["Name"]] or kstats  # the config's own kernel first
    top = max(pick, key=lambda r: float(r["TotalDurationNs"]))
    main = [r for r in crc if r["Kernel_Name"] == top["Name"]]
    steps = int(os.environ.get("BENCH_STEPS", "20"))  # bench.py's timed steps (default 20, after 15 warmup)
    warmup = int(os.environ.get("BENCH_WARMUP", "15"))
    # bench.py launches nothing of this kernel before its warmup steps (non-verify
    # runs); after the timed steps come its per-step pass, the host_inclusive
    # block and (cfg5) the verify windows, so the timed launches are counted
    # from the front
    timed = main[warmup:warmup + steps]
    last = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    return {"kernel": top["Name"], "dispatches": int(top["Calls"]), "avg_ms_all_dispatches": float(top["AverageNs"]) / 1e6,
            "timed_dispatches": len(last),
            "avg_ms_timed_region": sum(last) / len(last) / 1e6 if last else None}


def main():
    o = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "round")
    rnd = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    s = {"round": rnd, "source": "tools/gpu_round_profile.sh on one MI355X (gpurun)"}
    s["bench_line_cfg3"] = bench_line(os.path.join(o, "bench.json"))
    s["other_bench_lines"] = [b for b in (bench_line(os.path.join(o, f"bench_{k}.json"))
                                          for k in ("verify", "cfg4", "cfg2", "cfg5")) if b]
    # the headline's own kernel (8 lanes per 16,400-B frame); the cfg4 block and its proxy add more G = 16 time
    s["rocprof_cfg3"] = kernel_trace(o, "trace", rnd, "cfg3", prefer="k_frames<8, 1, false, false")
    s["rocprof_cfg5"] = kernel_trace(o, "trace5", rnd, "cfg5", prefer="k_frames_ragged")
    s["pmc_traffic_cfg3"] = traffic(o, "pmc_fetch", "pmc_write", "cfg3", "pmc_cfg3.json")
    s["pmc_traffic_cfg3_verify"] = traffic(o, "pmc_fetch_v", None, "cfg3_verify", "pmc_cfg3_verify.json")
    s["pmc_traffic_cfg5"] = traffic(o, "pmc_fetch5", "pmc_write5", "cfg5", "pmc_cfg5.json")
    sq = os.path.join(o, "pmc_sq", "p_counter_collection.csv")
    if os.path.exists(sq):
        names = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY",
                 "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"]
        s["pmc_sq_cfg3_per_launch"] = {n: per_launch(sq, n)[0] for n in names}
        q = s["pmc_sq_cfg3_per_launch"]
        s["sq_wait_any_over_wave_cycles"] = q["SQ_WAIT_ANY"] / q["SQ_WAVE_CYCLES"]
        s["lds_bank_conflict_cycles_per_lds_instr"] = q["SQ_LDS_BANK_CONFLICT"] / q["SQ_INSTS_LDS"]
    prov = os.path.join(o, "provenance.json")
    if os.path.exists(prov):
        s["provenance"] = json.load(open(prov))
    pt = os.path.join(o, "pytest_gpu.log")
    if os.path.exists(pt):
        s["pytest_gpu_tail"] = open(pt).read().strip().splitlines()[-2:]
    out = os.path.join(ROOT, "profiles", f"r{rnd:02d}_summary.json")
    with open(out, "w") as f:
        json.dump(s, f, indent=1)
    print(json.dumps({k: s[k] for k in ("bench_line_cfg3", "rocprof_cfg3", "pmc_traffic_cfg3")}, indent=1)[:3000])


if __name__ == "__main__":
    main()
