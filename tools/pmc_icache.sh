# Instruction-cache and wait counters of k_region (8 MiB) and k_frames (cfg2), separate passes.
set -o pipefail
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/icache; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $O/ic_region -o p -- python3 $R/tools/prof_region.py 8388608 20 > $O/ic_region.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_IFETCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $O/sq_region -o p -- python3 $R/tools/prof_region.py 8388608 20 > $O/sq_region.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $O/ic_cfg2 -o p -- python3 $R/tools/prof_target.py cfg2 20 > $O/ic_cfg2.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_IFETCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $O/sq_cfg2 -o p -- python3 $R/tools/prof_target.py cfg2 20 > $O/sq_cfg2.log 2>&1
rc=$?
for f in ic_region sq_region ic_cfg2 sq_cfg2; do echo "== $f"; python3 - "$O/$f/p_counter_collection.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-40:]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
done
exit $rc
