# Ragged tail timeline (-DVCRC_TIMING build) and geometry A/Bs of short frames. Tooling only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tg; mkdir -p $O
timeout -k 10 300 python tools/timing_ragged_tail.py build/libval_T.so cfg5log > $O/tail_cfg5log.log 2>&1 && \
timeout -k 10 300 python tools/ab_geom.py u1100d 0:-1 4:2 8:1 2:1 > $O/geom.log 2>&1 && \
timeout -k 10 300 python tools/ab_geom.py s1100 0:-1 4:2 8:1 >> $O/geom.log 2>&1 && \
timeout -k 10 300 python tools/ab_geom.py u4200d 0:-1 4:2 8:1 >> $O/geom.log 2>&1 && \
timeout -k 10 300 python tools/ab_geom.py u600d 0:-1 2:2 4:1 >> $O/geom.log 2>&1
rc=$?; grep -v amdgpu $O/tail_cfg5log.log | head -8; grep -v amdgpu $O/geom.log; echo rc=$rc; exit $rc
