# Round-end measurement: tests, smoke, bench lines (cfg3 headline with its
# host_inclusive and cfg4_strong blocks, verify, cfg4, cfg2, cfg5 ragged),
# rocprofv3 kernel trace of the bench command, and separate PMC passes (HBM
# traffic for cfg3 and cfg5, SQ counters), with provenance (VAL_TREE = the
# commit, set by the caller; the box; the library's source hash).
# Then: python tools/round_summary.py gpurun_out/round NN  (on the CPU side).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
echo "{\"tree\": \"${VAL_TREE:-unknown}\", \"box\": \"$(hostname)\", \"date\": \"$(date -u +%FT%TZ)\", \"lib_srchash\": \"$(cat $R/val_protocol_amd/libval_crc_hip.so.srchash)\"}" > $O/provenance.json
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python bench.py --verify --no-cpu-baseline > $O/bench_verify.json 2> $O/bench_verify.err && \
timeout -k 10 600 python bench.py --config cfg4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
timeout -k 10 600 python bench.py --config cfg2 --no-cpu-baseline --steps 200 > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 600 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 $R/bench.py --no-cpu-baseline > $O/trace.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace5 -o bench -- python3 $R/bench.py --config cfg5 --no-cpu-baseline > $O/trace5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- python3 $R/tools/prof_target.py cfg3 3 > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- python3 $R/tools/prof_target.py cfg3 3 > $O/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_v -o p -- python3 $R/tools/prof_target.py cfg3 3 verify > $O/pmc_fetch_v.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch5 -o p -- python3 $R/tools/prof_target.py cfg5 3 > $O/pmc_fetch5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write5 -o p -- python3 $R/tools/prof_target.py cfg5 3 > $O/pmc_write5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -o p -- python3 $R/tools/prof_target.py cfg3 3 > $O/pmc_sq.log 2>&1 && \
cd $R && bash tools/pmc_short.sh u1100d cfg2 > $O/pmc_short.log 2>&1
echo "round profile rc=$?"
# short-frame PMC passes land in gpurun_out/pmcs: python tools/pmc_short_summary.py > profiles/rNN_pmc_short.json
