# Round 6: lanes per frame for the cfg4 proxy's slices (tools/slice_geometry_probe.py).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6n
mkdir -p $O
timeout -k 10 600 python -u tools/slice_geometry_probe.py > $O/slice_geometry.jsonl 2> $O/slice_geometry.err
rc=$?; cat $O/slice_geometry.jsonl; tail -n 5 $O/slice_geometry.err; exit $rc
