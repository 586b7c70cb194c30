# Round 6: the driver's bench command at the final tree, twice.
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.$i.json 2> $O/bench.$i.err || exit 5
  python3 -c "import json; d=json.load(open('$O/bench.$i.json')); r=d['roofline']; s=d['cfg4_strong']; print(d['value'], r['kernel_ms'], r['frac'], r['read_roof'], r['frac_of_read_roof'], r['traffic_source']['same_library_sources'], '| block', s['per_rank'][0]['kernel_ms'], s['roofline']['frac'], '| proxy', {k:(v['kernel_ms'], v['est_aggregate_GiB_s']) for k,v in d['cfg4_strong_proxy'].items() if k in '1248'})"
done
