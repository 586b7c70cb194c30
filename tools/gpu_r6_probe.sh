# Round 6 probe on one MI355X: the self-launching bench (--gpus 8 over gloo),
# the cfg4 block against standalone cfg4 (warm-up and placement A/B, two
# alternations), the single-GPU 1/2/4/8 proxy, and the bounce-copy scaling.
# Any failure ends the script there.
set -o pipefail
O=gpurun_out/r6
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multiproc.py \
    > $O/pytest_multiproc.log 2>&1 || { tail -30 $O/pytest_multiproc.log; exit 3; }
tail -3 $O/pytest_multiproc.log
summ() { python3 - "$1" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
s = d.get("cfg4_strong") or {}
r = s.get("roofline") or {}
print(sys.argv[1].split("/")[-1], "value", d["value"], "kern", d["roofline"]["kernel_ms"],
      "| block", s.get("per_rank", [{}])[0].get("kernel_ms"), "warm", s.get("warmup_launches"),
      "roof", r.get("read_roof"), "frac", r.get("frac"), "of_roof", r.get("frac_of_read_roof"))
p = d.get("cfg4_strong_proxy")
if p:
    print("  proxy", {k: (v["kernel_ms"], v["est_aggregate_GiB_s"]) for k, v in p.items() if k in "1248"})
EOF
}
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg4 --warmup 5 --no-cpu-baseline --no-host-inclusive > $O/cfg4_alone.$i.json 2> $O/cfg4_alone.$i.err || exit 4
  summ $O/cfg4_alone.$i.json
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.$i.json 2> $O/driver.$i.err || exit 5
  summ $O/driver.$i.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --block-warmup-ms 100 > $O/bw100.$i.json 2> $O/bw100.$i.err || exit 6
  summ $O/bw100.$i.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cfg4-alloc-first --no-cfg4-proxy > $O/allocfirst.$i.json 2> $O/allocfirst.$i.err || exit 7
  summ $O/allocfirst.$i.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-cfg4-proxy > $O/nogap.$i.json 2> $O/nogap.$i.err || exit 8
  summ $O/nogap.$i.json
done
timeout -k 10 300 python tools/bounce_copy_scaling.py --pinned 1 > $O/bounce_copy_scaling.jsonl 2> $O/bounce.err || exit 9
cat $O/bounce_copy_scaling.jsonl
