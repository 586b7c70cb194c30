# Same-box A/B of build/libval_A.so against each of build/libval_{B,C,D,...}.so
# named in $VARIANTS (default "B C") on the workloads given as arguments
# (tools/ab_libs.py names). Tooling only; no GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abn
mkdir -p $O
rc=0
for v in ${VARIANTS:-B C}; do
  timeout -k 10 600 python tools/ab_libs.py build/libval_A.so build/libval_$v.so "$@" > $O/ab_$v.log 2>&1 || { rc=$?; break; }
done
for v in ${VARIANTS:-B C}; do echo "== A vs $v"; grep -v amdgpu.ids $O/ab_$v.log; done
echo "rc=$rc"; exit $rc
