# Micro-benchmarks on the GPU box (tooling only): each bench/micro binary
# named as an argument (with its own arguments after a colon, e.g. mb14:600),
# under its own time limit; PROF=1 adds a rocprofv3 kernel trace of each.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/micro; mkdir -p $O
for spec in "$@"; do
  b=${spec%%:*}; a=""; [ "$b" != "$spec" ] && a=${spec#*:}
  if [ "${PROF:-0}" = 1 ]; then
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/trace_$b -o p -- $R/bench/micro/$b $a > $O/$b.log 2>&1) || { echo "$b failed"; exit 1; }
  else
    timeout -k 10 300 $R/bench/micro/$b $a > $O/$b.log 2>&1 || { echo "$b failed"; exit 1; }
  fi
  grep -v amdgpu.ids $O/$b.log
done
echo "rc=0"
