set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1
grep -i -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_SALU\|SQ_WAIT_INST_ANY\|SQ_INST_CYCLES_SALU\|SQC_TC_INST[A-Z_]*" gpurun_out/avail.txt | sort -u
