# quick iteration: GPU tests then the geometry sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 900 python tools/sweep_geometry.py ${SWEEP_CFGS:-cfg3 cfg2 cfg4} > gpurun_out/sweep.log 2>&1
echo done
