#!/bin/bash
# usage: scripts/gpu_round.sh   (run on the GPU box): GPU parity tests, then benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for wl in ${WLS:-c2 c4}; do
  timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 3 > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err || { echo "bench $wl failed"; tail -20 gpurun_out/bench_$wl.err; exit 1; }
  cat gpurun_out/bench_$wl.json
done
