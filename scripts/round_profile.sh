#!/bin/bash
# usage: scripts/round_profile.sh <round> [workloads]   (run on the GPU box)
# GPU parity tests, one bench line per workload, then rocprofv3 kernel stats + PMC
# passes (scripts/prof.sh) for each workload; everything lands under gpurun_out/.
set -o pipefail
RND=${1:-r03}; WLS=${2:-"c2 c3 c4 c5 ref"}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for wl in $WLS; do
  timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 3 > gpurun_out/${RND}_${wl}_bench.json 2> gpurun_out/bench_$wl.err || { echo "bench $wl failed"; tail -20 gpurun_out/bench_$wl.err; exit 1; }
  cut -c 1-300 gpurun_out/${RND}_${wl}_bench.json
done
for wl in $WLS; do
  bash scripts/prof.sh $wl gpurun_out/prof_$wl > gpurun_out/prof_$wl.log 2>&1 || { echo "prof $wl failed"; tail -20 gpurun_out/prof_$wl.log; exit 1; }
  echo "profiled $wl"
done
