#!/bin/bash
# usage (GPU box): scripts/gpu_bench_round.sh <round> "<name:bench args;...>"
# one full bench line per entry (CPU baseline included) -> gpurun_out/<round>_<name>_bench.json
set -o pipefail
RND=$1
mkdir -p gpurun_out
IFS=';' read -ra BL <<< "$2"
for b in "${BL[@]}"; do
  name="${b%%:*}"; args="${b#*:}"
  timeout -k 10 400 python -u bench.py $args > gpurun_out/${RND}_${name}_bench.json 2> gpurun_out/${RND}_${name}_bench.err
  rc=$?
  [ $rc -eq 0 ] || { echo "bench $name failed (status $rc)"; tail -5 gpurun_out/${RND}_${name}_bench.err; exit 2; }
  cut -c 1-240 gpurun_out/${RND}_${name}_bench.json
done
