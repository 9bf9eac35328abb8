#!/bin/bash
# usage (GPU box): scripts/prof_round.sh "<workloads>"  -- rocprofv3 kernel stats + PMC passes
# (scripts/prof.sh) for each workload into gpurun_out/prof_<wl>; summarise them here with
# scripts/pmc_summary.py into profiles/<round>_<wl>_*.
set -o pipefail
mkdir -p gpurun_out
for wl in $1; do
  bash scripts/prof.sh $wl gpurun_out/prof_$wl > gpurun_out/prof_$wl.log 2>&1 || { echo "prof $wl failed"; tail -20 gpurun_out/prof_$wl.log; exit 1; }
  echo "profiled $wl"
done
