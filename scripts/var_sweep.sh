#!/bin/bash
# usage (GPU box): VARS="a b" scripts/var_sweep.sh -- C2 kernel time of diagnostic builds variants/<v>.so
set -o pipefail
for rep in 1 2; do
  for v in ${VARS}; do
    MSA_LIB_PATH=variants/$v.so timeout -k 10 60 python -u scripts/sweep_m.py 10000 10000 > gpurun_out/var_$v.log 2>&1 || exit 1
    echo "$v $(grep '^h' gpurun_out/var_$v.log)"
  done
done
