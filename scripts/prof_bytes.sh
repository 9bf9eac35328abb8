#!/bin/bash
# usage: scripts/prof_bytes.sh <workload> <outdir> [lib]   (run on the GPU box)
# HBM-side bytes of a workload's kernels: FETCH_SIZE and WRITE_SIZE in passes of their own (they cannot
# share one: MI355X_MICROARCH.md), optionally on a variant build (MSA_LIB_PATH) -- e.g. the MSA_ABL
# ablations that drop one buffer's stores, to attribute the counted bytes per buffer
set -e
WL=$1; OUT=$2; LIB=${3:-}
export TMPDIR=/tmp
mkdir -p $OUT
[ -n "$LIB" ] && export MSA_LIB_PATH=$LIB
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 scripts/prof_run.py $WL 3
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 scripts/prof_run.py $WL 2
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 scripts/prof_run.py $WL 2
# instruction mix of the same variant (SQ counters share a pass; attributes VALU per pass with MSA_ABL=1)
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -d $OUT/pmc_sq -o run --output-format csv -- python3 scripts/prof_run.py $WL 2
