#!/bin/bash
# usage: scripts/build_variant.sh <name> [-DFOO=1 ...]: vlib/libmsa_<name>.so from the in-tree sources with
# extra defines (A/B builds for scripts/gpu_variants.sh; built here, on the CPU)
set -e
name=$1; shift
mkdir -p vlib
D=cse305_parallel_sequence_alignment_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-strict-aliasing -fPIC -shared -Iinclude "$@" \
  -o vlib/libmsa_$name.so $D/msa_capi.hip
