# time one plan under several library builds: VARIANTS="name ..." (vlib/libmsa_<name>.so, "prod" = in-tree),
# ARGS = scripts/time_plan.py arguments
set -o pipefail
mkdir -p gpurun_out
for v in $VARIANTS; do
  if [ "$v" = prod ]; then lib=cse305_parallel_sequence_alignment_amd/libmsa.so; else lib=vlib/libmsa_$v.so; fi
  MSA_LIB_PATH=$lib timeout -k 10 120 python scripts/time_plan.py $ARGS > gpurun_out/tv_$v.txt 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/tv_$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/tv_$v.txt)"
done
