# walk breakdown for the diagnostic builds named in $VARS (vlib/libmsa_<name>.so), workloads $WLS
set -o pipefail
mkdir -p gpurun_out
for v in $VARS; do for w in ${WLS:-c5 ref refwhole}; do
  MSA_LIB_PATH=vlib/libmsa_$v.so timeout -k 10 180 python -u scripts/tb_stats.py --workload $w > gpurun_out/tbv_${v}_$w.txt 2>&1 || { echo "tb_stats $v $w failed"; tail -5 gpurun_out/tbv_${v}_$w.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/tbv_${v}_$w.txt | cut -c 1-400)"
done; done
