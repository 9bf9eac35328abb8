# walk breakdown (diagnostic build vlib/libmsa_tbstats.so) for the C5, ref 10k and whole-pair walks
set -o pipefail
mkdir -p gpurun_out
for w in c5 ref refwhole; do
  MSA_LIB_PATH=vlib/libmsa_tbstats.so timeout -k 10 180 python -u scripts/tb_stats.py --workload $w > gpurun_out/tbs_$w.txt 2>&1 || { echo "tb_stats $w failed"; tail -5 gpurun_out/tbs_$w.txt; exit 1; }
  tail -1 gpurun_out/tbs_$w.txt
done
