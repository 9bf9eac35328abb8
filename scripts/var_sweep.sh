set -o pipefail
for v in v0 v1 v2 v3; do
  MSA_LIB_PATH=variants/$v.so timeout -k 10 60 python -u scripts/sweep_m.py 10000 64,2560,10000 > gpurun_out/var_$v.log 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu gpurun_out/var_$v.log
done
