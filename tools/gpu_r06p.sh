#!/bin/bash
# r06p: bisect of r06o's failure (fused prediction vs fused output stores) on the head-model tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
for v in storeonly predonly; do
  ACINOSET_HIP_LIB=$B/lib$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_ekf.py -m gpu -q -x -k "reference_head or float64_matches_oracle" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_${v}_r06p.log 2>&1; echo "$v rc=$?"; tail -n 2 $OUT/pytest_ekf_${v}_r06p.log
done
echo done
