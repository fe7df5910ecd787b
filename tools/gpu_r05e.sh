#!/bin/bash
# r05 session E: EKF whole-clip / default-model tests, FTE + CR tests with own-all copies (eager)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-6} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
TAILN=30 step pytest_ekf_r05e 900 python -u -m pytest tests/test_gpu_ekf.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_pipeline.py -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider
step pytest_fte_r05e 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
echo done
