#!/bin/bash
# r05 session A: GPU suite, whole-clip EKF drift survey, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n 4 $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
step pytest_gpu_r05a 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step drift_r05a 600 python -u tools/ekf_drift_survey.py 8 250
step bench_r05a 600 python -u bench.py
grep '^{' $OUT/bench_r05a.log > $OUT/bench_r05a.json || true
echo done
