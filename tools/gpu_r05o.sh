#!/bin/bash
# r05 session O: k_ekf_gain_t phase times (EKF_PROFILE build), EKF gain tests, default leg times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-6} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
TAILN=3 step pytest_ekf_r05o 600 python -u -m pytest tests/test_gpu_ekf.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "gains or 12cam_float64 or analytic"
ACS_PROF_LIB=$PWD/acinoset_amd/csrc/build/libprof_ekf.so step gainprof 300 python tools/prof_ekf_gain.py 64 500
step ekfdef 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ekfdef -o run -- python3 tools/time_ekf_leg.py default fd
grep -o '"ms_per_call[^,]*, "gpu_ms_per_call[^,]*' $OUT/ekfdef.log
find $OUT/ekfdef -name '*kernel_stats.csv' -exec cp {} $OUT/ekfdef_stats_r05o.csv \; ; grep gain $OUT/ekfdef_stats_r05o.csv | cut -c1-120; rm -rf $OUT/ekfdef

timeout -k 10 120 ./tools/probe/lds_occ_probe > $OUT/lds_occ_probe.log 2>&1; cat $OUT/lds_occ_probe.log
echo done
