#!/bin/bash
# r05 session C: k_cr_level timelines of the wide levels (10k frames), default-model EKF per frame
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n 30 $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
ACS_PROF_LIB=$PWD/acinoset_amd/csrc/build/libprof_w0.so step tl_L0_10k 300 python -u tools/prof_cr_timeline.py 10000
ACS_PROF_LIB=$PWD/acinoset_amd/csrc/build/libprof_w3.so step tl_L3_10k 300 python -u tools/prof_cr_timeline.py 10000
ACS_PROF_LIB=$PWD/acinoset_amd/csrc/build/libprof.so step tl_deep_1k 300 python -u tools/prof_cr_timeline.py 1000
step ekf_default_frames 300 python -u tools/ekf_default_frames.py 30
echo done
