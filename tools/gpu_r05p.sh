#!/bin/bash
# r05 session P: k_ekf_gain_t workgroups in flight (EKF_PROFILE build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-8} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
ACS_PROF_LIB=$PWD/acinoset_amd/csrc/build/libprof_ekf.so step gainprof_p 300 python tools/prof_ekf_gain.py 64 500
echo done
