#!/bin/bash
# r05 session K: merged-body k_cr_wide (38 spills): 10k parity + trace on/off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-3} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
export ACS_CR_WIDE_MIN=256
step pytest_wide_r05k 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k fte
step tr10k_wide 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_wide -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
python tools/fte_iter_sequence.py $OUT/tr10k_wide > $OUT/seq10k_wide2.log 2>&1; head -6 $OUT/seq10k_wide2.log; grep kernels $OUT/seq10k_wide2.log
rm -rf $OUT/tr10k_wide
echo done
