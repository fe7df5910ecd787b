#!/bin/bash
# r05 session G: k_cr_wide (two blocks per CU at the wide levels): 10k FTE parity, traces on/off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-6} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
step pytest_wide_r05g 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_fullsize_oracle.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider -k "fte or cfg3"
for v in on off; do
  if [ $v = off ]; then export ACS_CR_WIDE_MIN=0; else unset ACS_CR_WIDE_MIN; fi
  step tr10k_$v 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_$v -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
  python tools/fte_iter_sequence.py $OUT/tr10k_$v > $OUT/seq10k_wide_$v.log 2>&1; grep -E "level  [0-4] |kernels" $OUT/seq10k_wide_$v.log | head -8
  rm -rf $OUT/tr10k_$v
done
unset ACS_CR_WIDE_MIN
echo done
