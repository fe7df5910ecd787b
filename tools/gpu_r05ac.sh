#!/bin/bash
# r05 session AC: the 16-camera FTE fix as a k_cr_level<NB, true> instance (GR = 32 only): FTE + dist tests, the 10k / 1k iteration sequences
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${T:-r05ac}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fte_$T.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_fte_$T.log; [ $rc -eq 0 ] || exit $rc
for F in 10000 1000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ftetrace_$F -o run -- python3 tools/prof_fte.py --frames $F > $OUT/ftetrace$F.log 2>&1 || { echo "trace $F failed"; tail -5 $OUT/ftetrace$F.log; exit 1; }
  python tools/fte_iter_sequence.py $OUT/ftetrace_$F > $OUT/seq_${T}_$F.log 2>&1; grep -E "k_fte_linearize|kernels" $OUT/seq_${T}_$F.log | head -3
  python tools/fte_iter_breakdown.py $OUT/ftetrace_$F $F > $OUT/fte_kernel_totals_${T}_$F.log 2>&1
  rm -rf $OUT/ftetrace_$F
done
echo done
