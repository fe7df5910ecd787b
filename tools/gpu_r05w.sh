#!/bin/bash
# r05 session W: the final tree: GPU suite, smoke, bench, kernel stats, FTE 10k / 1k iteration
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05w STEPS=test,smoke,bench,prof bash tools/gpu_session.sh || exit $?
OUT=$PWD/gpurun_out; export TMPDIR=/tmp
for F in 1000 10000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ftetrace_$F -o run -- python3 tools/prof_fte.py --frames $F > $OUT/ftetrace$F.log 2>&1 || { echo "trace $F failed"; exit 1; }
  python tools/fte_iter_sequence.py $OUT/ftetrace_$F > $OUT/seq_r05w_$F.log 2>&1; grep -E "k_fte_lm|kernels" $OUT/seq_r05w_$F.log | head -2
  python tools/fte_iter_breakdown.py $OUT/ftetrace_$F $F > $OUT/fte_kernel_totals_r05w_$F.log 2>&1
  rm -rf $OUT/ftetrace_$F
done
echo done
