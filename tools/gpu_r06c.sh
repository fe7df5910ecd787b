#!/bin/bash
# r06c: upper-tile D (k_cr_assemble_build stores D's upper tiles, levels 0-1 read it so) and the
# mirrored pending Schur terms: FTE / dist / full-size / symmetry tests, then the 10k / 1k
# iteration kernel totals with upper-tile D and with ACS_D_FULL=1 (A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${T:-r06c}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fte_symmetry.py tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize_oracle.py tests/test_fte_reference.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fte_$T.log 2>&1; rc=$?; tail -n 12 $OUT/pytest_fte_$T.log; case $rc in 0|1) ;; *) exit $rc;; esac
for V in up full; do
  for F in 10000 1000; do
    if [ $V = full ]; then export ACS_D_FULL=1; else unset ACS_D_FULL; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ftetrace_$F -o run -- python3 tools/prof_fte.py --frames $F > $OUT/ftetrace_${V}_$F.log 2>&1 || { echo "trace $F failed"; tail -5 $OUT/ftetrace_${V}_$F.log; exit 1; }
    python tools/fte_iter_breakdown.py $OUT/ftetrace_$F $F > $OUT/fte_kernel_totals_${T}_${V}_$F.log 2>&1
    python tools/fte_iter_sequence.py $OUT/ftetrace_$F > $OUT/seq_${T}_${V}_$F.log 2>&1
    echo "$V $F: $(tail -n 1 $OUT/fte_kernel_totals_${T}_${V}_$F.log)"; grep rep $OUT/ftetrace_${V}_$F.log | tail -1
    rm -rf $OUT/ftetrace_$F
  done
done
unset ACS_D_FULL
echo done
