#!/bin/bash
# r05 session D: own-all column copies + pivot priority: FTE tests, timelines, per-level traces A/B (PIVPRIO 2 vs 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
B=$PWD/acinoset_amd/csrc/build
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-4} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
step pytest_fte_r05d 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
TAILN=24 ACS_PROF_LIB=$B/libprof_w0.so step tl_L0_prio 300 python -u tools/prof_cr_timeline.py 10000
TAILN=24 ACS_PROF_LIB=$B/libprof_w0np.so step tl_L0_noprio 300 python -u tools/prof_cr_timeline.py 10000
TAILN=24 ACS_PROF_LIB=$B/libprof.so step tl_deep_prio 300 python -u tools/prof_cr_timeline.py 1000
for v in main np; do
  if [ $v = main ]; then unset ACINOSET_HIP_LIB; else export ACINOSET_HIP_LIB=$B/libvar_np.so; fi
  step tr10k_$v 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_$v -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
  python tools/fte_iter_sequence.py $OUT/tr10k_$v > $OUT/seq10k_$v.log 2>&1; tail -n 15 $OUT/seq10k_$v.log
  step tr1k_$v 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr1k_$v -o run -- python3 tools/prof_fte.py --frames 1000 --reps 3
  python tools/fte_iter_sequence.py $OUT/tr1k_$v > $OUT/seq1k_$v.log 2>&1; grep -E "kernels|level" $OUT/seq1k_$v.log | tail -n 12
  rm -rf $OUT/tr10k_$v $OUT/tr1k_$v
done
unset ACINOSET_HIP_LIB
echo done
