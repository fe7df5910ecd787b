#!/bin/bash
# r05 session N: EKF suite with the explicit-inverse tiled gains; default leg kernel times;
# FTE tests with the tau partials in the top CR launch; k_cr_back_all late W loads for the
# coarse levels (ACS_BACK_LATE_LV) A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-4} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
TAILN=12 step pytest_ekf_r05n 900 python -u -m pytest tests/test_gpu_ekf.py tests/test_gpu_pipeline.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step ekfdef 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ekfdef -o run -- python3 tools/time_ekf_leg.py default fd
grep -o '"ms_per_call[^,]*, "gpu_ms_per_call[^,]*' $OUT/ekfdef.log
find $OUT/ekfdef -name '*kernel_stats.csv' -exec cp {} $OUT/ekfdef_stats_r05n.csv \; ; head -6 $OUT/ekfdef_stats_r05n.csv | cut -c1-120; rm -rf $OUT/ekfdef
step pytest_fte_r05n 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for lv in 30; do
  export ACS_BACK_LATE_LV=$lv
  step tr10k_late$lv 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_late$lv -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
  python tools/fte_iter_sequence.py $OUT/tr10k_late$lv > $OUT/seq10k_late$lv.log 2>&1; grep -E "back_all|k_cr_level.*grid +1 |kernels" $OUT/seq10k_late$lv.log | head -4
  rm -rf $OUT/tr10k_late$lv
  TAILN=18 step backtr10k_late$lv 300 python tools/prof_back_all.py 10000
done
unset ACS_BACK_LATE_LV
echo done
