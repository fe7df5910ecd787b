#!/bin/bash
# r06g: same-session A/B of k_cr_level's early next-pivot start in the production build
# (libacinoset_hip.so, CR_EARLY_PIVOT=1) against acinoset_amd/csrc/build/libvar0.so
# (-DCR_EARLY_PIVOT=0, no profiling), interleaved A B A B, kernel traces at 1,000 and 10,000
# frames; then the SBA tests after the status-count fix and the new seed-61 EKF window test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
VAR=$PWD/acinoset_amd/csrc/build/libvar0.so
trace() {  # name frames [lib]
  local d=$OUT/abtrace_$1
  if [ -n "${3:-}" ]; then
    ACINOSET_HIP_LIB=$3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/prof_fte.py --frames $2 > $d.log 2>&1
  else
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/prof_fte.py --frames $2 > $d.log 2>&1
  fi
  local rc=$?; [ $rc -eq 0 ] || { echo "trace $1 rc=$rc"; tail -5 $d.log; exit 1; }
  python tools/fte_iter_breakdown.py $d $2 > $OUT/fte_kernel_totals_$1_r06g.log 2>&1
  echo "$1: $(tail -n 1 $OUT/fte_kernel_totals_$1_r06g.log)"
  rm -rf $d
}
trace early_1k_a 1000
trace barrier_1k_a 1000 $VAR
trace early_1k_b 1000
trace barrier_1k_b 1000 $VAR
trace early_10k 10000
trace barrier_10k 10000 $VAR
timeout -k 10 600 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_fullsize.py "tests/test_gpu_ekf.py::test_ekf_12cam_default_seed61_window_matches_oracle" -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sba_r06g.log 2>&1; rc=$?; tail -n 5 $OUT/pytest_sba_r06g.log
echo done rc=$rc
