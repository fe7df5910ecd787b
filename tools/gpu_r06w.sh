#!/bin/bash
# r06w: k_fte_linearize with its frames walked by resident workgroups (table and cameras staged
# once per workgroup, the pose stencil in LDS) against the round-6 tree (libbase.so) and against
# one workgroup per frame of the new kernel (ACS_LIN_PER_FRAME=1); kernel traces at 1,000 and
# 10,000 frames, interleaved; then the FTE GPU tests on the new library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
BASE=$PWD/acinoset_amd/csrc/build/libbase.so
TAG=${TAG:-r06w}
trace() {  # name frames [lib] [per_frame]
  local d=$OUT/abtrace_$1
  local lib=${3:-}
  env ${lib:+ACINOSET_HIP_LIB=$lib} ACS_LIN_PER_FRAME=${4:-0} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/prof_fte.py --frames $2 > $d.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "trace $1 rc=$rc"; tail -5 $d.log; exit 1; }
  python tools/fte_iter_breakdown.py $d $2 > $OUT/fte_kernel_totals_$1_$TAG.log 2>&1
  echo "$1: $(grep -m1 k_fte_linearize $OUT/fte_kernel_totals_$1_$TAG.log) | $(tail -n 1 $OUT/fte_kernel_totals_$1_$TAG.log)"
  rm -rf $d
}
trace base_1k_a 1000 $BASE
trace loop_1k_a 1000
trace base_10k_a 10000 $BASE
trace loop_10k_a 10000
trace perframe_10k_a 10000 "" 1
trace base_10k_b 10000 $BASE
trace loop_10k_b 10000
trace perframe_10k_b 10000 "" 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_fte_symmetry.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fte_$TAG.log 2>&1; rc=$?; tail -n 5 $OUT/pytest_fte_$TAG.log
echo done rc=$rc
