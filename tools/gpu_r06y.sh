#!/bin/bash
# r06y: k_cr_assemble_build with 512 threads and compact LDS rows (four blocks per CU) against
# libbase.so (the round-6 tree before the assembly changes) and libv7.so (the same kernel with
# a 7-entry load batch: one round, 12 spilled VGPRs); kernel traces at 1,000 and 10,000 frames,
# bitwise solve check against the base, then the FTE GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
BD=$PWD/acinoset_amd/csrc/build
TAG=${TAG:-r06y}
trace() {  # name frames [lib]
  local d=$OUT/abtrace_$1
  local lib=${3:-}
  env ${lib:+ACINOSET_HIP_LIB=$lib} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/prof_fte.py --frames $2 > $d.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "trace $1 rc=$rc"; tail -5 $d.log; exit 1; }
  python tools/fte_iter_breakdown.py $d $2 > $OUT/fte_kernel_totals_$1_$TAG.log 2>&1
  echo "$1: $(grep -m1 k_cr_assemble_build $OUT/fte_kernel_totals_$1_$TAG.log) | $(tail -n 1 $OUT/fte_kernel_totals_$1_$TAG.log)"
  rm -rf $d
}
trace base_1k_a 1000 $BD/libbase.so
trace asm2_1k_a 1000
trace v7_1k_a 1000 $BD/libv7.so
trace base_10k_a 10000 $BD/libbase.so
trace asm2_10k_a 10000
trace v7_10k_a 10000 $BD/libv7.so
trace base_10k_b 10000 $BD/libbase.so
trace asm2_10k_b 10000
trace v7_10k_b 10000 $BD/libv7.so
timeout -k 10 240 env ACINOSET_HIP_LIB=$BD/libbase.so python tools/ab_fte_bits.py save base > $OUT/bits_base_$TAG.log 2>&1 || { echo "bits base failed"; exit 1; }
timeout -k 10 240 python tools/ab_fte_bits.py save asm2 > $OUT/bits_asm2_$TAG.log 2>&1 || { echo "bits asm2 failed"; exit 1; }
python tools/ab_fte_bits.py cmp base asm2 | tee $OUT/fte_bits_asm2_vs_base_$TAG.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_fte_symmetry.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fte_$TAG.log 2>&1; rc=$?; tail -n 5 $OUT/pytest_fte_$TAG.log
echo done rc=$rc
