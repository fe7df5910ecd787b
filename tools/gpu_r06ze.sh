#!/bin/bash
# r06ze: assemble_row with its loads in two round trips per wave (batch loads touched before use, the
# special loads regrouped one branch per wave, unconditional) against libbase.so (the committed
# tree): kernel traces at 1,000 and 10,000 frames, bitwise check, FTE GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
BD=$PWD/acinoset_amd/csrc/build
TAG=${TAG:-r06ze}
trace() {  # name frames [lib]
  local d=$OUT/abtrace_$1
  local lib=${3:-}
  env ${lib:+ACINOSET_HIP_LIB=$lib} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/prof_fte.py --frames $2 > $d.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "trace $1 rc=$rc"; tail -5 $d.log; exit 1; }
  python tools/fte_iter_breakdown.py $d $2 > $OUT/fte_kernel_totals_$1_$TAG.log 2>&1
  echo "$1: $(grep -m1 k_cr_assemble_build $OUT/fte_kernel_totals_$1_$TAG.log) | $(tail -n 1 $OUT/fte_kernel_totals_$1_$TAG.log)"
  rm -rf $d
}
for r in a b; do
  trace base_1k_$r 1000 $BD/libbase.so
  trace asm4_1k_$r 1000
done
for r in a b; do
  trace base_10k_$r 10000 $BD/libbase.so
  trace asm4_10k_$r 10000
done
timeout -k 10 240 env ACINOSET_HIP_LIB=$BD/libbase.so python tools/ab_fte_bits.py save base > $OUT/bits_base_$TAG.log 2>&1 || { echo "bits base failed"; exit 1; }
timeout -k 10 240 python tools/ab_fte_bits.py save asm4 > $OUT/bits_asm4_$TAG.log 2>&1 || { echo "bits asm4 failed"; exit 1; }
python tools/ab_fte_bits.py cmp base asm4 | tee $OUT/fte_bits_asm4_vs_base_$TAG.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_fte_symmetry.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fte_$TAG.log 2>&1; rc=$?; tail -n 5 $OUT/pytest_fte_$TAG.log
echo done rc=$rc
