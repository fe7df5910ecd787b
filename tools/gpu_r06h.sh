#!/bin/bash
# r06h: k_sba_lm occupancy A/B (SBA_WPE = 1 in libacinoset_hip.so, i.e. unconstrained: 186 VGPRs,
# 2 waves per SIMD for <4,3>; libsba{2,3,4}.so: the register budget of 2 / 3 / 4 waves per SIMD)
# on the SBA bench legs, and the SBA GPU tests with the hoisted camera records loaded from
# global memory (no LDS stage / barrier in the headline instance)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
timeout -k 10 300 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sba_r06h.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_sba_r06h.log; case $rc in 0|1) ;; *) exit $rc;; esac
sbabench() {  # tag [lib]
  if [ -n "${2:-}" ]; then
    ACINOSET_HIP_LIB=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --ekf-seqs 0 --pipeline-seqs 0 --window-frames 0 > $OUT/bench_sba_$1_r06h.log 2>&1
  else
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --ekf-seqs 0 --pipeline-seqs 0 --window-frames 0 > $OUT/bench_sba_$1_r06h.log 2>&1
  fi
  local rc=$?; [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -5 $OUT/bench_sba_$1_r06h.log; exit 1; }
  grep '^{' $OUT/bench_sba_$1_r06h.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['sba_at_scale']; print('$1', 'headline', round(d['value']), round(d['roofline']['kernel_ms']*1e3, 3), 'us; scale', round(s['ms_per_step'], 4), round(s['roofline']['kernel_ms'], 4), 'ms')"
}
sbabench w1a
sbabench w2 $B/libsba2.so
sbabench w3 $B/libsba3.so
sbabench w4 $B/libsba4.so
sbabench w1b
echo done
