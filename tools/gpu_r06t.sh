#!/bin/bash
# r06t: A/B of the head model's smoothed-state recursion with 2 lanes per row (one wave, the
# tree) against 8 lanes per row (libsxg8.so), interleaved EKF / pipeline bench legs, then the
# EKF / pipeline GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
ekfbench() {  # tag [lib]
  local envlib=""
  [ -n "${2:-}" ] && envlib="ACINOSET_HIP_LIB=$2"
  env $envlib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --window-frames 0 > $OUT/bench_ekf_$1_r06t.log 2>&1 || { echo "bench $1 rc=$?"; tail -5 $OUT/bench_ekf_$1_r06t.log; exit 1; }
  grep '^{' $OUT/bench_ekf_$1_r06t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['ekf']; p=d['sba_ekf_pipeline']; print('$1', 'ekf', round(e['us_per_frame_per_seq'], 3), 'us/frame; pipeline', round(p['ms_per_step'], 3), 'ms', round(p['frames_per_s']), e['smoothed_rms_vs_truth_m'])"
}
ekfbench g2_a
ekfbench sxg8_a $B/libsxg8.so
ekfbench g2_b
ekfbench sxg8_b $B/libsxg8.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_ekf.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize_oracle.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_r06t.log 2>&1; tail -n 3 $OUT/pytest_ekf_r06t.log
echo done
