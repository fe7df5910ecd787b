#!/bin/bash
# r06s: A/B of k_ekf_filter_w1's output stores by the update's threads (no store phase;
# libstorefused.so) against the kept tree, interleaved EKF / pipeline bench legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
ekfbench() {  # tag [lib]
  local envlib=""
  [ -n "${2:-}" ] && envlib="ACINOSET_HIP_LIB=$2"
  env $envlib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --window-frames 0 > $OUT/bench_ekf_$1_r06s.log 2>&1 || { echo "bench $1 rc=$?"; tail -5 $OUT/bench_ekf_$1_r06s.log; exit 1; }
  grep '^{' $OUT/bench_ekf_$1_r06s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['ekf']; p=d['sba_ekf_pipeline']; print('$1', 'ekf', round(e['us_per_frame_per_seq'], 3), 'us/frame; pipeline', round(p['ms_per_step'], 3), 'ms', round(p['frames_per_s']), e['smoothed_rms_vs_truth_m'])"
}
ekfbench kept_a
ekfbench storefused_a $B/libstorefused.so
ekfbench kept_b
ekfbench storefused_b $B/libstorefused.so
echo done
