#!/bin/bash
# r06q (r06o with the barrier the early trig tables need before the FK items; r06o raced; and
# k_tri_dense undistorting every view once, against libabold.so's tri): k_ekf_filter_w1 with the prediction's covariance passes fused (2 barriers instead of 5, Q
# added by the thread that forms the element), the outputs stored by the update's threads (no
# store phase) and the trig tables' parameter loop unrolled (P known at compile time). EKF /
# libunfused.so (neither fusion, Q read from global memory); libabold.so (before round 6's EKF
# changes); phase profile, bit-identity against libabold.so, EKF tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
ekfbench() {  # tag [lib]
  local envlib=""
  [ -n "${2:-}" ] && envlib="ACINOSET_HIP_LIB=$2"
  env $envlib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --window-frames 0 > $OUT/bench_ekf_$1_r06q.log 2>&1 || { echo "bench $1 rc=$?"; tail -5 $OUT/bench_ekf_$1_r06q.log; exit 1; }
  grep '^{' $OUT/bench_ekf_$1_r06q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['ekf']; p=d['sba_ekf_pipeline']; print('$1', 'ekf', round(e['us_per_frame_per_seq'], 3), 'us/frame; pipeline', round(p['ms_per_step'], 3), 'ms', round(p['frames_per_s']))"
}
ekfbench new_a
ekfbench unfused_a $B/libunfused.so
ekfbench old_a $B/libabold.so
ekfbench new_b
ekfbench unfused_b $B/libunfused.so
ACS_PROF_LIB=$B/libprof.so timeout -k 10 200 python tools/prof_ekf_phases.py head 12 200 fd > $OUT/ekf_phases_head_new_r06q.log 2>&1 || { echo "prof new rc=$?"; exit 1; }
tail -n +2 $OUT/ekf_phases_head_new_r06q.log
ACINOSET_HIP_LIB=$B/libabold.so timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_old_o.npz 250 head > $OUT/ekf_ab_r06q.log 2>&1 || { echo "ab old rc=$?"; exit 1; }
timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_new_o.npz 250 head >> $OUT/ekf_ab_r06q.log 2>&1 || { echo "ab new rc=$?"; exit 1; }
python tools/ekf_gain_ab.py --compare $OUT/ekf_ab_old_o.npz $OUT/ekf_ab_new_o.npz >> $OUT/ekf_ab_r06q.log 2>&1; echo "ab compare rc=$?"; tail -n 4 $OUT/ekf_ab_r06q.log
ACINOSET_HIP_LIB=$B/libabold.so timeout -k 10 200 python tools/tri_ab.py $OUT/tri_ab_old.npz > $OUT/tri_ab_r06q.log 2>&1 || { echo "tri old rc=$?"; exit 1; }
timeout -k 10 200 python tools/tri_ab.py $OUT/tri_ab_new.npz >> $OUT/tri_ab_r06q.log 2>&1 || { echo "tri new rc=$?"; exit 1; }
python tools/tri_ab.py --compare $OUT/tri_ab_old.npz $OUT/tri_ab_new.npz >> $OUT/tri_ab_r06q.log 2>&1; echo "tri compare rc=$?"; tail -n 2 $OUT/tri_ab_r06q.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_ekf.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize_oracle.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_r06q.log 2>&1; tail -n 3 $OUT/pytest_ekf_r06q.log
echo done
