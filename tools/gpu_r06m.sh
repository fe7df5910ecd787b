#!/bin/bash
# r06m: k_ekf_filter_w1 with the one-joint FK plan (EKF_PLAN_D 2, the trig table kept) and Q /
# the measurement rows kept off the frame chain (EKF_W1_PREFETCH): EKF and pipeline bench legs
# of the three builds interleaved (libacinoset_hip.so; libnopf.so = EKF_W1_PREFETCH 0;
# libabold.so = before the plan), phase profiles, bit-identity against libabold.so, EKF tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
ekfbench() {  # tag [lib]
  local envlib=""
  [ -n "${2:-}" ] && envlib="ACINOSET_HIP_LIB=$2"
  env $envlib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --window-frames 0 > $OUT/bench_ekf_$1_r06m.log 2>&1 || { echo "bench $1 rc=$?"; tail -5 $OUT/bench_ekf_$1_r06m.log; exit 1; }
  grep '^{' $OUT/bench_ekf_$1_r06m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['ekf']; p=d['sba_ekf_pipeline']; print('$1', 'ekf', round(e['us_per_frame_per_seq'], 3), 'us/frame; pipeline', round(p['ms_per_step'], 3), 'ms', round(p['frames_per_s']))"
}
ekfbench new_a
ekfbench nopf_a $B/libnopf.so
ekfbench old_a $B/libabold.so
ekfbench new_b
ekfbench nopf_b $B/libnopf.so
ekfbench old_b $B/libabold.so
ACS_PROF_LIB=$B/libprof_old.so timeout -k 10 200 python tools/prof_ekf_phases.py head 12 200 fd > $OUT/ekf_phases_head_old_r06m.log 2>&1 || { echo "prof old rc=$?"; exit 1; }
ACS_PROF_LIB=$B/libprof.so timeout -k 10 200 python tools/prof_ekf_phases.py head 12 200 fd > $OUT/ekf_phases_head_new_r06m.log 2>&1 || { echo "prof new rc=$?"; exit 1; }
paste $OUT/ekf_phases_head_old_r06m.log $OUT/ekf_phases_head_new_r06m.log | tail -n +2 | cut -c1-160
ACINOSET_HIP_LIB=$B/libabold.so timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_old_m.npz 250 head > $OUT/ekf_ab_r06m.log 2>&1 || { echo "ab old rc=$?"; exit 1; }
timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_new_m.npz 250 head >> $OUT/ekf_ab_r06m.log 2>&1 || { echo "ab new rc=$?"; exit 1; }
python tools/ekf_gain_ab.py --compare $OUT/ekf_ab_old_m.npz $OUT/ekf_ab_new_m.npz >> $OUT/ekf_ab_r06m.log 2>&1; echo "ab compare rc=$?"; tail -n 4 $OUT/ekf_ab_r06m.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ekf.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize_oracle.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_r06m.log 2>&1; tail -n 3 $OUT/pytest_ekf_r06m.log
echo done
