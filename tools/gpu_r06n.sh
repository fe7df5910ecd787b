#!/bin/bash
# r06n: k_ekf_filter_w1 with the one-joint FK's trig tables formed inside the prediction by idle
# threads (EKF_W1_TRIG_EARLY): EKF and pipeline bench legs of the three builds interleaved
# (libacinoset_hip.so; libnoearly.so = EKF_W1_TRIG_EARLY 0; libabold.so = before round 6's EKF
# changes), phase profile (old: libprof_old.so is gone, the profiling build of this tree only),
# bit-identity against libabold.so, EKF tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
ekfbench() {  # tag [lib]
  local envlib=""
  [ -n "${2:-}" ] && envlib="ACINOSET_HIP_LIB=$2"
  env $envlib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --window-frames 0 > $OUT/bench_ekf_$1_r06n.log 2>&1 || { echo "bench $1 rc=$?"; tail -5 $OUT/bench_ekf_$1_r06n.log; exit 1; }
  grep '^{' $OUT/bench_ekf_$1_r06n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['ekf']; p=d['sba_ekf_pipeline']; print('$1', 'ekf', round(e['us_per_frame_per_seq'], 3), 'us/frame; pipeline', round(p['ms_per_step'], 3), 'ms', round(p['frames_per_s']))"
}
ekfbench new_a
ekfbench noearly_a $B/libnoearly.so
ekfbench old_a $B/libabold.so
ekfbench new_b
ekfbench noearly_b $B/libnoearly.so
ekfbench old_b $B/libabold.so
ACS_PROF_LIB=$B/libprof.so timeout -k 10 200 python tools/prof_ekf_phases.py head 12 200 fd > $OUT/ekf_phases_head_new_r06n.log 2>&1 || { echo "prof new rc=$?"; exit 1; }
tail -n +2 $OUT/ekf_phases_head_new_r06n.log
ACINOSET_HIP_LIB=$B/libabold.so timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_old_m.npz 250 head > $OUT/ekf_ab_r06n.log 2>&1 || { echo "ab old rc=$?"; exit 1; }
timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_new_m.npz 250 head >> $OUT/ekf_ab_r06n.log 2>&1 || { echo "ab new rc=$?"; exit 1; }
python tools/ekf_gain_ab.py --compare $OUT/ekf_ab_old_m.npz $OUT/ekf_ab_new_m.npz >> $OUT/ekf_ab_r06n.log 2>&1; echo "ab compare rc=$?"; tail -n 4 $OUT/ekf_ab_r06n.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ekf.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize_oracle.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_r06n.log 2>&1; tail -n 3 $OUT/pytest_ekf_r06n.log
echo done
