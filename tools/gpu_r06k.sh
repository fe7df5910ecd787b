#!/bin/bash
# r06l: the one-joint FK plan with per-item sines / cosines and translation (no trig table or barrier):
# table walk per frame: phase profile before / after (libprof_old.so / libprof.so, the FK/proj
# phase split into the trig tables and the items), bit-identity A/B of the head filter against
# the previous build (libabold.so), EKF tests, the EKF and pipeline bench legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
ACS_PROF_LIB=$B/libprof_old.so timeout -k 10 200 python tools/prof_ekf_phases.py head 12 200 fd > $OUT/ekf_phases_head_old_r06k.log 2>&1 || { echo "prof old rc=$?"; tail -5 $OUT/ekf_phases_head_old_r06k.log; exit 1; }
ACS_PROF_LIB=$B/libprof.so timeout -k 10 200 python tools/prof_ekf_phases.py head 12 200 fd > $OUT/ekf_phases_head_plan_r06k.log 2>&1 || { echo "prof plan rc=$?"; tail -5 $OUT/ekf_phases_head_plan_r06k.log; exit 1; }
paste $OUT/ekf_phases_head_old_r06k.log $OUT/ekf_phases_head_plan_r06k.log | cut -c1-160
ACINOSET_HIP_LIB=$B/libabold.so timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_old.npz 250 head > $OUT/ekf_ab_r06k.log 2>&1 || { echo "ab old rc=$?"; tail -5 $OUT/ekf_ab_r06k.log; exit 1; }
timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_new.npz 250 head >> $OUT/ekf_ab_r06k.log 2>&1 || { echo "ab new rc=$?"; tail -5 $OUT/ekf_ab_r06k.log; exit 1; }
python tools/ekf_gain_ab.py --compare $OUT/ekf_ab_old.npz $OUT/ekf_ab_new.npz >> $OUT/ekf_ab_r06k.log 2>&1; echo "ab compare rc=$?"; tail -n 4 $OUT/ekf_ab_r06k.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ekf.py tests/test_gpu_pipeline.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_r06k.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_ekf_r06k.log; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --window-frames 0 > $OUT/bench_ekf_r06k.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_ekf_r06k.log; exit 1; }
grep '^{' $OUT/bench_ekf_r06k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['ekf']; p=d['sba_ekf_pipeline']; print('ekf', round(e['us_per_frame_per_seq'], 3), 'us/frame', round(e['frames_per_s']), 'pipeline', round(p['ms_per_step'], 3), 'ms', round(p['frames_per_s']))"
echo done
