#!/bin/bash
# r06r: the kept EKF / triangulation tree: EKF and pipeline bench legs (two runs), bit-identity of
# the head filter and the dense triangulation against libabold.so (before round 6's EKF / tri
# changes), EKF / pipeline / drop-in / full-size oracle GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
B=$PWD/acinoset_amd/csrc/build
for t in a b; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --window-frames 0 > $OUT/bench_ekf_${t}_r06r.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_ekf_${t}_r06r.log; exit 1; }
  grep '^{' $OUT/bench_ekf_${t}_r06r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['ekf']; p=d['sba_ekf_pipeline']; print('$t', 'ekf', round(e['us_per_frame_per_seq'], 3), 'us/frame; pipeline', round(p['ms_per_step'], 3), 'ms', round(p['frames_per_s']))"
done
ACINOSET_HIP_LIB=$B/libabold.so timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_old_r.npz 250 head > $OUT/ekf_ab_r06r.log 2>&1 || { echo "ab old rc=$?"; exit 1; }
timeout -k 10 200 python tools/ekf_gain_ab.py $OUT/ekf_ab_new_r.npz 250 head >> $OUT/ekf_ab_r06r.log 2>&1 || { echo "ab new rc=$?"; exit 1; }
python tools/ekf_gain_ab.py --compare $OUT/ekf_ab_old_r.npz $OUT/ekf_ab_new_r.npz >> $OUT/ekf_ab_r06r.log 2>&1; echo "ab compare rc=$?"; tail -n 4 $OUT/ekf_ab_r06r.log
ACINOSET_HIP_LIB=$B/libabold.so timeout -k 10 200 python tools/tri_ab.py $OUT/tri_ab_old_r.npz > $OUT/tri_ab_r06r.log 2>&1 || { echo "tri old rc=$?"; exit 1; }
timeout -k 10 200 python tools/tri_ab.py $OUT/tri_ab_new_r.npz >> $OUT/tri_ab_r06r.log 2>&1 || { echo "tri new rc=$?"; exit 1; }
python tools/tri_ab.py --compare $OUT/tri_ab_old_r.npz $OUT/tri_ab_new_r.npz >> $OUT/tri_ab_r06r.log 2>&1; echo "tri compare rc=$?"; tail -n 2 $OUT/tri_ab_r06r.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_ekf.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize_oracle.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_r06r.log 2>&1; tail -n 3 $OUT/pytest_ekf_r06r.log
echo done
