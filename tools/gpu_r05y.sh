#!/bin/bash
# r05 session Y: k_ekf_gain_t with row k + 1 split between waves k and k + 1: A/B of the
# smoothed states against the previous build (bit-identical expected), EKF GPU tests, the
# default-model leg's kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
ACINOSET_HIP_LIB=$PWD/acinoset_amd/libacinoset_hip_old.so timeout -k 10 300 python tools/ekf_gain_ab.py $OUT/ab_old.npz 60 > $OUT/ab_old.log 2>&1 || { echo "old failed"; tail $OUT/ab_old.log; exit 1; }
timeout -k 10 300 python tools/ekf_gain_ab.py $OUT/ab_new.npz 60 > $OUT/ab_new.log 2>&1 || { echo "new failed"; tail $OUT/ab_new.log; exit 1; }
python tools/ekf_gain_ab.py --compare $OUT/ab_old.npz $OUT/ab_new.npz | tee $OUT/ab_cmp_r05y.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_ekf.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ekf_r05y.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_ekf_r05y.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ekfleg_r05y -o run -- python3 tools/time_ekf_leg.py default fd 64 500 > $OUT/ekfleg_r05y.log 2>&1 || { echo "leg failed"; tail $OUT/ekfleg_r05y.log; exit 1; }
tail -n 1 $OUT/ekfleg_r05y.log | cut -c1-300
grep -h "ekf_gain" $OUT/ekfleg_r05y/run_kernel_stats.csv | cut -c1-160
echo done
