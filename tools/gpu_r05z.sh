#!/bin/bash
# r05 session Z: k_ekf_gain_t with the product's A operand loaded at entry (launch bound 768,
# 144 VGPRs): A/B of the smoothed states against the round's previous build, the default-model
# leg's kernel stats at one and two gains per workgroup, the phase profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${T:-r05z}
ACINOSET_HIP_LIB=$PWD/acinoset_amd/libacinoset_hip_old.so timeout -k 10 300 python tools/ekf_gain_ab.py $OUT/ab_old.npz 60 > $OUT/ab_old.log 2>&1 || { echo "old failed"; tail $OUT/ab_old.log; exit 1; }
timeout -k 10 300 python tools/ekf_gain_ab.py $OUT/ab_new.npz 60 > $OUT/ab_new.log 2>&1 || { echo "new failed"; tail $OUT/ab_new.log; exit 1; }
python tools/ekf_gain_ab.py --compare $OUT/ab_old.npz $OUT/ab_new.npz | tee $OUT/ab_cmp_$T.log
for GP in 1 2; do
  ACS_EKF_GAIN_GP=$GP timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ekfleg_${T}_gp$GP -o run -- python3 tools/time_ekf_leg.py default fd 64 500 > $OUT/ekfleg_${T}_gp$GP.log 2>&1 || { echo "leg failed"; tail $OUT/ekfleg_${T}_gp$GP.log; exit 1; }
  echo "GP=$GP"; grep -h "ekf_gain_t\|ekf_filter<" $OUT/ekfleg_${T}_gp$GP/run_kernel_stats.csv | cut -c1-40,150-260
done
timeout -k 10 300 python tools/prof_ekf_gain.py > $OUT/gainprof_$T.log 2>&1 || { echo "prof failed"; exit 1; }
grep -v amdgpu.ids $OUT/gainprof_$T.log | cut -c1-160
echo done
