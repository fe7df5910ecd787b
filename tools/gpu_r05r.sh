#!/bin/bash
# r05 session R: k_ekf_gain_t one vs two gains per workgroup (launch bound 1024)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for gp in 1 2; do
  export ACS_EKF_GAIN_GP=$gp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/eg$gp -o run -- python3 tools/time_ekf_leg.py default fd > $OUT/eg$gp.log 2>&1 || { echo fail $gp; exit 1; }
  grep -o '"ms_per_call[^,]*' $OUT/eg$gp.log
  find $OUT/eg$gp -name '*kernel_stats.csv' -exec cp {} $OUT/ekfdef_stats_gp$gp.csv \; ; grep gain_t $OUT/ekfdef_stats_gp$gp.csv | cut -c1-110; rm -rf $OUT/eg$gp
done
unset ACS_EKF_GAIN_GP
timeout -k 10 600 python -u -m pytest tests/test_gpu_ekf.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "gains" > $OUT/pytest_gain_r05r.log 2>&1; tail -2 $OUT/pytest_gain_r05r.log
echo done
