#!/bin/bash
# r06b: the fixed EKF fallback test, rank-round timing (k_cr_back_chain vs per-level back
# launches), the bench and its rocprofv3 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  case $rc in 0|1) return 0;; *) echo "fatal $rc"; exit $rc;; esac
}
step pytest_ekf_r06b 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ekf.py -k "indefinite or singular"
step time_dist_r06b 600 python -u tools/time_dist.py 10000 --worlds 1,8
ACS_DIST_BACK_LEVELS=1 step time_dist_levels_r06b 600 python -u tools/time_dist.py 10000 --worlds 8
step bench_r06b 600 python -u bench.py
grep '^{' gpurun_out/bench_r06b.log > gpurun_out/bench_r06b.json || true
export TMPDIR=/tmp
step rocprof_r06b 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06b -o run -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 20
echo done
