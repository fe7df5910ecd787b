#!/bin/bash
# r06a: the new round-6 GPU tests, then the whole GPU suite, then the two-rank bench rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ekf.py::test_ekf_head_indefinite_fallbacks_match_oracle \
  tests/test_gpu_ekf.py::test_ekf_singular_count_after_device_call \
  tests/test_gpu_dist.py::test_fte_dist_reset_reuses_handles_without_allocation \
  tests/test_gpu_dist.py::test_fte_dist_chain_back_launch_equals_per_level_launches \
  > gpurun_out/pytest_new_r06a.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -n 15 gpurun_out/pytest_new_r06a.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_r06a.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -n 8 gpurun_out/pytest_gpu_r06a.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/rehearse_dist.sh
