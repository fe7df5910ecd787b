set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ekf.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ekf.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_ekf.log; [ $rc -eq 0 ] || exit $rc
ACINOSET_HIP_LIB=$PWD/acinoset_amd/csrc/build/libprof_ekf.so timeout -k 10 200 python tools/prof_ekf_phases.py > gpurun_out/ekf_phases.log 2>&1 || exit $?
cat gpurun_out/ekf_phases.log
timeout -k 10 200 python tools/time_ekf.py > gpurun_out/time_ekf.log 2>&1 || exit $?
tail -5 gpurun_out/time_ekf.log
