set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ftetrace -o run -- python3 tools/prof_fte.py > gpurun_out/ftetrace.log 2>&1 || exit $?
python tools/fte_trace_summary.py gpurun_out/ftetrace > gpurun_out/ftetrace_summary.txt 2>&1; head -30 gpurun_out/ftetrace_summary.txt; grep rep gpurun_out/ftetrace.log
