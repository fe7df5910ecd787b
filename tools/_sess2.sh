set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log > gpurun_out/bench_r01f.json
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ftetrace -o run -- python3 tools/prof_fte.py --reps 3 > gpurun_out/ftetrace.log 2>&1 || exit $?
grep rep gpurun_out/ftetrace.log
python tools/fte_iter_breakdown.py gpurun_out/ftetrace 1000 > gpurun_out/fte_breakdown.log; head -30 gpurun_out/fte_breakdown.log
