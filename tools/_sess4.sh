set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_dist.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fte.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fte.log; true
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ftetrace10k -o run -- python3 tools/prof_fte.py --reps 2 --frames 10000 > gpurun_out/ftetrace10k.log 2>&1 || exit $?
grep rep gpurun_out/ftetrace10k.log
python tools/fte_iter_breakdown.py gpurun_out/ftetrace10k 10000 > gpurun_out/fte_breakdown10k.log; head -8 gpurun_out/fte_breakdown10k.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ftetrace -o run -- python3 tools/prof_fte.py --reps 3 > gpurun_out/ftetrace.log 2>&1 || exit $?
grep rep gpurun_out/ftetrace.log
python tools/fte_iter_breakdown.py gpurun_out/ftetrace 1000 > gpurun_out/fte_breakdown.log; head -4 gpurun_out/fte_breakdown.log
timeout -k 10 120 python tools/prof_lin_phases.py 1000 > gpurun_out/lin_phases.log 2>&1; cat gpurun_out/lin_phases.log
