#!/bin/bash
# r06e: k_cr_level deep-level timeline with and without the early next-pivot start
# (-DCR_EARLY_PIVOT=0: libprof0.so), and the SBA kernel with the folded Jacobian / shared weight
# reciprocal / forced v_fma_f64 Horner steps: SBA parity tests + bench legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python tools/prof_cr_timeline.py 1000 > $OUT/cr_timeline_early_r06e.log 2>&1; echo "early rc=$?"; tail -n 22 $OUT/cr_timeline_early_r06e.log
ACS_PROF_LIB=$PWD/acinoset_amd/csrc/build/libprof0.so timeout -k 10 300 python tools/prof_cr_timeline.py 1000 > $OUT/cr_timeline_barrier_r06e.log 2>&1; echo "barrier rc=$?"; tail -n 22 $OUT/cr_timeline_barrier_r06e.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sba_r06e.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_sba_r06e.log; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --ekf-seqs 0 --pipeline-seqs 0 --window-frames 0 > $OUT/bench_sba_r06e.log 2>&1; echo "bench rc=$?"
grep '^{' $OUT/bench_sba_r06e.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline', d['value'], d['roofline']['kernel_ms'], 'scale', d['sba_at_scale']['ms_per_step'], d['sba_at_scale']['roofline']['kernel_ms'], d['convergence']['iters_max'], d['pos_vs_ref_m'])"
echo done
