#!/bin/bash
# r06i: k_sba_lm with one shared logarithm per lane over its slots (S > 1): SBA GPU tests and the
# SBA bench legs (headline instance unchanged, configs[4]-shape instance 2,182 -> 2,002 static
# instructions)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_edge.py tests/test_gpu_pipeline.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sba_r06i.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_sba_r06i.log; case $rc in 0|1) ;; *) exit $rc;; esac
for t in a b; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --ekf-seqs 0 --pipeline-seqs 0 --window-frames 0 > $OUT/bench_sba_${t}_r06i.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_sba_${t}_r06i.log; exit 1; }
  grep '^{' $OUT/bench_sba_${t}_r06i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['sba_at_scale']; print('$t', 'headline', round(d['value']), round(d['roofline']['kernel_ms']*1e3, 3), 'us; scale', round(s['ms_per_step'], 4), round(s['roofline']['kernel_ms'], 4), 'ms', s['gn_steps_mean'], s['status'], s['pos_rms_vs_truth_m'])"
done
echo done
