#!/bin/bash
# r06zd: k_sba_lm's prologue loads in one wait (unconditional clamped loads, every loaded value
# touched before the early exits) against libbase.so (the committed tree): the SBA bench legs
# interleaved A B A B A B, the bitwise check of both SBA problems, then the SBA GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
BASE=$PWD/acinoset_amd/csrc/build/libbase.so
sbabench() {  # tag [lib]
  local lib=${2:-}
  env ${lib:+ACINOSET_HIP_LIB=$lib} timeout -k 10 300 python bench.py --no-cpu-baseline --no-fte --ekf-seqs 0 --pipeline-seqs 0 --window-frames 0 > $OUT/bench_sba_$1_r06zd.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench_sba_$1_r06zd.log; exit 1; }
  grep '^{' $OUT/bench_sba_$1_r06zd.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['sba_at_scale']; print('$1', 'headline', round(d['value']), round(d['ms_per_step']*1e3, 3), 'us/step', round(d['roofline']['kernel_ms']*1e3, 3), 'us kernel; stream', round(d['stream_launch']['kernel_ms']*1e3, 3), 'us; scale', round(s['ms_per_step'], 4), 'ms')"
}
for t in a b c; do
  sbabench base_$t $BASE
  sbabench new_$t
done
timeout -k 10 300 env ACINOSET_HIP_LIB=$BASE python tools/sba_bitcheck.py head > $OUT/sba_bits_base_r06zd.log 2>&1 || { echo "bits base failed"; exit 1; }
timeout -k 10 300 python tools/sba_bitcheck.py new > $OUT/sba_bits_new_r06zd.log 2>&1 || { echo "bits new failed"; exit 1; }
tail -3 $OUT/sba_bits_new_r06zd.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_fullsize.py tests/test_gpu_edge.py tests/test_gpu_pipeline.py tests/test_gpu_dropin.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sba_r06zd.log 2>&1; rc=$?; tail -n 3 $OUT/pytest_sba_r06zd.log
echo done rc=$rc
