#!/bin/bash
# r05 session B: FTE tests with the deferred pending terms, per-level traces (deferred vs eager), drift survey
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n 4 $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
step pytest_fte_r05b 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step trace10k_def 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_def -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
python tools/fte_iter_sequence.py $OUT/tr10k_def > $OUT/seq10k_def.log 2>&1; tail -n 20 $OUT/seq10k_def.log
export ACS_CR_EAGER=1
step trace10k_eager 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_eager -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
unset ACS_CR_EAGER
python tools/fte_iter_sequence.py $OUT/tr10k_eager > $OUT/seq10k_eager.log 2>&1; tail -n 20 $OUT/seq10k_eager.log
step trace1k 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr1k -o run -- python3 tools/prof_fte.py --frames 1000 --reps 3
python tools/fte_iter_sequence.py $OUT/tr1k > $OUT/seq1k.log 2>&1; tail -n 14 $OUT/seq1k.log
rm -rf $OUT/tr10k_def $OUT/tr10k_eager $OUT/tr1k
step drift_r05b 600 python -u tools/ekf_drift_survey.py 8 250
echo done
