#!/bin/bash
# r05 session M: EKF default tests (ring seed 62, tiled gains), default leg kernel times; FTE tests;
# 10k / 1k traces and the back-substitution timeline (k_cr_back_all<NB, GRB>, 16 loads in flight
# in the tau partials)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-4} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
TAILN=8 step pytest_ekf_r05m 600 python -u -m pytest tests/test_gpu_ekf.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "gains or default"
step ekfdef 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ekfdef -o run -- python3 tools/time_ekf_leg.py default fd
grep -o '"ms_per_call[^,]*, "gpu_ms_per_call[^,]*' $OUT/ekfdef.log
find $OUT/ekfdef -name '*kernel_stats.csv' -exec cp {} $OUT/ekfdef_stats.csv \; ; head -8 $OUT/ekfdef_stats.csv | cut -c1-120; rm -rf $OUT/ekfdef
step pytest_fte_r05m 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_fullsize.py -k "fte or FTE or cfg" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step tr10k 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
python tools/fte_iter_sequence.py $OUT/tr10k > $OUT/seq10k_r05m.log 2>&1; grep -E "assemble|back_all|linearize|kernels" $OUT/seq10k_r05m.log | head -5
step tr1k 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr1k -o run -- python3 tools/prof_fte.py --frames 1000 --reps 3
python tools/fte_iter_sequence.py $OUT/tr1k > $OUT/seq1k_r05m.log 2>&1; grep -E "assemble|back_all|linearize|kernels" $OUT/seq1k_r05m.log | head -5
rm -rf $OUT/tr10k $OUT/tr1k
TAILN=20 step backtr10k_r05m 300 python tools/prof_back_all.py 10000
echo done
