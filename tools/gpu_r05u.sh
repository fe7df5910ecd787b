#!/bin/bash
# r05 session U/V: k_fte_linearize changes (U: coalesced transposed Hloc stores, not kept; V: the
# single-chunk observation phase without the hoisted-constant spills; X: D stored as upper tiles):
# FTE tests, 10k / 1k
# iteration sequence, FTE 10k HBM traffic (PMC, calibrated)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=r05x
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-3} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
step pytest_fte_${TAG} 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py tests/test_fte_reference.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for F in 1000 10000; do
  step ftetrace$F 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ftetrace_$F -o run -- python3 tools/prof_fte.py --frames $F
  python tools/fte_iter_breakdown.py $OUT/ftetrace_$F $F > $OUT/fte_breakdown_${TAG}_$F.log 2>&1; tail -1 $OUT/fte_breakdown_${TAG}_$F.log
  python tools/fte_iter_sequence.py $OUT/ftetrace_$F > $OUT/seq_${TAG}_$F.log 2>&1; grep -E "linearize|kernels" $OUT/seq_${TAG}_$F.log | head -2
  rm -rf $OUT/ftetrace_$F
done
step ftepmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ftepmc_${TAG}_fetch -o run -- python3 tools/prof_fte.py --frames 10000 --reps 1
step ftepmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/ftepmc_${TAG}_write -o run -- python3 tools/prof_fte.py --frames 10000 --reps 1
python tools/pmc_summary.py $OUT/ftepmc_${TAG} $OUT/traffic_fte10k_${TAG}.json > $OUT/ftepmc_summary_${TAG}.log 2>&1
rm -rf $OUT/ftepmc_${TAG}_fetch $OUT/ftepmc_${TAG}_write
echo done
