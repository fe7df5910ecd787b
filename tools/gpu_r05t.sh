#!/bin/bash
# r05 session T: FTE iteration breakdowns (1,000 / 10,000 frames), FTE 10k HBM traffic (PMC,
# calibrated), bench-kernel PMC traffic / FP64 counts, frame-window rank rounds (1 and 8 ranks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=r05t
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-3} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
for F in 1000 10000; do
  step ftetrace$F 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ftetrace_$F -o run -- python3 tools/prof_fte.py --frames $F
  python tools/fte_iter_breakdown.py $OUT/ftetrace_$F $F > $OUT/fte_breakdown_${TAG}_$F.log 2>&1; tail -3 $OUT/fte_breakdown_${TAG}_$F.log
  python tools/fte_iter_sequence.py $OUT/ftetrace_$F > $OUT/seq_${TAG}_$F.log 2>&1; grep kernels $OUT/seq_${TAG}_$F.log
  rm -rf $OUT/ftetrace_$F
done
step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib_${TAG}_fetch -o run -- ./tools/probe/fetch_calib
step ftepmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ftepmc_${TAG}_fetch -o run -- python3 tools/prof_fte.py --frames 10000 --reps 1
step ftepmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/ftepmc_${TAG}_write -o run -- python3 tools/prof_fte.py --frames 10000 --reps 1
python tools/pmc_summary.py $OUT/ftepmc_${TAG} $OUT/traffic_fte10k_${TAG}.json > $OUT/ftepmc_summary_${TAG}.log 2>&1; tail -5 $OUT/ftepmc_summary_${TAG}.log
PMC_ARGS="--no-cpu-baseline --no-fte --steps 3 --warmup 1 --ekf-seqs 0 --pipeline-seqs 0 --window-frames 0"
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_${TAG}_fetch -o run -- python3 bench.py $PMC_ARGS
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_${TAG}_write -o run -- python3 bench.py $PMC_ARGS
step pmc_valu 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_${TAG}_valu -o run -- python3 bench.py $PMC_ARGS
python tools/pmc_summary.py $OUT/pmc_${TAG} $OUT/traffic_${TAG}.json > $OUT/pmc_summary_${TAG}.log 2>&1; tail -5 $OUT/pmc_summary_${TAG}.log
rm -rf $OUT/pmc_${TAG}_fetch $OUT/pmc_${TAG}_write $OUT/pmc_${TAG}_valu $OUT/ftepmc_${TAG}_fetch $OUT/ftepmc_${TAG}_write $OUT/calib_${TAG}_fetch
TAILN=20 step time_dist_${TAG} 600 python tools/time_dist.py 10000 --worlds 1,8
echo done
