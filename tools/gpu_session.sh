#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}
run() {
  local name=$1 lim=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
  tail -n 5 "$OUT/$name.log"
  case $rc in 124|137|134|139|143) echo "[$name] fatal rc=$rc, stopping session"; exit $rc;; esac
  return 0
}
STEPS=${STEPS:-all}
if [[ $STEPS == *all* || $STEPS == *test* ]]; then
  run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
fi
if [[ $STEPS == *all* || $STEPS == *smoke* ]]; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == *all* || $STEPS == *bench* ]]; then
  run bench 600 python bench.py ${BENCH_ARGS:-}
  grep '^{' "$OUT/bench.log" > "$OUT/bench_${TAG}.json" || true
fi
if [[ $STEPS == *all* || $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}" -o run -- python3 "$REPO/bench.py" --no-cpu-baseline --steps 200 --warmup 20 ${BENCH_ARGS:-}
fi
if [[ $STEPS == *ftetrace* ]]; then
  export TMPDIR=/tmp
  run ftetrace 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ftetrace_${TAG}" -o run -- python3 "$REPO/tools/prof_fte.py" --frames ${FTE_FRAMES:-1000}
  python tools/fte_iter_breakdown.py "$OUT/ftetrace_${TAG}" ${FTE_FRAMES:-1000} > "$OUT/fte_breakdown_${TAG}.log" 2>&1 || true
  tail -n 3 "$OUT/fte_breakdown_${TAG}.log"
fi
if [[ $STEPS == *list* ]]; then
  run counters 120 rocprofv3 -L
fi
if [[ ",$STEPS," == *,pmc,* ]]; then
  # HBM traffic (guide: separate passes; FETCH_SIZE x2 on gfx950) and FP64 VALU counts
  export TMPDIR=/tmp
  PMC_ARGS="--no-cpu-baseline --no-fte --steps 3 --warmup 1 --ekf-seqs 0 --pipeline-seqs 0 --window-frames 0"
  PMC_VALU=${PMC_VALU:-"SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES"}
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_${TAG}_fetch" -o run -- python3 "$REPO/bench.py" $PMC_ARGS
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_${TAG}_write" -o run -- python3 "$REPO/bench.py" $PMC_ARGS
  if [[ -n "${PMC_VALU:-}" ]]; then
    run pmc_valu 600 rocprofv3 --pmc $PMC_VALU --output-format csv -d "$OUT/pmc_${TAG}_valu" -o run -- python3 "$REPO/bench.py" $PMC_ARGS
  fi
  python tools/pmc_summary.py "$OUT/pmc_${TAG}" "$OUT/traffic_${TAG}.json" > "$OUT/pmc_summary_${TAG}.log" 2>&1 || true
fi
if [[ $STEPS == *ftepmc* ]]; then
  # FTE HBM traffic at configs[3] size (FETCH_SIZE / WRITE_SIZE passes of one 10k-frame solve)
  # and the FETCH_SIZE factor of 8-B and 16-B per lane streams (tools/probe/fetch_calib)
  export TMPDIR=/tmp
  run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_${TAG}_fetch" -o run -- "$REPO/tools/probe/fetch_calib"
  run ftepmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/ftepmc_${TAG}_fetch" -o run -- python3 "$REPO/tools/prof_fte.py" --frames 10000 --reps 1
  run ftepmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/ftepmc_${TAG}_write" -o run -- python3 "$REPO/tools/prof_fte.py" --frames 10000 --reps 1
  python tools/pmc_summary.py "$OUT/ftepmc_${TAG}" "$OUT/traffic_fte10k_${TAG}.json" > "$OUT/ftepmc_summary_${TAG}.log" 2>&1 || true
fi
echo done
