#!/bin/bash
# r06d: FTE per-iteration profiles (configs[2] 1,000 and configs[3] 10,000 frames): kernel trace
# -> iteration sequence, FETCH_SIZE / WRITE_SIZE passes -> calibrated HBM bytes per launch,
# joined into fte_iter_<n>k.json (tools/fte_iter_json.py) for bench.py's roofline fields
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
T=${T:-r06d}
for F in 10000 1000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/ftetrace_$F -o run -- python3 tools/prof_fte.py --frames $F > $OUT/ftetrace_$F.log 2>&1 || { echo "trace $F failed"; tail -5 $OUT/ftetrace_$F.log; exit 1; }
  python tools/fte_iter_sequence.py $OUT/ftetrace_$F > $OUT/seq_${T}_$F.log 2>&1
  python tools/fte_iter_breakdown.py $OUT/ftetrace_$F $F > $OUT/fte_kernel_totals_${T}_$F.log 2>&1
  tail -n 1 $OUT/fte_kernel_totals_${T}_$F.log
  rm -rf $OUT/ftetrace_$F
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ftepmc_${T}_${F}_fetch -o run -- python3 tools/prof_fte.py --frames $F --reps 1 > $OUT/ftepmc_fetch_$F.log 2>&1 || { echo "fetch pass $F failed"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/ftepmc_${T}_${F}_write -o run -- python3 tools/prof_fte.py --frames $F --reps 1 > $OUT/ftepmc_write_$F.log 2>&1 || { echo "write pass $F failed"; exit 1; }
  python tools/pmc_summary.py $OUT/ftepmc_${T}_${F} $OUT/traffic_fte${F}_${T}.json > $OUT/ftepmc_summary_${T}_$F.log 2>&1
  python tools/fte_traffic_iter.py $OUT/traffic_fte${F}_${T}.json $OUT/seq_${T}_$F.log > $OUT/fte_traffic_iter_${T}_$F.log 2>&1
  tail -n 1 $OUT/fte_traffic_iter_${T}_$F.log
  python tools/fte_iter_json.py $OUT/fte_traffic_iter_${T}_$F.log $F $OUT/fte_iter_$((F / 1000))k.json
  rm -rf $OUT/ftepmc_${T}_${F}_fetch/*/*agent* $OUT/ftepmc_${T}_${F}_write/*/*agent* 2>/dev/null
done
echo done
