#!/bin/bash
# r06v: k_fte_linearize phase timeline (block 0, -DFTE_PROFILE library) at 1,000 and 10,000
# frames, and the smoke of the fresh-container build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_r06v.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke_r06v.log; exit 1; }
tail -2 $OUT/smoke_r06v.log
for n in 1000 10000; do
  timeout -k 10 300 python tools/prof_lin_phases.py $n > $OUT/lin_phases_r06v_$n.log 2>&1 || { echo "lin $n rc=$?"; tail -5 $OUT/lin_phases_r06v_$n.log; exit 1; }
  cat $OUT/lin_phases_r06v_$n.log
done
echo done
