#!/bin/bash
# r06zf: the compact-row assembly with the special loads in their old per-kind branches and the
# batch touch (libv.so: 2 spilled VGPRs) against the production form (regrouped specials: 9
# spilled VGPRs), kernel traces at 10,000 frames interleaved, and WRITE_SIZE of both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
V=$PWD/acinoset_amd/csrc/build/libv.so
TAG=r06zf
trace() {  # name frames [lib]
  local d=$OUT/abtrace_$1
  local lib=${3:-}
  env ${lib:+ACINOSET_HIP_LIB=$lib} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/prof_fte.py --frames $2 > $d.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "trace $1 rc=$rc"; tail -5 $d.log; exit 1; }
  python tools/fte_iter_breakdown.py $d $2 > $OUT/fte_kernel_totals_$1_$TAG.log 2>&1
  echo "$1: $(grep -m1 k_cr_assemble_build $OUT/fte_kernel_totals_$1_$TAG.log)"
  rm -rf $d
}
for r in a b c; do
  trace prod_10k_$r 10000
  trace v_10k_$r 10000 $V
done
for x in prod v; do
  lib=""; [ $x = v ] && lib=$V
  env ${lib:+ACINOSET_HIP_LIB=$lib} timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$x -o run -- python3 tools/prof_fte.py --frames 10000 --reps 1 > $OUT/pmcw_$x.log 2>&1 || { echo "pmc $x failed"; exit 1; }
  python - $OUT/pmcw_$x <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'k_cr_assemble_build' in r['Kernel_Name']:
        acc[r['Dispatch_Id']].append(float(r['Counter_Value']))
v = [sum(x) for x in acc.values()]
print(sys.argv[1].split('/')[-1], 'k_cr_assemble_build WRITE_SIZE per launch (KB, uncalibrated)', round(sum(v) / len(v)), 'over', len(v))
PY
  rm -rf $OUT/pmcw_$x
done
echo done
