#!/bin/bash
# r05 session H: occupancy of k_cr_wide vs k_cr_level (PMC: SQ_WAVE_CYCLES, SQ_WAVES, GRBM_GUI_ACTIVE)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-3} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
step pmc_occ 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_occ -o run -- python3 tools/prof_fte.py --frames 10000 --reps 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_occ/**/*counter_collection.csv', recursive=True)
if not f: print('no csv'); raise SystemExit
rows = list(csv.DictReader(open(f[0])))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = (r['Kernel_Name'].split('(')[0][:26], int(r['Grid_Size']) // max(1, int(r['Workgroup_Size'])))
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in acc.items():
    if 'k_cr' not in k[0]: continue
    print(k, {c: f'{x:.3g}' for c, x in v.items()})
PY
rm -rf $OUT/pmc_occ
echo done
