#!/bin/bash
# r05 session I: level-0 zero skips in k_cr_level (tests + traces); k_cr_wide occupancy (PMC)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-3} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
step pytest_fte_r05i 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_dist.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step tr10k_l0 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_l0 -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
python tools/fte_iter_sequence.py $OUT/tr10k_l0 > $OUT/seq10k_l0skip.log 2>&1; grep -E "level  [0-4] |kernels" $OUT/seq10k_l0skip.log | head -8
step tr1k_l0 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr1k_l0 -o run -- python3 tools/prof_fte.py --frames 1000 --reps 3
python tools/fte_iter_sequence.py $OUT/tr1k_l0 > $OUT/seq1k_l0skip.log 2>&1; grep -E "level  [0-2] |kernels" $OUT/seq1k_l0skip.log | head -5
rm -rf $OUT/tr10k_l0 $OUT/tr1k_l0
export ACS_CR_WIDE_MIN=256
step pmc_occ 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_occ -o run -- python3 tools/prof_fte.py --frames 10000 --reps 1
unset ACS_CR_WIDE_MIN
python3 - > $OUT/pmc_occ_summary.log 2>&1 <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/pmc_occ/**/*counter_collection.csv', recursive=True)
rows = list(csv.DictReader(open(f[0])))
print(list(rows[0].keys()))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = (r['Kernel_Name'].split('(')[0][:26], r.get('Grid_Size', '?'), r.get('Workgroup_Size', '?'))
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in acc.items():
    if 'k_cr' not in k[0]: continue
    print(k, {c: f'{x:.4g}' for c, x in v.items()})
PY
cat $OUT/pmc_occ_summary.log | head -20
rm -rf $OUT/pmc_occ
echo done
