#!/bin/bash
# r05 session Q: register / LDS footprint the hardware sees for k_ekf_gain_t (kernel-trace columns)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kq -o run -- python3 tools/time_ekf_leg.py default fd 8 60 > $OUT/kq.log 2>&1; echo rc=$?
f=$(find $OUT/kq -name '*kernel_trace.csv' | head -1)
head -1 $f
grep -m2 "gain_t\|k_cr_back_all\|k_cr_level" $f | cut -c1-400
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
seen = set()
for r in rows:
    k = r.get('Kernel_Name', '')[:60]
    if k in seen: continue
    seen.add(k)
    print(k, {c: r[c] for c in r if any(x in c for x in ('VGPR', 'SGPR', 'LDS', 'Scratch', 'Workgroup_Size'))})
PY
rm -rf $OUT/kq
