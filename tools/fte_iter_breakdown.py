"""Per-kernel (name, grid) time per LM iteration of the last FTE solve(s) in a rocprofv3
kernel trace: python tools/fte_iter_breakdown.py gpurun_out/ftetrace [frames]."""
import collections
import csv
import glob
import sys

f = glob.glob(f'{sys.argv[1]}/**/*kernel_trace.csv', recursive=True)[0]
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
rows = rows[len(rows) * 2 // 3:]
acc = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').split('<')[0]
    g = int(r['Grid_Size_X']) // max(int(r['Workgroup_Size_X']), 1)
    acc[(n, g)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
nit = max(1, len(acc.get(('k_fte_linearize', nf), [])))
tot = 0.0
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f'{k[0]:24s} grid {k[1]:6d} calls {len(v):4d} mean {sum(v) / len(v):8.2f} us  per-iter {sum(v) / nit:7.1f} us')
print(f'iterations {nit}, kernel time per iteration {tot / nit:.1f} us')
