"""Per-kernel / per-grid-size durations from a rocprofv3 kernel_trace.csv (last solve)."""
import collections
import csv
import glob
import sys

path = sys.argv[1]
f = path if path.endswith('.csv') else sorted(glob.glob(f'{path}/**/*kernel_trace.csv', recursive=True))[-1]
rows = list(csv.DictReader(open(f)))
acc = collections.defaultdict(list)
for r in rows:
    name = r['Kernel_Name'].split('(')[0].replace('void ', '')
    if not name.startswith('k_'):
        continue
    grid = int(r.get('Grid_Size_X', r.get('Grid_Size', 0)))
    wg = int(r.get('Workgroup_Size_X', r.get('Workgroup_Size', 1)))
    acc[(name, grid // max(wg, 1))].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = 0.0
for (name, nb), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f'{name:24s} blocks {nb:6d} calls {len(v):5d} mean {sum(v) / len(v):8.2f} us total {sum(v) / 1e3:8.2f} ms')
print(f'total {tot / 1e3:.2f} ms')
