"""One LM iteration of the last FTE solve in a rocprofv3 kernel trace, kernel by kernel in
launch order (name, grid, duration, gap before it), plus the per-level means of
k_cr_level over the solve's iterations:
    python tools/fte_iter_sequence.py gpurun_out/ftetrace_TAG"""
import collections
import csv
import glob
import sys

f = glob.glob(f'{sys.argv[1]}/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))


def name(r):
    return r['Kernel_Name'].split('(')[0].replace('void ', '')


def grid(r):
    return int(r['Grid_Size_X']) // max(int(r['Workgroup_Size_X']), 1)


lm = [i for i, r in enumerate(rows) if name(r) == 'k_fte_lm']
# iterations = spans between consecutive k_fte_lm launches of the last solve
its = [rows[a + 1:b + 1] for a, b in zip(lm[:-1], lm[1:])]
its = its[len(its) * 2 // 3:]
mid = its[len(its) // 2]
print(f'one iteration ({len(mid)} kernels), in launch order:')
prev_end = None
tot = 0.0
for r in mid:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    prev_end = e
    tot += (e - s) / 1e3
    print(f'  {name(r):26s} grid {grid(r):6d}  {(e - s) / 1e3:8.2f} us   gap {gap:6.2f} us')
print(f'  kernels {tot:.1f} us, wall {(int(mid[-1]["End_Timestamp"]) - int(mid[0]["Start_Timestamp"])) / 1e3:.1f} us')
# the k-th k_cr_level launch of each iteration, averaged
lv = collections.defaultdict(list)
for it in its:
    k = 0
    for r in it:
        if name(r).startswith('k_cr_level'):
            lv[k].append((grid(r), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
            k += 1
print('k_cr_level by position in the iteration (mean over iterations):')
for k in sorted(lv):
    v = lv[k]
    print(f'  level {k:2d} grid {v[0][0]:6d}  {sum(t for _, t in v) / len(v):8.2f} us  (n={len(v)})')
