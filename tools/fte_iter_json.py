"""One FTE LM iteration at a given size as JSON for bench.py's configs[3] line: the per-launch
table written by tools/fte_traffic_iter.py (kernel, grid, mean us, MB read, MB written per
launch, in iteration order) -> {frames, kernel_us_per_iter, hbm_bytes_per_iter, kernels:
[{kernel, grid, us, share, hbm_bytes}], dominant}.
    python tools/fte_iter_json.py fte_traffic_iter_10k.log 10000 out.json"""
import json
import re
import os
import sys

rows = []
for line in open(sys.argv[1]):
    m = re.match(r'(k_[a-z_]+)\s+grid\s+(\d+)\s+([\d.]+) us\s+([\d.]+) MB read\s+([\d.]+) MB written', line)
    if m:
        rows.append(dict(kernel=m.group(1), grid=int(m.group(2)), us=float(m.group(3)),
                         hbm_bytes=(float(m.group(4)) + float(m.group(5))) * 1e6))
tot_us = sum(r['us'] for r in rows)
for r in rows:
    r['share'] = r['us'] / tot_us
by = {}
for r in rows:
    by.setdefault(r['kernel'], [0.0, 0.0])
    by[r['kernel']][0] += r['us']
    by[r['kernel']][1] += r['hbm_bytes']
dom = max(by.items(), key=lambda kv: kv[1][0])
out = {'frames': int(sys.argv[2]), 'kernel_us_per_iter': tot_us, 'hbm_bytes_per_iter': sum(r['hbm_bytes'] for r in rows),
       'kernels': rows,
       'by_kernel': {k: {'us': v[0], 'share': v[0] / tot_us, 'hbm_bytes': v[1]} for k, v in by.items()},
       'dominant': {'kernel': dom[0], 'us': dom[1][0], 'share': dom[1][0] / tot_us, 'hbm_bytes': dom[1][1]},
       'source': os.path.basename(sys.argv[1])}
json.dump(out, open(sys.argv[3], 'w'), indent=1)
print(json.dumps(out['dominant']), f"{out['hbm_bytes_per_iter'] / 1e9:.3f} GB/iter, {tot_us:.0f} us/iter")
