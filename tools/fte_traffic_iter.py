"""HBM bytes of one FTE LM iteration by kernel: the per-launch PMC summary of one solve
(tools/pmc_summary.py over FETCH_SIZE / WRITE_SIZE passes of tools/prof_fte.py, FETCH_SIZE
calibrated) applied to the iteration's launch sequence (tools/fte_iter_sequence.py):
python tools/fte_traffic_iter.py traffic_fte10k.json seq10k.log. Launches of one kernel at one
grid share a PMC entry (its mean over the solve), e.g. levels 0 and 1 at 10,000 frames."""
import json
import re
import sys

BLOCK = {'k_cr_level': 1024, 'k_cr_assemble_build': 1024, 'k_cr_back_all': 640, 'k_fte_linearize': 256,
         'k_fte_lm': 256}
pl = json.load(open(sys.argv[1]))['per_launch']
tot = rd = wr = 0.0
rows = []
for line in open(sys.argv[2]):
    m = re.match(r'\s+(k_[a-z_]+)(<[^>]*>)?\s+grid\s+(\d+)\s+([\d.]+) us', line)
    if not m:
        if line.startswith('k_cr_level by position'):
            break
        continue
    name, grid, us = m.group(1), int(m.group(3)), float(m.group(4))
    block = BLOCK.get(name, 256)
    targs = [a.strip() for a in (m.group(2) or '<>')[1:-1].split(',')]
    if name == 'k_cr_assemble_build' and len(targs) == 2:  # <NB, threads> since round 6
        block = int(targs[1])
    e = pl.get(f'{name}@{grid * block}')
    if e is None:
        rows.append((name, grid, us, None, None))
        continue
    tot += e['hbm_bytes']
    rd += e['fetch_bytes']
    wr += e['write_bytes']
    rows.append((name, grid, us, e['fetch_bytes'], e['write_bytes']))
for name, grid, us, f, w in rows:
    s = f'{f / 1e6:8.1f} MB read {w / 1e6:8.1f} MB written' if f is not None else '   (no PMC entry)'
    print(f'{name:22s} grid {grid:6d} {us:8.2f} us {s}')
print(f'per iteration: {tot / 1e9:.3f} GB ({rd / 1e9:.3f} read, {wr / 1e9:.3f} written)')
