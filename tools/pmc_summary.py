"""Summarise rocprofv3 --pmc passes (tools/gpu_session.sh STEPS=pmc) into
profiles/<round>/traffic.json: per (kernel, grid size) HBM bytes per launch and FP64 VALU
flops per launch.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE come from separate passes and are reported in KiB. On gfx950 FETCH_SIZE counts
half of the bytes of coalesced streaming reads. The guide gives this for 16 B per lane;
tools/probe/fetch_calib measured it for 8 B per lane too (profiles/r04/fetch_calib.txt: 1 GiB
read as double or double2, FETCH_SIZE = 0.500 GiB both times). So the x2 correction applies to
the share of a kernel's reads that are 8- or 16-B-per-lane streams (WIDE_SHARE below, from
the kernel's own load widths); the rest is taken as counted
(fetch_bytes = FETCH_SIZE x (1 + share)). Kernels without an entry are reported uncorrected,
with `fetch_calibrated: false`.
FP64 flops = 64 lanes x (2 FMA + ADD + MUL + TRANS) wave instructions (SQ_INSTS_VALU_*_F64;
an upper bound when lanes are masked off).

    python tools/pmc_summary.py gpurun_out/pmc_<tag> profiles/r01/traffic.json
"""
import json
import sys

import pandas as pd


# share of the algorithmic read bytes loaded 8 or 16 B per lane, per kernel. k_sba_lm reads,
# per point, 16 B x C of observations (double2 per lane), C mask bytes (1 B per lane:
# uncalibrated, taken as counted) and 24 B of start point (8-B loads): (96 + 24) / 126 at
# C = 6. The FTE kernels read float64 rows (8-B loads; the skeleton table's ints are
# negligible).
WIDE_SHARE = {'k_sba_lm': 120.0 / 126.0, 'k_cr_level': 1.0, 'k_cr_assemble_build': 1.0, 'k_cr_back_all': 1.0,
              'k_fte_linearize': 1.0, 'k_fte_cost': 1.0, 'k_cr_build': 1.0, 'k_fte_assemble': 1.0,
              'k_cr_back': 1.0, 'k_cr_trial': 1.0, 'k_cr_tau_partial': 1.0, 'k_cr_top': 1.0}


def load(prefix, kind):
    d = pd.read_csv(f'{prefix}_{kind}/run_counter_collection.csv')
    d['kernel'] = d.Kernel_Name.str.extract(r'(k_[a-z0-9_]+)')[0]
    return d.dropna(subset=['kernel'])


def main(prefix, out):
    rows = {}
    for kind in ('fetch', 'write', 'valu'):
        try:
            d = load(prefix, kind)
        except FileNotFoundError:
            continue
        g = d.groupby(['kernel', 'Grid_Size', 'Counter_Name']).Counter_Value.mean()
        for (k, grid, c), v in g.items():
            rows.setdefault(f'{k}@{grid}', {})[c] = float(v)
    res = {}
    for key, c in rows.items():
        r = {}
        if 'FETCH_SIZE' in c:
            kname = key.split('@')[0]
            share = WIDE_SHARE.get(kname)
            r['fetch_bytes'] = 1024 * c['FETCH_SIZE'] * (1.0 + (share or 0.0))
            r['fetch_calibrated'] = share is not None
            r['fetch_wide_share'] = share
        if 'WRITE_SIZE' in c:
            r['write_bytes'] = 1024 * c['WRITE_SIZE']
        if 'fetch_bytes' in r and 'write_bytes' in r:
            r['hbm_bytes'] = r['fetch_bytes'] + r['write_bytes']
        if 'SQ_INSTS_VALU_FMA_F64' in c:
            r['fp64_flops'] = 64 * (2 * c['SQ_INSTS_VALU_FMA_F64'] + c.get('SQ_INSTS_VALU_ADD_F64', 0)
                                    + c.get('SQ_INSTS_VALU_MUL_F64', 0) + c.get('SQ_INSTS_VALU_TRANS_F64', 0))
            r['valu_insts'] = c.get('SQ_INSTS_VALU')
        r['counters'] = c
        res[key] = r
    with open(out, 'w') as f:
        json.dump({'source': prefix, 'per_launch': res}, f, indent=1, sort_keys=True)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != 'counters'} for k, v in res.items()}, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
