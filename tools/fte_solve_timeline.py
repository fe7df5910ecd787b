"""Per-solve timeline of a rocprofv3 kernel trace of tools/prof_fte_dev.py: the span from a
solve's first kernel to its last, the kernel time inside it and the idle gaps, split into
before the first k_fte_linearize, the iterations, and after the last k_fte_lm.
python tools/fte_solve_timeline.py <trace dir>"""
import glob
import sys

import pandas as pd

f = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
d = pd.read_csv(f).sort_values('Start_Timestamp')
d['k'] = d.Kernel_Name.str.extract(r'(k_[a-z0-9_]+|__amd_rocclr_[a-zA-Z]+|[a-z_]+elementwise)')[0].fillna('other')
# solves are separated by the host's synchronisation: a gap > 200 us
gap = d.Start_Timestamp.diff().fillna(1e12)
d['solve'] = (gap > 200e3).cumsum()
for s, g in d.groupby('solve'):
    t0, t1 = g.Start_Timestamp.min(), g.End_Timestamp.max()
    busy = (g.End_Timestamp - g.Start_Timestamp).sum()
    lin = g[g.k == 'k_fte_linearize']
    lm = g[g.k == 'k_fte_lm']
    if len(lin) == 0:
        continue
    pre = lin.Start_Timestamp.min() - t0
    post = t1 - lm.End_Timestamp.max() if len(lm) else 0
    print(f'solve {s}: span {(t1 - t0) / 1e3:8.1f} us, kernels {busy / 1e3:8.1f} us, idle {(t1 - t0 - busy) / 1e3:7.1f} us, '
          f'before the 1st linearize {pre / 1e3:6.1f} us, after the last LM {post / 1e3:6.1f} us, '
          f'{len(lm)} k_fte_lm, {len(g)} kernels')
    if s == d.solve.max():
        print(g.groupby('k').apply(lambda x: pd.Series({'n': len(x), 'us': (x.End_Timestamp - x.Start_Timestamp).sum() / 1e3}))
              .sort_values('us', ascending=False).to_string())
