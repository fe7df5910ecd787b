"""Per-kernel resource usage of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage):
VGPRs, AGPRs, VGPR / SGPR spills, scratch and LDS, one line per kernel.
usage: python tools/kres.py acinoset_amd/csrc/ekf.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950', '-I', 'include', '-c', src,
       '-o', '/tmp/kres.o', '-Rpass-analysis=kernel-resource-usage']
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r'remark: ([^:]+): (.*?) \[-Rpass', line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == 'Function Name':
        cur = {'name': v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt not in r['name']:
        continue
    print(f"{r['name'][:70]:70s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>4} "
          f"vspill {r.get('VGPRs Spill', '?'):>4} sspill {r.get('SGPRs Spill', '?'):>4} "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} lds {r.get('LDS Size [bytes/block]', '?'):>6} occ {r.get('Occupancy [waves/SIMD]', '?')}")
