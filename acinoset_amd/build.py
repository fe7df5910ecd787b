"""Build libacinoset_hip.so in-tree: hipcc --offload-arch=gfx950, one object per
csrc/*.hip compiled in parallel, then linked into acinoset_amd/libacinoset_hip.so.
The built .so travels to the GPU box with the repo snapshot (it is git-ignored)."""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, 'libacinoset_hip.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'
CFLAGS = ['-O3', '-std=c++17', '-fPIC', f'--offload-arch={ARCH}', '-I', os.path.join(REPO, 'include'),
          '-Wno-unused-result']


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


def build(force: bool = False, verbose: bool = True, jobs: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    deps = srcs + glob.glob(os.path.join(CSRC, '*.hpp')) + [os.path.join(REPO, 'include', 'acinoset_hip.h')]
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= _newest(deps):
        return OUT
    objdir = os.path.join(CSRC, 'build')
    os.makedirs(objdir, exist_ok=True)
    hdr_t = _newest([d for d in deps if not d.endswith('.hip')])

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + '.o')
        if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_t):
            return obj
        cmd = [HIPCC, *CFLAGS, '-c', src, '-o', obj]
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', *objs, '-o', OUT]
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
