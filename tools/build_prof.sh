#!/bin/bash
# Profiling build of the library (run here, on the CPU; the .so travels to the GPU box):
#   tools/build_prof.sh ekf   -> ekf.hip with -DEKF_PROFILE   (tools/prof_ekf_phases.py)
#   tools/build_prof.sh fte   -> fte.hip with -DFTE_PROFILE   (tools/prof_fte_phases.py, prof_cr_timeline.py)
#   FTE_PROF_DEFS="-DFTE_PROF_WIDE=1000" tools/build_prof.sh fte: the k_cr_level timeline of the
#   levels with >= 1000 elimination workgroups (-DFTE_PROF_WIDE_MAX=n: and <= n)
#   FTE_PROF_DEFS="-DPIVPRIO=0" OUT=libvar.so tools/build_prof.sh ftevar: fte.hip with other
#   compile-time settings and no profiling (A/B variants, loaded through ACINOSET_HIP_LIB)
# Output: acinoset_amd/csrc/build/libprof.so (the other objects from the normal build);
# OUT=name: acinoset_amd/csrc/build/name instead.
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "from acinoset_amd import build; build.build(verbose=False)"
B=acinoset_amd/csrc/build
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -Wno-unused-result"
case "${1:-ekf}" in
  ekf) /opt/rocm/bin/hipcc $F -DEKF_PROFILE -c acinoset_amd/csrc/ekf.hip -o $B/ekf_prof.o
       objs="$B/ctx.o $B/ekf_prof.o $B/fk.o $B/fte.o $B/sba.o $B/sba_ext.o $B/tri.o $B/pipeline.o";;
  fte) /opt/rocm/bin/hipcc $F -DFTE_PROFILE ${FTE_PROF_DEFS:-} -c acinoset_amd/csrc/fte.hip -o $B/fte_prof.o
       objs="$B/ctx.o $B/ekf.o $B/fk.o $B/fte_prof.o $B/sba.o $B/sba_ext.o $B/tri.o $B/pipeline.o";;
  ftevar) /opt/rocm/bin/hipcc $F ${FTE_PROF_DEFS:-} -c acinoset_amd/csrc/fte.hip -o $B/fte_var.o
       objs="$B/ctx.o $B/ekf.o $B/fk.o $B/fte_var.o $B/sba.o $B/sba_ext.o $B/tri.o $B/pipeline.o";;
  *) echo "usage: $0 ekf|fte|ftevar"; exit 2;;
esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $B/${OUT:-libprof.so}
echo "built $B/${OUT:-libprof.so} (${1:-ekf})"
