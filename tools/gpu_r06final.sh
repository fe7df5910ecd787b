#!/bin/bash
# Round-6 closing session: FTE per-iteration profiles (fte_iter_{1,10}k.json for the bench line),
# then the GPU tests, smoke, bench, rocprofv3 kernel stats of the bench and the SBA PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:-r06final} bash tools/gpu_r06d.sh || exit $?
cp gpurun_out/fte_iter_1k.json gpurun_out/fte_iter_10k.json profiles/r06/
TAG=${TAG:-r06final} STEPS="test,smoke,bench,prof,pmc" bash tools/gpu_session.sh
