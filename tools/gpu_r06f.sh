#!/bin/bash
# r06f: r06e (early-pivot timeline A/B, SBA tests + SBA bench legs) then r06d (FTE per-iteration
# profiles at 1,000 and 10,000 frames) in one box session
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r06e.sh || exit $?
T=r06f bash tools/gpu_r06d.sh
