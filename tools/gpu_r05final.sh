#!/bin/bash
# r05 final tree: GPU suite, smoke, bench, kernel stats, then the two-rank bench rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05final} STEPS=test,smoke,bench,prof bash tools/gpu_session.sh || exit $?
bash tools/rehearse_dist.sh
