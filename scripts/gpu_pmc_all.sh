#!/bin/bash
# PMC passes for c2, c3, c4 (each pass its own time limit; stop at the first fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "$@"; do
  bash scripts/gpu_pmc.sh $cfg || exit $?
done
