#!/bin/bash
# Round-5 box session: the driver's sequence (GPU tier, smoke, bench line + full record), then
# the stub A/B. Output under gpurun_out/$1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
name=${1:-r5}
bash scripts/box_round.sh "$name" || exit $?
OUT="$name/stub_ab" RUNS=${RUNS:-6} bash scripts/box_r5_stub_ab.sh
