#!/bin/bash
# Multi-rank rehearsal of the driver's scaling run on the 1-GPU box (ranks share cuda:0 and the
# box's CPU share): N=2 with every extra phase on rank 0 (the driver's default line), N=4 without.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/${1:-r5_scale}
mkdir -p "$out"
run() {  # run <n> <port> <tag> [bench args...]
  local n=$1 port=$2 tag=$3
  shift 3
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus "$n" --steps 20 --warmup 5 "$@" > "$out/$tag.json" 2> "$out/$tag.err"
}
run 2 29611 n2 --full-out "$out/n2_full.json" &&
run 4 29612 n4 --no-extras --full-out "$out/n4_full.json"
