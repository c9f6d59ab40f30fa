#!/bin/bash
# Rehearsal of the multi-rank bench path on a one-GPU box: ranks share device 0, so the
# numbers are not a scaling measurement -- this exercises the gloo barrier, reduce_timing,
# the tile / cascade / column-band shard plans and global tile seeds on hardware.
set -o pipefail
O=gpurun_out/${TAG:-r02m}; mkdir -p $O
run() {  # name world args...
  local name=$1 world=$2; shift 2
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $world --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $world "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; return 1; }
  echo "$name: $(cat $O/$name.json)"
}
run cfg4_w2 2 --config cfg4 --steps 40 --warmup 5 && \
run cfg5_w2 2 --config cfg5 --steps 40 --warmup 5 && \
run cfg5_w8 8 --config cfg5 --steps 40 --warmup 5 && \
run cfg3_w2 2 --config cfg3 --steps 100 --warmup 10
