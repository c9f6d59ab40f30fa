#!/bin/bash
# Multi-rank rehearsal of the round-4 tree on the one-GPU box (ranks share device 0: not a scaling
# measurement): the driver's cfg3 N = 2 / 4 launch shape, the cfg4 and cfg5 shard plans over gloo.
set -o pipefail
export TAG=${TAG:-r04_multi}
bash tools/sessions/r02_multi.sh || exit 1
O=gpurun_out/$TAG
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 4 --steps 100 --warmup 10 > $O/cfg3_w4.json 2> $O/cfg3_w4.err || { tail -20 $O/cfg3_w4.err; exit 2; }
echo "cfg3_w4: $(cat $O/cfg3_w4.json)"
