#!/bin/bash
# Round-2 closing profile on the GPU box: the fused cfg3 frame (kernel trace + FETCH / WRITE
# passes, tools/profile.sh), the operator IFFT's kernel stats, and cfg5's 8-way shard times.
set -o pipefail
TAG=${TAG:-r02y}
O=gpurun_out/prof_$TAG
bash tools/profile.sh $TAG || exit $?
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ifft -o run -- python3 tools/ifft_bench.py 200 > $O/ifft.log 2>&1 || exit 4
timeout -k 10 300 python3 tools/shard_bench.py --config cfg5 --worlds 8 --steps 50 > $O/shard_cfg5.jsonl 2> $O/shard.err || exit 5
echo done
