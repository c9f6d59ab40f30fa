#!/bin/bash
# rocprofv3 kernel statistics of the cfg2 / cfg4 / cfg5 bench workloads (one pass each, tracing only).
set -o pipefail
O=gpurun_out/prof_${TAG:-r02cfg}
mkdir -p $O
export TMPDIR=/tmp
for c in cfg2 cfg4 cfg5; do
  steps=200; [ $c = cfg2 ] && steps=2000; [ $c = cfg5 ] && steps=40
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- \
    python3 bench.py --config $c --steps $steps --warmup 10 --no-cpu-baseline > $O/$c.json 2> $O/$c.log || exit 1
done
echo done
