#!/bin/bash
# A/B of library builds on one shard shape of tools/shard_bench.py, interleaved over rounds:
#   bash tools/ab_shard.sh "<variant> ..." [config] [world] [rounds] [extra shard_bench args]
set -e
mkdir -p gpurun_out
for r in $(seq 1 ${4:-2}); do
  for v in $1; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 300 python tools/shard_bench.py --config ${2:-cfg5} --worlds ${3:-8} \
      --steps 50 $5 > gpurun_out/abs_$v.json 2> gpurun_out/abs_$v.err
    echo "$r $v $(python -c "
import json;d=json.load(open('gpurun_out/abs_$v.json'))
print(d['projected_frames_per_s'], [(s['ms_per_frame'], s['pass_a_ms'], s['pass_b_ms']) for s in d['shards'].values()])")"
  done
done
