#!/bin/bash
# Round 4: the cfg5 shard projection and the cfg5 / cfg3 bench lines again on another box (VERDICT r03
# item 6: >= 7x against the same run's single-GPU frame on two boxes)
set -o pipefail
OUT=gpurun_out/r04_box2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/shard_bench.py --config cfg5 --worlds 1,2,4,8 --steps 100 > $OUT/shard_cfg5.jsonl 2> $OUT/shard_cfg5.err || { tail $OUT/shard_cfg5.err; exit 1; }
cat $OUT/shard_cfg5.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --config cfg5 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail $OUT/bench_cfg5.err; exit 2; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
hostname > $OUT/host.txt
echo session done
