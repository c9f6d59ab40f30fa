#!/bin/bash
# Round 4 closing run on one box: the GPU test suite + smoke, the bench lines of every config, the cfg5
# shard projection (tools/shard_bench.py) and SQ counters of the cfg5 frame (pass A3Q) and of a parity
# shard (pass A3PP).  Outputs under gpurun_out/r04_final/
set -o pipefail
OUT=gpurun_out/r04_final; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/sessions/r04_tests.sh r04_final || exit 1
# the chip ceilings the bench line quotes (built in the build container: hipcc -O3 tools/<x>.hip -o tools/<x>)
timeout -k 10 60 ./tools/wrbench > $OUT/wrbench.txt 2>&1 || exit 6
timeout -k 10 60 ./tools/aqbench > $OUT/aqbench.txt 2>&1 || exit 7
timeout -k 10 60 ./tools/bqbench > $OUT/bqbench.txt 2>&1 || exit 8
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 3; }
done
timeout -k 10 300 python tools/shard_bench.py --config cfg5 --worlds 1,2,4,8 --steps 100 > $OUT/shard_cfg5.jsonl 2> $OUT/shard_cfg5.err || { tail $OUT/shard_cfg5.err; exit 4; }
cat $OUT/shard_cfg5.jsonl
bash tools/pmc_sq_cmd.sh $OUT/sq_cfg5 python3 bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu-baseline --no-ifft-stage --no-beyond-cache --no-update-loop || exit 5
echo session done
