#!/bin/bash
# Round-3 closing measurements, part 2: the bench lines of every config (after part 1's profiles are
# committed, so the cfg3 line quotes this round's records), the operator beyond the cache under
# rocprofv3, and the cfg5 shard projection.
set -o pipefail
O=gpurun_out/r03z2; mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 1
cat $O/bench_cfg3.json
timeout -k 10 200 python3 bench.py --config cfg2 --steps 2000 --warmup 100 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit 2
timeout -k 10 300 python3 bench.py --config cfg4 --steps 50 --warmup 5 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit 3
timeout -k 10 300 python3 bench.py --config cfg5 --steps 50 --warmup 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 4
timeout -k 10 400 python3 tools/shard_bench.py --config cfg5 --worlds 1,2,4,8 --steps 50 > $O/shard_cfg5.jsonl 2> $O/shard.err || exit 5
echo done
