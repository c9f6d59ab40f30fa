#!/bin/bash
# Round-3 closing run after the N >= 2048 operator change -> gpurun_out/r03zz (copied into profiles/r03zz):
# -m gpu suite, smoke, rocprofv3 of the cfg3 frame (trace + FETCH + WRITE), the bench line of every
# config, and the cfg5 shard projection.
set -o pipefail
O=gpurun_out/r03zz; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
bash tools/profile.sh r03zz || exit 6
timeout -k 10 300 python3 bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 7
timeout -k 10 200 python3 bench.py --config cfg2 --steps 2000 --warmup 100 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit 8
timeout -k 10 300 python3 bench.py --config cfg4 --steps 50 --warmup 5 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit 9
timeout -k 10 300 python3 bench.py --config cfg5 --steps 50 --warmup 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 10
timeout -k 10 400 python3 tools/shard_bench.py --config cfg5 --worlds 1,2,4,8 --steps 50 > $O/shard_cfg5.jsonl 2> $O/shard.err || exit 11
echo done
