#!/bin/bash
# Round-3 closing run after the folded operator at 4096 -> gpurun_out/r03zzz (copied into profiles/r03zzz*):
# -m gpu suite, smoke, rocprofv3 of the cfg3 frame (trace + FETCH + WRITE), rocprofv3 of the 4096 operator,
# the bench line of every config, and the cfg5 shard projection.
set -o pipefail
O=gpurun_out/r03zzz; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
bash tools/profile.sh r03zzz || exit 6
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P=gpurun_out/prof_r03zzz_op4k; mkdir -p $P
PROG="python3 tools/ifft_op.py 4096 4 1 10"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $PROG > $P/trace.log 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $PROG > $P/fetch.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $PROG > $P/write.log 2>&1 || exit 13
timeout -k 10 300 python3 bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 7
timeout -k 10 200 python3 bench.py --config cfg2 --steps 2000 --warmup 100 > $O/bench_cfg2.json 2> $O/bench_cfg2.err || exit 8
timeout -k 10 300 python3 bench.py --config cfg4 --steps 50 --warmup 5 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit 9
timeout -k 10 300 python3 bench.py --config cfg5 --steps 50 --warmup 5 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || exit 10
timeout -k 10 400 python3 tools/shard_bench.py --config cfg5 --worlds 1,2,4,8 --steps 50 > $O/shard_cfg5.jsonl 2> $O/shard.err || exit 11
echo done
