#!/bin/bash
# Round 6 final run (second: the mips change) of the tree on one box: the GPU suite + smoke, every config's bench line (cfg1 on
# the host, cfg2..cfg5), the cfg5 shard projection, and the multi-rank rehearsal (ranks share device 0: not a
# scaling measurement).  Outputs under gpurun_out/r06_final2/
set -o pipefail
OUT=gpurun_out/r06_final2; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/sessions/r04_tests.sh r06_final2 || exit 1
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('cfg3',d['value'],d['kernels_us'],d['roofline']['frac'],d['update_loop']['frames_per_s'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || { tail $OUT/bench_drv.err; exit 2; }
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 3; }
  python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c',d['value'],d['kernels_us'],d['roofline']['frac'])"
done
timeout -k 10 120 python bench.py --config cfg1 > $OUT/bench_cfg1.json 2> $OUT/bench_cfg1.err || { tail $OUT/bench_cfg1.err; exit 3; }
timeout -k 10 300 python tools/shard_bench.py --config cfg5 --worlds 1,2,4,8 --steps 100 > $OUT/shard_cfg5.jsonl 2> $OUT/shard_cfg5.err || { tail $OUT/shard_cfg5.err; exit 4; }
cat $OUT/shard_cfg5.jsonl
TAG=r06_final2/multi bash tools/sessions/r02_multi.sh || exit 5
echo session done
