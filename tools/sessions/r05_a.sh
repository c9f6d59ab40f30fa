#!/bin/bash
# Round 5, session a: the readback engine (tools/d2hbench under rocprofv3, ring sequence with the D2H and
# the no-CU copy kinds), SURVEY section 7's pointwise clause measured (tools/pointwise.py), and the
# driver-shaped bench line with the reworked update loop.  Outputs under gpurun_out/r05_a/
set -o pipefail
OUT=gpurun_out/r05_a; mkdir -p $OUT
export TMPDIR=/tmp
for k in D2H NOCU; do
  timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$k -o run -- ./tools/d2hbench 10 0 $k > $OUT/prof_$k.log 2>&1 || exit 3
done
timeout -k 10 100 ./tools/d2hbench 20 > $OUT/d2hbench.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_drv.json 2> $OUT/bench_drv.err || { tail $OUT/bench_drv.err; exit 5; }
timeout -k 10 420 python -u tools/pointwise.py $OUT/pointwise.json > $OUT/pointwise.log 2>&1 || { tail $OUT/pointwise.log; exit 6; }
echo session done
