#!/bin/bash
# Round 5, session g: the default bench line (cfg3) and the cfg5 line of the current library, with the r05p_*
# records in the tree (record.match "lib" expected), and smoke().
set -o pipefail
OUT=gpurun_out/r05_g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
timeout -k 10 300 python bench.py --config cfg5 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { tail $OUT/bench_cfg5.err; exit 3; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 4; }
echo session done
