#!/bin/bash
# Round 5, session m: what holds pass BQ once DISP stays in the cache -- bqbench's DC shape (mode 13), and
# cfg3 with 4-column tiles (OCEAN_TILE_W=4: two pass-BQ workgroups per CU) against the default 8.
set -o pipefail
OUT=gpurun_out/r05_m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/bqbench > $OUT/bqbench.txt 2>&1 || exit 2
grep -E "grid|texture layout, nt |TURB carries|DISP cached" $OUT/bqbench.txt
bash tools/ab_env_lib.sh cfg3 "base:- base:OCEAN_TILE_W=4" 300 3 > $OUT/ab_tw.txt 2>&1 || { tail $OUT/ab_tw.txt; exit 3; }
cat $OUT/ab_tw.txt
echo session done
