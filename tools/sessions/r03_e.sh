#!/bin/bash
# A/B of pass A at cfg3 / cfg4 (mirror-pair AQ against one-row A3Q at 1024, slim image), then SQ counters.
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
bash tools/ab_env_lib.sh cfg3 "base:- base:OCEAN_AQ_ROWS=1 base:OCEAN_AQ_ROWS=2 base:OCEAN_AQ_ROWS=2,OCEAN_AQ_ROWS_PF=0" 300 3 > $O/ab_cfg3.txt 2>&1 || { cat $O/ab_cfg3.txt; exit 1; }
bash tools/ab_env_lib.sh cfg4 "base:- base:OCEAN_AQ_ROWS=2 base:OCEAN_AQ_ROWS=2,OCEAN_AQ_ROWS_PF=0" 50 2 > $O/ab_cfg4.txt 2>&1 || { cat $O/ab_cfg4.txt; exit 2; }
bash tools/r03_d.sh || exit 3
echo done
