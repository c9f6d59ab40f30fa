#!/bin/bash
# Mirror-factor sharing in the one-row Q pass: A/B at cfg3 (vs AQ) and cfg5 (A3Q at 4096), parity check.
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
bash tools/ab_env_lib.sh cfg3 "base:- base:OCEAN_AQ_ROWS=2 base:OCEAN_AQ_ROWS=3 base:OCEAN_AQ_ROWS=3,OCEAN_AQ_ROWS_PF=0" 300 3 > $O/ab_cfg3.txt 2>&1 || { cat $O/ab_cfg3.txt; exit 1; }
cat $O/ab_cfg3.txt
bash tools/ab_env_lib.sh cfg5 "base:- base:OCEAN_A3Q_SHARE=1" 50 2 > $O/ab_cfg5.txt 2>&1 || { cat $O/ab_cfg5.txt; exit 2; }
cat $O/ab_cfg5.txt
