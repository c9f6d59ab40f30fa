#!/bin/bash
# Timing build (wrong outputs): pass AQ at cfg3 with its 2052 items cut to 2048 (8 per CU), to size the
# cost of the 4 items past an even deal (the self-mirror rows 0 and N/2 of each unit)
set -o pipefail
O=gpurun_out/r03tail; mkdir -p $O
bash tools/ab_lib.sh cfg3 "base tail" 500 3 > $O/ab_cfg3.txt 2>&1 || exit 3
cat $O/ab_cfg3.txt
