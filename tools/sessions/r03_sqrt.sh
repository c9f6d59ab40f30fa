#!/bin/bash
# mirror_factors' square roots without the generic denormal / class handling (default) against sqrtf
# (OCEAN_SQRT_CR=0 build): frame parity incl. large play times and the column-parity shards, then A/B
set -o pipefail
O=gpurun_out/r03sqrt; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frames or cfg4 or large_time or three_plane or parity or variants" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_lib.sh cfg3 "base sq0" 500 3 > $O/ab_cfg3.txt 2>&1 || exit 3
bash tools/ab_lib.sh cfg4 "base sq0" 50 2 > $O/ab_cfg4.txt 2>&1 || exit 4
cat $O/ab_cfg3.txt $O/ab_cfg4.txt
