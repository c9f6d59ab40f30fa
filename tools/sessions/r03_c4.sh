#!/bin/bash
# C1 / C2 (N = 4096 column passes) through scalar bases + 32-bit lane offsets (default) against the
# 64-bit addresses (c4old build): frame parity at 2048 / 4096 incl. the column-parity shards, then A/B on cfg5
set -o pipefail
O=gpurun_out/r03c4; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "4096 or 2048 or column or band or shard" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_lib.sh cfg5 "base c4old" 50 3 > $O/ab_cfg5.txt 2>&1 || exit 3
cat $O/ab_cfg5.txt
