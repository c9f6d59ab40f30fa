#!/bin/bash
# SQ counters: cfg3 frame (pass AQ, BQ) and the cfg5 8-GPU parity shard (pass A3P, C1, C2).
set -o pipefail
bash tools/pmc_sq_cmd.sh gpurun_out/r03d_sq_cfg3 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-ifft-stage --no-beyond-cache || exit 1
bash tools/pmc_sq_cmd.sh gpurun_out/r03d_sq_cfg5p python3 tools/shard_bench.py --config cfg5 --worlds 8 --steps 20 --warmup 3 || exit 2
echo done
