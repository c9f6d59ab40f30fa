#!/bin/bash
# Round 4 closing profiles of the final library (stamped, tools/profile.sh): the cfg3 bench frame, the
# update loop (mip kernels), the cfg5 and cfg4 frames; SQ counters of the cfg5 parity shards (pass A3PP).  Summaries: python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>
set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ifft-stage --no-beyond-cache --no-update-loop"
bash tools/profile.sh r04f_cfg3 cfg3 || exit 1
bash tools/profile.sh r04f_update update_loop python3 bench.py --only-update-loop --steps 200 --warmup 20 || exit 2
bash tools/profile.sh r04f_cfg5 cfg5 $B --config cfg5 --steps 30 --warmup 5 || exit 3
bash tools/profile.sh r04f_cfg4 cfg4 $B --config cfg4 --steps 30 --warmup 5 || exit 4
bash tools/pmc_sq_cmd.sh gpurun_out/r04_final_sq_shard python3 tools/shard_bench.py --config cfg5 --worlds 8 --steps 20 || exit 5
echo session done
