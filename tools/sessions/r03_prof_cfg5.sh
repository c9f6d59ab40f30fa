#!/bin/bash
# rocprofv3 stats + FETCH/WRITE of the cfg5 frame (4 x 4096^2) -> gpurun_out/prof_r03final_cfg5
set -o pipefail
bash tools/profile.sh r03final_cfg5 --config cfg5 --steps 20 --warmup 5 --no-cpu-baseline --no-ifft-stage --no-beyond-cache || exit 1
echo done
