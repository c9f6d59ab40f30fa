#!/bin/bash
# Round 6 final profiles of the library with TURB's mips from the foam state (stamped, tools/profile.sh): the cfg3 frame, the cfg3 operator
# (in and beyond the cache), the 4096 operator, the update loop, the cfg5 and cfg4 frames.
#   python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>
set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ifft-stage --no-beyond-cache --no-update-loop"
bash tools/profile.sh r06i_cfg3 cfg3 || exit 1
bash tools/profile.sh r06i_ifft ifft python3 tools/ifft_op.py 1024 4 1 100 || exit 2
bash tools/profile.sh r06i_ifft_bc ifft_bc python3 tools/ifft_op.py 1024 4 4 50 || exit 3
bash tools/profile.sh r06i_op4k op4k python3 tools/ifft_op.py 4096 4 1 12 || exit 4
bash tools/profile.sh r06i_update update_loop python3 bench.py --only-update-loop --steps 200 --warmup 20 || exit 5
bash tools/profile.sh r06i_cfg5 cfg5 $B --config cfg5 --steps 30 --warmup 5 || exit 6
bash tools/profile.sh r06i_cfg4 cfg4 $B --config cfg4 --steps 30 --warmup 5 || exit 7
echo session done
