#!/bin/bash
# The chip ceilings bench.py quotes (roofline.writes, roofline.memory_shape): tools/wrbench, aqbench and
# bqbench (built in the build container: hipcc --offload-arch=gfx950 -O3 tools/<x>.hip -o tools/<x>),
# run on the GPU box from the repo root, plus the ceilings.json stamp bench._ceiling_dirs selects by.
# Usage: tools/ceilings.sh <out dir>   (then copy the directory under profiles/)
set -o pipefail
OUT=${1:?out dir}
mkdir -p $OUT
timeout -k 10 60 ./tools/wrbench > $OUT/wrbench.txt 2>&1 || exit 6
timeout -k 10 60 ./tools/aqbench > $OUT/aqbench.txt 2>&1 || exit 7
timeout -k 10 60 ./tools/bqbench > $OUT/bqbench.txt 2>&1 || exit 8
python3 tools/stamp.py --ceilings $OUT || exit 9
echo "ceilings -> $OUT"
