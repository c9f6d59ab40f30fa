#!/bin/bash
# Round 4 closing run of the final tree: the GPU test suite + smoke, then the default bench line
set -o pipefail
OUT=gpurun_out/r04_final2; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/sessions/r04_tests.sh r04_final2 || exit 1
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 2; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['kernels_us'],d['roofline']['frac'],d['update_loop']['frames_per_s'])"
echo session done
