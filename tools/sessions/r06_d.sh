#!/bin/bash
# Round 6, session d: the ABI-4 library (height-only readback, pooled readback events, OCEAN_DISP_CACHED):
# the GPU suite + smoke, then the driver-shaped bench line with both update loops.
set -o pipefail
OUT=gpurun_out/r06_d; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/sessions/r04_tests.sh r06_d || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err || { tail $OUT/bench_drv.err; exit 2; }
python -c "import json;d=json.load(open('$OUT/bench_drv.json'));u=d['update_loop'];print('cfg3',d['value'],d['kernels_us'],d['roofline']['frac']);print('height',u['height']['frames_per_s'],u['height']['d2h'],'rgba',u['rgba']['frames_per_s'],u['rgba']['d2h'],'ratio',u['height_over_rgba'])"
echo session done
