#!/bin/bash
# Round 6, session g: the mips tail built in LDS: mip / sampling parity, then the update loop (mip kernel time).
set -o pipefail
OUT=gpurun_out/r06_g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sample.py -k "mip or sample or water_body" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --only-update-loop --steps 300 --warmup 20 > $OUT/ul.json 2> $OUT/ul.err || { tail $OUT/ul.err; exit 2; }
  python -c "import json;d=json.load(open('$OUT/ul.json'));s=d['step_with_mips'];print('$r', 'step+mips', s['frames_per_s'], s['kernel_us'], 'height', d['height']['frames_per_s'], 'rgba', d['rgba']['frames_per_s'])"
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --only-update-loop --steps 200 --warmup 20 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 3; }
grep -i mips $OUT/trace/run_kernel_stats.csv | cut -c1-200
echo session done
