#!/bin/bash
# Round 6, session f: mip levels 1..3 fused into pass BQ (OCEAN_F_MIPS, three-plane frame): the mip / frame
# parity tests, then the update loop against the unfused build (liboceanhip_nofuse.so), alternating.
set -o pipefail
OUT=gpurun_out/r06_f; mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/ocean-simulation_amd/ocean_hip
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "mip or frames_vs_oracle or water_body or cfg4_shape or chunked" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do
  for v in base nofuse; do
    lib=$L/liboceanhip.so; [ $v != base ] && lib=$L/liboceanhip_$v.so
    OCEAN_HIP_LIB=$lib timeout -k 10 200 python bench.py --only-update-loop --steps 300 --warmup 20 > $OUT/ul_$v.json 2> $OUT/ul_$v.err || { tail $OUT/ul_$v.err; exit 2; }
    python -c "import json;d=json.load(open('$OUT/ul_$v.json'));s=d['step_with_mips'];print('$r $v', 'step+mips', s['frames_per_s'], s['kernel_us'], 'height', d['height']['frames_per_s'], d['height']['kernel_us_in_loop'], 'rgba', d['rgba']['frames_per_s'])"
  done
done
echo session done
