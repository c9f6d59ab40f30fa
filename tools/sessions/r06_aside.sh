#!/bin/bash
# Round 6, session aside: the height readback's extraction on the copy stream beside the step's mips (base)
# against the extraction on the ctx stream after them (noaside: OCEAN_HEIGHT_ASIDE=0).  Readback / facade
# parity tests per variant, then bench.py's update_loop three times per variant, interleaved.
set -o pipefail
OUT=gpurun_out/r06_aside; mkdir -p $OUT
V="noaside base"
lib() { [ "$1" = base ] && echo $PWD/ocean-simulation_amd/ocean_hip/liboceanhip.so || echo $PWD/ocean-simulation_amd/ocean_hip/liboceanhip_$1.so; }
for v in $V; do
  OCEAN_HIP_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py tests/test_gpu_state.py -x -q \
    --timeout 120 --timeout-method thread -k "readback or height or facade or host or state or caller" > $OUT/tests_$v.log 2>&1 || { tail -20 $OUT/tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $OUT/tests_$v.log)"
done
for r in 1 2 3; do
  for v in $V; do
    OCEAN_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-ifft-stage \
      --no-beyond-cache > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail -20 $OUT/b_${v}_$r.err; exit 2; }
    python - $OUT/b_${v}_$r.json $v $r <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.strip().startswith("{")][-1]
u = d["update_loop"]
print(sys.argv[3], sys.argv[2], "frame", d["value"], "mips_loop_fps", u["step_with_mips"]["frames_per_s"],
      "height_fps", u["height"]["frames_per_s"], u["height"]["kernel_us_in_loop"], "rgba_fps", u["rgba"]["frames_per_s"])
PY
  done
done
echo session done
