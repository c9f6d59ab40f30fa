#!/bin/bash
# Round 6, session mips: A/B of the mips kernels on cfg3's Update loop.  r06_mips: 64x64 blocks, nontemporal loads / stores;
# r06_mips2: TURB from the foam state (f1), nontemporal DERIV loads (n1); r06_mips3: the chain tails fused into the
# block kernel (base) against the separate tail kernel (sep).  Each variant first runs the mip /
# sampling parity tests, then bench.py's update_loop (other legs off), interleaved over rounds.
set -o pipefail
OUT=gpurun_out/r06_mips3; mkdir -p $OUT
V="sep base"
lib() { [ "$1" = base ] && echo $PWD/ocean-simulation_amd/ocean_hip/liboceanhip.so || echo $PWD/ocean-simulation_amd/ocean_hip/liboceanhip_$1.so; }
for v in $V; do
  OCEAN_HIP_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sample.py -x -q \
    --timeout 120 --timeout-method thread -k "mip or sample" > $OUT/tests_$v.log 2>&1 || { tail -20 $OUT/tests_$v.log; exit 1; }
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
      u["step_with_mips"]["kernel_us"], "height_fps", u["height"]["frames_per_s"], u["height"]["kernel_us_in_loop"])
PY
  done
done
echo session done
