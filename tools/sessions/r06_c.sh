#!/bin/bash
# Round 6, session c: pass AQ with row y2 reversed (OCEAN_AQ_REV, no mirrored LDS put) against the product:
# cfg3 parity of the variant, SQ_LDS_BANK_CONFLICT of both, and an interleaved A/B (3 rounds).
set -o pipefail
OUT=gpurun_out/r06_c; mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/ocean-simulation_amd/ocean_hip
OCEAN_HIP_LIB=$L/liboceanhip_rev.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "frames_vs_oracle and 1024 or pointwise or three_plane or mirror_pair or column_band or tiles_are" > $OUT/pytest_rev.log 2>&1 || { tail -20 $OUT/pytest_rev.log; exit 1; }
tail -2 $OUT/pytest_rev.log
for v in base rev; do
  lib=$L/liboceanhip.so; [ $v != base ] && lib=$L/liboceanhip_$v.so
  OCEAN_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq_$v -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-ifft-stage --no-beyond-cache --no-update-loop > $OUT/sq_$v.log 2>&1 || { tail -5 $OUT/sq_$v.log; exit 2; }
done
bash tools/ab_lib.sh cfg3 "base rev" 300 3 || exit 3
echo session done
