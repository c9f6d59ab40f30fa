#!/bin/bash
# Round 4 session 7: the 4096 operator with nontemporal plane loads in k_rowsf (opnt1),
# nontemporal stores in k_colsf (opnt2), both (opnt3): parity, then alternating timing (tools/ifft_op.py)
set -o pipefail
OUT=gpurun_out/r04_ab7; mkdir -p $OUT
export TMPDIR=/tmp
for v in opnt1 opnt2 opnt3; do
  OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -k "operator_large" -q --maxfail=2 --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
  for v in base opnt1 opnt2 opnt3; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so; [ $v != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    o=$(OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 200 python tools/ifft_op.py 4096 4 1 12) || exit 5
    echo "$r $v $o"
  done
done | tee $OUT/ab_op4k.txt
echo session done
