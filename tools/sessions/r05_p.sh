#!/bin/bash
# Round 5, session p: the 4096 operator's row launch with four workgroups per CU (build r4: <= 128 VGPRs,
# twiddle rows r = 1, 2 only): parity of the operator tests, then A/B against the product.
set -o pipefail
OUT=gpurun_out/r05_p; mkdir -p $OUT
export TMPDIR=/tmp
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_r4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "operator_large" > $OUT/pytest_r4.log 2>&1 || { tail -30 $OUT/pytest_r4.log; exit 1; }
tail -1 $OUT/pytest_r4.log
for r in 1 2 3; do
  for v in base r4; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op_$v.json 2>> $OUT/op.err || exit 3
    echo "$r $v $(python3 -c "import json;d=json.load(open('$OUT/op_$v.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'],d['rows_us'],d['cols_us'])")"
  done
done

bash tools/ab_lib.sh cfg2 "base b8pl" 2000 3 > $OUT/ab_cfg2.txt 2>&1 || { tail $OUT/ab_cfg2.txt; exit 4; }
cat $OUT/ab_cfg2.txt
echo session done
