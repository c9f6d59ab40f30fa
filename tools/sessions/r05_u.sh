#!/bin/bash
# Round 5, session u: the in-place 4096 operator with nontemporal row loads (ntl), nontemporal column
# stores (nts) or both (ntb), against the product: parity of the operator tests on ntb, then A/B.
set -o pipefail
OUT=gpurun_out/r05_u; mkdir -p $OUT
export TMPDIR=/tmp
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_ntb.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "operator_large" > $OUT/pytest_ntb.log 2>&1 || { tail -30 $OUT/pytest_ntb.log; exit 1; }
tail -1 $OUT/pytest_ntb.log
for r in 1 2 3; do
  for v in base ntl nts ntb; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op_$v.json 2>> $OUT/op.err || exit 3
    echo "$r $v $(python3 -c "import json;d=json.load(open('$OUT/op_$v.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'],d['rows_us'],d['cols_us'])")"
  done
done
echo session done
