#!/bin/bash
# Round 5: the in-place 4096 column launch with nontemporal loads (cl), and with nontemporal loads and
# default-policy stores (cld), against the product.
set -o pipefail
OUT=gpurun_out/r05_ab_cl; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in base cl cld; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op_$v.json 2>> $OUT/op.err || exit 3
    echo "$r $v $(python3 -c "import json;d=json.load(open('$OUT/op_$v.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'],d['rows_us'],d['cols_us'])")"
  done
done
echo session done
