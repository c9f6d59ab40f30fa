#!/bin/bash
# Round 5, session y: the N <= 2048 operator column launch (k_cols2) with nontemporal stores (c2nt; c2nt3: three quarters of the stores by output row)
# against the product, on cfg3's cache-resident planes, 4x beyond the cache, and 4 x 2048^2.
set -o pipefail
OUT=gpurun_out/r05_y; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for shape in "1024 4 1 100" "1024 4 4 50" "2048 4 1 30"; do
    for v in base c2nt3; do
      lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
      [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
      OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py $shape > $OUT/op.json 2>> $OUT/op.err || exit 3
      echo "$r $v [$shape] $(python3 -c "import json;d=json.load(open('$OUT/op.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'])")"
    done
  done
done
echo session done
