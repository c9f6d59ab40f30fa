#!/bin/bash
# Round 5: the N <= 2048 operator column launch with more XCD grouping (G 8-column halves of G/2
# 16-column tiles on one XCD; the product pairs halves, G = 2).
set -o pipefail
OUT=gpurun_out/r05_bf; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for shape in "1024 4 1 100" "1024 4 4 50" "2048 4 1 30"; do
    for v in base opg4 opg8 opg16; do
      lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
      [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
      OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py $shape > $OUT/op.json 2>> $OUT/op.err || exit 3
      echo "$r $v [$shape] $(python3 -c "import json;d=json.load(open('$OUT/op.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'])")"
    done
  done
done
echo session done
