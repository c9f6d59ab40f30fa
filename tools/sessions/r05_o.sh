#!/bin/bash
# Round 5, session o: the 4096 operator's row launch with an even item count per workgroup (build r4: four row workgroups per CU, compact twiddles; was: 683 workgroups x 6
# row pairs, build reven) against the persistent grid (768 x 5.33).
set -o pipefail
OUT=gpurun_out/r05_o; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in base r4; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op_$v.json 2>> $OUT/op.err || exit 3
    echo "$r $v $(python3 -c "import json;d=json.load(open('$OUT/op_$v.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'],d['rows_us'],d['cols_us'])")"
  done
done
echo session done
