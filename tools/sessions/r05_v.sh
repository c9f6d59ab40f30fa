#!/bin/bash
# Round 5, session v: the in-place 4096 operator's column stores nontemporal -- all (nts), only the
# held half (ntsh), only the direct ones (ntsd) -- against the product; then nts over chunk sizes.
set -o pipefail
OUT=gpurun_out/r05_v; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # round variant [chunk MiB]
  local lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
  [ "$2" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$2.so
  OCEAN_OP_CHUNK_MIB=${3:-0} OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op_$2.json 2>> $OUT/op.err || exit 3
  echo "$1 $2 ${3:-auto} $(python3 -c "import json;d=json.load(open('$OUT/op_$2.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'],d['rows_us'],d['cols_us'])")"
}
for r in 1 2 3; do
  for v in base nts ntsh ntsd; do run $r $v; done
done
for c in 128 384 512; do run 1 nts $c; run 1 base $c; done
echo session done
