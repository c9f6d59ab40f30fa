#!/bin/bash
# Folded operator: chunk size sweep (out-of-place rows + columns double the chunk's cache footprint)
set -o pipefail
O=gpurun_out/r03fold2; mkdir -p $O
for r in 1 2; do
for c in 64 128; do
  OCEAN_OP_FOLD=1 OCEAN_OP_CHUNK_MIB=$c timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_fold_c$c.r$r.json 2>> $O/err.log || exit 3
  OCEAN_OP_FOLD=1 OCEAN_FOLD_COLS=16 OCEAN_OP_CHUNK_MIB=$c timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_fold16_c$c.r$r.json 2>> $O/err.log || exit 3
  OCEAN_OP_FOLD=1 OCEAN_OP_CHUNK_MIB=$c timeout -k 10 120 python3 tools/ifft_op.py 2048 4 1 30 > $O/op2k_fold_c$c.r$r.json 2>> $O/err.log || exit 4
done
OCEAN_OP_FOLD=0 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_grouped.r$r.json 2>> $O/err.log || exit 5
done
for f in $O/op*.json; do echo "$f $(cat $f)"; done
