#!/bin/bash
# Operator chunk sizes with the frame's data in the planes (not zeros).
set -o pipefail
for mib in 128 192 256 320 384; do
  echo "bc $mib $(OCEAN_OP_CHUNK_MIB=$mib timeout -k 10 120 python tools/ifft_op.py 1024 4 4 50)"
done
for mib in 128 256; do
  echo "cfg4shape $mib $(OCEAN_OP_CHUNK_MIB=$mib timeout -k 10 120 python tools/ifft_op.py 512 4 32 20)"
done
echo "4096 default $(timeout -k 10 120 python tools/ifft_op.py 4096 4 1 10)"
echo "cfg3 $(timeout -k 10 120 python tools/ifft_op.py 1024 4 1 100)"
