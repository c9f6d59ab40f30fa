#!/bin/bash
# Operator chunk sweep with freshly evolved planes before every call (tools/ifft_op.py).
set -e
out=gpurun_out/r03q
mkdir -p $out
: > $out/chunks.txt
for c in 128 192 256 320 384; do
  echo "chunk $c MiB 1024x4x4" >> $out/chunks.txt
  OCEAN_OP_CHUNK_MIB=$c timeout -k 10 120 python3 tools/ifft_op.py 1024 4 4 50 >> $out/chunks.txt
done
for c in 128 256; do
  echo "chunk $c MiB 512x4x32" >> $out/chunks.txt
  OCEAN_OP_CHUNK_MIB=$c timeout -k 10 120 python3 tools/ifft_op.py 512 4 32 50 >> $out/chunks.txt
done
echo "unchunked (chunk 4096 MiB) 1024x4x4" >> $out/chunks.txt
OCEAN_OP_CHUNK_MIB=4096 timeout -k 10 120 python3 tools/ifft_op.py 1024 4 4 50 >> $out/chunks.txt
cat $out/chunks.txt
