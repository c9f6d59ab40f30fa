#!/bin/bash
# A/B: operator at 2048 / 4096, four-step (default) vs single-pass column tiles grouped on one XCD
# (OCEAN_COLS2_XQ: 1 = 4 columns x 4, 2 = 2 columns x 8, 3 = 8 columns x 2 at 2048), chunk sizes.
set -e
out=gpurun_out/r03x
mkdir -p $out
: > $out/xq2.txt
for n in 4096 2048; do
  for v in "OCEAN_COLS2_XQ=1" "OCEAN_COLS2_XQ=2" "OCEAN_COLS2_XQ=3" "OCEAN_COLS2_XQ=1 OCEAN_OP_CHUNK_MIB=128" "OCEAN_COLS2_XQ=1 OCEAN_OP_CHUNK_MIB=512"; do
    if [ $n = 4096 ] && [ "$v" = "OCEAN_COLS2_XQ=3" ]; then continue; fi
    echo "n=$n OCEAN_OP_FOUR_STEP=0 $v" >> $out/xq2.txt
    env OCEAN_OP_FOUR_STEP=0 $v timeout -k 10 120 python3 tools/ifft_op.py $n 1 1 30 >> $out/xq2.txt
  done
done
for v in 1 2; do
  echo "n=4096 C=4 OCEAN_OP_FOUR_STEP=0 OCEAN_COLS2_XQ=$v" >> $out/xq2.txt
  OCEAN_OP_FOUR_STEP=0 OCEAN_COLS2_XQ=$v timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 10 >> $out/xq2.txt
done
OCEAN_OP_FOUR_STEP=0 OCEAN_COLS2_XQ=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "large_vs_numpy or 2048_vs_oracle" >> $out/xq2.txt 2>&1
OCEAN_OP_FOUR_STEP=0 OCEAN_COLS2_XQ=3 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "2048_vs_oracle" >> $out/xq2.txt 2>&1
cat $out/xq2.txt
