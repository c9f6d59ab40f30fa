#!/bin/bash
# A/B at 4096: default grouped 4-column tiles (XQ=1) vs 8-column two-half tiles (XQ=4: G = 2, XQ=5: G = 1).
set -e
out=gpurun_out/r03v
mkdir -p $out
: > $out/h.txt
for r in 1 2; do
  for x in 1 4 5; do
    echo "xq=$x" >> $out/h.txt
    OCEAN_COLS2_XQ=$x timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 10 >> $out/h.txt
  done
done
OCEAN_COLS2_XQ=4 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "large_vs_numpy" >> $out/h.txt 2>&1
cat $out/h.txt
