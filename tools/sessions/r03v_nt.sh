#!/bin/bash
# A/B at 4096: grouped 4-column tiles (XQ=1) vs nontemporal column loads (XQ=6) vs 32-column groups (XQ=7).
set -e
out=gpurun_out/r03v
mkdir -p $out
: > $out/nt.txt
for r in 1 2; do
  for x in 1 6 7; do
    echo "xq=$x" >> $out/nt.txt
    OCEAN_COLS2_XQ=$x timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 10 >> $out/nt.txt
  done
done
cat $out/nt.txt
