#!/bin/bash
# Default operator at 2048 / 4096 (in-place rows + XCD-grouped whole-column tiles): parity + timing + rocprofv3.
set -e
out=gpurun_out/r03x
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "operator" > $out/op_tests.txt 2>&1
: > $out/op_default.txt
for a in "4096 1 1 30" "4096 4 1 10" "2048 1 1 30" "2048 4 1 20" "1024 4 4 50"; do
  echo "$a" >> $out/op_default.txt
  timeout -k 10 120 python3 tools/ifft_op.py $a >> $out/op_default.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof4k -o op -- python3 tools/ifft_op.py 4096 4 1 10 > /dev/null
tail -3 $out/op_tests.txt
cat $out/op_default.txt
