#!/bin/bash
# Round-3 first box call: -m gpu suite + smoke, then the operator IFFT beyond the Infinity Cache
# and the chip's HBM stream ceilings (tools/hbmbench.hip).
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
TAG=r03a bash tools/r02_tests.sh || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 60 ./tools/hbmbench 512 > $O/hbmbench.txt 2>&1 || exit 3
for s in "1024 4 1" "1024 4 4" "512 4 32" "2048 4 1" "4096 4 1"; do
  timeout -k 10 120 python tools/ifft_op.py $s 30 >> $O/ifft_op.jsonl 2>>$O/ifft_op.err || exit 4
done
echo done
