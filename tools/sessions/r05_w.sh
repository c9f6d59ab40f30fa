#!/bin/bash
# Round 5, session w: the library with the 4096 column launch's direct stores nontemporal -- the GPU
# suite + smoke, then the 4096 operator three times (tools/ifft_op.py).
set -o pipefail
OUT=gpurun_out/r05_w; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/sessions/r04_tests.sh r05_w || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op.json 2>> $OUT/op.err || exit 3
  echo "$r product $(python3 -c "import json;d=json.load(open('$OUT/op.json'));print(d['rows_frac'],d['cols_frac'],d['wall_frac'],d['rows_us'],d['cols_us'])")"
done
echo session done
