#!/bin/bash
# Round 5: cfg4's unit chunk (OCEAN_CHUNK_MIB) re-swept with pass BQ's XCD-grouped tile order.
set -o pipefail
OUT=gpurun_out/r05_bh; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for c in 192 128 256 384 96; do
    OCEAN_CHUNK_MIB=$c timeout -k 10 300 python bench.py --config cfg4 --steps 300 --warmup 20 --no-cpu-baseline \
      --no-ifft-stage --no-beyond-cache --no-update-loop > $OUT/b.json 2> $OUT/b.err || exit 3
    echo "$r chunk $c $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'],d['kernels_us'])")"
  done
done
echo session done
