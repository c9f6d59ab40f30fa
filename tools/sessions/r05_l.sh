#!/bin/bash
# Round 5, session l: cfg4 with smaller unit chunks, where a chunk's re-read set plus DISP fits the cache and
# pass BQ's DC form applies (OCEAN_CHUNK_MIB 96 / 64), against the default 192 MiB chunks.
set -o pipefail
OUT=gpurun_out/r05_l; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for c in 192 96 64 128; do
    OCEAN_CHUNK_MIB=$c timeout -k 10 300 python bench.py --config cfg4 --steps 100 --warmup 20 --no-cpu-baseline --no-ifft-stage \
      --no-beyond-cache --no-update-loop > $OUT/c$c.json 2> $OUT/c$c.err || exit 3
    echo "$r chunk $c $(python -c "import json;d=json.load(open('$OUT/c$c.json'));print(d['value'],d['kernels_us'])")"
  done
done
echo session done
