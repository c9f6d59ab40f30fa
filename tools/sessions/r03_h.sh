#!/bin/bash
# cfg5 8-GPU parity shard: column-pass bands per unit (C1 + C2 re-reading from the Infinity Cache).
set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
for r in 1 2; do for b in 1 2 4; do
  OCEAN_C4_BANDS=$b timeout -k 10 200 python tools/shard_bench.py --config cfg5 --worlds 8 --steps 50 > $O/b$b.json 2>/dev/null || exit 2
  echo "$r bands=$b $(python -c "
import json;d=json.load(open('$O/b$b.json'))
print(d['projected_frames_per_s'], [(s['ms_per_frame'], s['pass_a_ms'], s['pass_b_ms']) for s in d['shards'].values()])")"
done; done
