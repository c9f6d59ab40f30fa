#!/bin/bash
# Pass A3PP (mirror-pair parity rows): parity shards vs oracle under it, then A/B on the cfg5 8-GPU shard.
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
for p in 2 1; do
  OCEAN_A3P_PAIR=$p timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "column_parity_shards" > $O/pytest_$p.log 2>&1 || { tail -30 $O/pytest_$p.log; exit 1; }
  grep -E "PASSED|FAILED" $O/pytest_$p.log
done
for r in 1 2; do for p in 0 1 2; do
  OCEAN_A3P_PAIR=$p timeout -k 10 200 python tools/shard_bench.py --config cfg5 --worlds 8 --steps 50 > $O/p$p.json 2>/dev/null || exit 2
  echo "$r pair=$p $(python -c "
import json;d=json.load(open('$O/p$p.json'))
print(d['projected_frames_per_s'], [(s['ms_per_frame'], s['pass_a_ms'], s['pass_b_ms']) for s in d['shards'].values()])")"
done; done
