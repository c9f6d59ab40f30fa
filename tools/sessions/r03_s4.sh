#!/bin/bash
# Pass A3PP on 1024 lanes with 32-bit store offsets: parity tests, then A/B pair 3 / 4 / 0 on the cfg5 8-GPU shard.
set -o pipefail
O=gpurun_out/r03s4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "column_parity" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest.log
for r in 1 2; do for p in 4 3 0; do
  OCEAN_A3P_PAIR=$p timeout -k 10 200 python tools/shard_bench.py --config cfg5 --worlds 8 --steps 50 > $O/p$p.json 2>/dev/null || exit 2
  echo "$r pair=$p $(python -c "
import json;d=json.load(open('$O/p$p.json'))
print(d['projected_frames_per_s'], [(s['ms_per_frame'], s['pass_a_ms'], s['pass_b_ms']) for s in d['shards'].values()])")"
done; done
