#!/bin/bash
# Mirror-factor sharing: parity + variant-vs-oracle tests, then A/B of A3P (cfg5 8-GPU shard), AQ vs the
# one-row pass at cfg3, A3Q share at cfg5.
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "parity or variants_vs_oracle" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest.log | grep -E "parity_|variants"
for r in 1 2; do for sh in 1 0; do
  OCEAN_A3P_SHARE=$sh timeout -k 10 200 python tools/shard_bench.py --config cfg5 --worlds 8 --steps 50 > $O/s$sh.json 2>/dev/null || exit 2
  echo "$r share=$sh $(python -c "
import json;d=json.load(open('$O/s$sh.json'))
print(d['projected_frames_per_s'], [(s['ms_per_frame'], s['pass_a_ms'], s['pass_b_ms']) for s in d['shards'].values()])")"
done; done
bash tools/r03_g.sh || exit 3
