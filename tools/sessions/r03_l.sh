#!/bin/bash
# AQ share A/B (cfg3, cfg4); frame graph: bit-identity tests + cfg2 / cfg3 A/B.
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "GRAPH" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest.log
bash tools/ab_env_lib.sh cfg2 "base:- base:OCEAN_GRAPH=1" 2000 3 || exit 2
bash tools/ab_env_lib.sh cfg3 "base:- base:OCEAN_GRAPH=1" 300 2 || exit 3
bash tools/ab_lib.sh cfg3 "base share" 300 3 || exit 4
bash tools/ab_lib.sh cfg4 "base share" 50 2 || exit 5
