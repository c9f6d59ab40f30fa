#!/bin/bash
# Pass AQ intermediate stores through a scalar unit base + 32-bit lane offsets (default) against 64-bit
# addresses (OCEAN_AQ_WST=0 build): A/B interleaved on cfg3 and cfg4, then the parity tests of the frame
set -o pipefail
O=gpurun_out/r03wst; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frames or cfg4 or large_time or three_plane" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_lib.sh cfg3 "base wst0" 500 3 > $O/ab_cfg3.txt 2>&1 || exit 3
bash tools/ab_lib.sh cfg4 "base wst0" 50 3 > $O/ab_cfg4.txt 2>&1 || exit 4
cat $O/ab_cfg3.txt $O/ab_cfg4.txt
