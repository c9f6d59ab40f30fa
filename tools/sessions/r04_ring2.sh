#!/bin/bash
# Round 4: the facades with 4 readbacks in flight: facade tests, the probe and the bench's update loop
set -o pipefail
OUT=gpurun_out/r04_ring2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -k "water_body or host" -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 250 python tools/readback_probe.py 200 > $OUT/probe.json 2> $OUT/probe.err || exit 2
cat $OUT/probe.json
timeout -k 10 300 python bench.py --only-update-loop --steps 1000 --warmup 20 > $OUT/update_loop.json 2> $OUT/update_loop.err || exit 3
cut -c1-600 $OUT/update_loop.json
echo session done
