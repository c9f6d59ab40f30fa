#!/bin/bash
# Round 4: the WaterBody facade keeps the landed readback in its pinned slot (no 16 MiB host copy per
# frame): facade test, the readback probe and the update loop
set -o pipefail
OUT=gpurun_out/r04_zc; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -k "water_body or host" -q --timeout 250 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python tools/readback_probe.py 200 > $OUT/readback_probe.json 2> $OUT/readback_probe.err || exit 2
cat $OUT/readback_probe.json
timeout -k 10 300 python bench.py --only-update-loop --steps 400 --warmup 20 > $OUT/update_loop.json 2> $OUT/update_loop.err || exit 3
cat $OUT/update_loop.json | cut -c1-400
echo session done
