#!/bin/bash
# Round-2 baseline on the GPU box: gpu tests, bench, rocprofv3 stats of the fused frame and the operator IFFT.
set -o pipefail
O=gpurun_out/r02a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 2
cat $O/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/frame -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ifft-stage > $O/frame.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ifft -o run -- python3 tools/ifft_bench.py 200 > $O/ifft.log 2>&1 || exit 4
echo done
