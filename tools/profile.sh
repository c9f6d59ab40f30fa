#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root):
#   1) --kernel-trace --stats   (per-kernel durations; compare with bench.py's HIP-event numbers)
#   2) --pmc FETCH_SIZE         (separate pass: counters never share a pass with tracing domains)
#   3) --pmc WRITE_SIZE
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ARGS=${@:---steps 200 --warmup 20 --no-cpu-baseline --no-ifft-stage --no-beyond-cache}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit 13
echo done
