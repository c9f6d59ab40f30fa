#!/bin/bash
# rocprofv3 passes of one workload (run on the GPU box from the repo root):
#   1) --kernel-trace --stats   (per-kernel durations; compare with bench.py's HIP-event numbers)
#   2) --pmc FETCH_SIZE         (separate pass: counters never share a pass with tracing domains)
#   3) --pmc WRITE_SIZE
# plus a stamp (tools/stamp.py: config, library and source sha256, UTC time) of what ran.
# Usage: tools/profile.sh <tag> <config> [program args...]   (default: the cfg3 bench frame)
# Then, in the build container: python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>
set -o pipefail
TAG=${1:?tag}; shift
CONFIG=${1:?config}; shift
CMD=("$@")
if [ ${#CMD[@]} -eq 0 ]; then
    CMD=(python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ifft-stage --no-beyond-cache --no-update-loop)
fi
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
python3 tools/stamp.py $OUT/stamp.json "$CONFIG" "${CMD[@]}" || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- "${CMD[@]}" > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- "${CMD[@]}" > $OUT/fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- "${CMD[@]}" > $OUT/write.log 2>&1 || exit 13
echo "profile $TAG ($CONFIG) done"
