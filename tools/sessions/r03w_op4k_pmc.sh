#!/bin/bash
# rocprofv3 of the default operator at 4 x 4096^2 x 4 planes (tools/ifft_op.py): kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE in separate passes, then the L2 -> memory write request sizes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/prof_r03w_op4k
mkdir -p $OUT
PROG="python3 tools/ifft_op.py 4096 4 1 10"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $PROG > $OUT/trace.log 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $PROG > $OUT/fetch.log 2>&1 || exit 12
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $PROG > $OUT/write.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/wrreq -o run -- $PROG > $OUT/wrreq.log 2>&1 || echo "wrreq pass failed"
echo done
