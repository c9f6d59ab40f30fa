#!/bin/bash
# A3P variants on the cfg5 8-GPU parity shard; the chunked operator at cfg4's shape; rocprofv3 of the
# beyond-cache operator (kernel trace + FETCH / WRITE passes) -> gpurun_out/r03c.
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
bash tools/ab_shard.sh "base p0w0 p0w4 p1w4" cfg5 8 2 > $O/ab_a3p.txt 2>&1 || { cat $O/ab_a3p.txt; exit 1; }
for mib in 128 256 512; do
  OCEAN_OP_CHUNK_MIB=$mib timeout -k 10 120 python tools/ifft_op.py 512 4 32 20 >> $O/ifft_op.jsonl 2>>$O/ifft_op.err || exit 4
done
timeout -k 10 120 python tools/ifft_op.py 1024 4 4 30 >> $O/ifft_op.jsonl 2>>$O/ifft_op.err || exit 5
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bc/trace -o run -- python3 tools/ifft_op.py 1024 4 4 30 > $O/bc_trace.log 2>&1 || exit 8
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/bc/fetch -o run -- python3 tools/ifft_op.py 1024 4 4 30 > $O/bc_fetch.log 2>&1 || exit 9
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/bc/write -o run -- python3 tools/ifft_op.py 1024 4 4 30 > $O/bc_write.log 2>&1 || exit 10
echo done
