#!/bin/bash
# Column-parity shards + chunked operator: targeted GPU tests, operator sweeps, cfg5 shard times.
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "parity or split_ocean or operator or four_step or large_n" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -cE "PASSED" $O/pytest.log
for mib in 64 128 192 256 100000; do
  OCEAN_OP_CHUNK_MIB=$mib timeout -k 10 120 python tools/ifft_op.py 1024 4 4 30 >> $O/ifft_op.jsonl 2>>$O/ifft_op.err || exit 4
done
for mib in 128 256; do
  OCEAN_OP_CHUNK_MIB=$mib timeout -k 10 120 python tools/ifft_op.py 4096 4 1 10 >> $O/ifft_op.jsonl 2>>$O/ifft_op.err || exit 5
done
timeout -k 10 300 python tools/shard_bench.py --config cfg5 --worlds 1,8 --steps 50 > $O/shard_cfg5.jsonl 2> $O/shard.err || exit 6
timeout -k 10 300 python tools/shard_bench.py --config cfg5 --worlds 8 --steps 50 --no-interleave >> $O/shard_cfg5.jsonl 2>> $O/shard.err || exit 7
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/op4k -o run -- python3 tools/ifft_op.py 4096 4 1 10 > $O/op4k.log 2>&1 || exit 8
echo done
