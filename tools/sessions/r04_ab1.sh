#!/bin/bash
# Round 4 session 1: A/B of pass AQ pass-1 variants (cfg3, cfg4), the default bench line, operator profiles
set -o pipefail
OUT=gpurun_out/r04_ab1; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/ab_lib.sh cfg3 "base aqx1 aqx2 aqx3" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base aqx1" 100 2 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 5; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['kernels_us'],d['update_loop'])"
bash tools/profile.sh r04a_ifft ifft python3 tools/ifft_op.py 1024 4 1 100 || exit 6
bash tools/profile.sh r04a_ifft_bc ifft_bc python3 tools/ifft_op.py 1024 4 4 50 || exit 7
bash tools/profile.sh r04a_op4k op4k python3 tools/ifft_op.py 4096 4 1 12 || exit 8
echo session done
