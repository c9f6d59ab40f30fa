#!/bin/bash
# Round 6, session e: WRITE_SIZE calibration of the 4096 operator column launch's store shape (tools/wrcal.hip),
# timing + two PMC passes.
set -o pipefail
OUT=gpurun_out/r06_e; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/wrcal > $OUT/wrcal.txt 2>&1 || { cat $OUT/wrcal.txt; exit 1; }
cat $OUT/wrcal.txt
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p1 -o run -- ./tools/wrcal > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 2; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/p2 -o run -- ./tools/wrcal > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 3; }
echo session done
