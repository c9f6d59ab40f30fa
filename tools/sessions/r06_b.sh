#!/bin/bash
# Round 6, session b: (1) SQ_LDS_BANK_CONFLICT per LDS pattern of pass AQ (tools/ldsbench.hip);
# (2) the pointwise record after the correctly rounded init (tools/pointwise.py, all three configs, and
# tools/pointwise_stages.py); (3) the parity tests the init change touches.
set -o pipefail
OUT=gpurun_out/r06_b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ldsbench > $OUT/ldsbench.txt 2>&1 || { cat $OUT/ldsbench.txt; exit 1; }
cat $OUT/ldsbench.txt
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/lds -o run -- ./tools/ldsbench > $OUT/lds.log 2>&1 || { tail -5 $OUT/lds.log; exit 2; }
timeout -k 10 600 python -u tools/pointwise.py $OUT/pointwise.json > $OUT/pointwise.log 2>&1 || { tail -5 $OUT/pointwise.log; exit 3; }
cat $OUT/pointwise.log
timeout -k 10 300 python -u tools/pointwise_stages.py base $OUT/stages_base.json cfg2,cfg3 > $OUT/stages.log 2>&1 || { tail -5 $OUT/stages.log; exit 4; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "init_spectrum or golden or pointwise or frames_vs_oracle or evolve_operator" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 5; }
tail -3 $OUT/pytest.log
echo session done
