#!/bin/bash
# GPU test suite + smoke on one box (round 4); results under gpurun_out/$1
set -o pipefail
OUT=gpurun_out/${1:-r04_tests}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 5
tail -2 $OUT/smoke.log
