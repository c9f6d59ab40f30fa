#!/bin/bash
# GPU test run on the box: -m gpu tests, one process, per-test timeout (TESTS: files, K: -k expression).
set -o pipefail
O=gpurun_out/${TAG:-r02t}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -15
exit $rc
