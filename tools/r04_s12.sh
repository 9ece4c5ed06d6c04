#!/bin/bash
# round-4 GPU session 12: the whole GPU suite and smoke() on the round-4 build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/s12_tests.log 2>&1
rc=$?; tail -5 gpurun_out/s12_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
