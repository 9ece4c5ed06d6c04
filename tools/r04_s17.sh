#!/bin/bash
# round-4 GPU session 17: the final build -- whole GPU suite + smoke, then
# the bench lines (tools/r04_s13.sh into gpurun_out/s17)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/s17_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s17_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
OUTDIR=s17 tools/r04_s13.sh
