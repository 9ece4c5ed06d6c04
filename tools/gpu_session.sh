#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box; stops at the first step that
# times out, aborts or faults (exit >= 124), continues past ordinary failures.
# usage: tools/gpu_session.sh "<secs> <name> <cmd...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
    secs=${spec%% *}; rest=${spec#* }; name=${rest%% *}; cmd=${rest#* }
    echo "[session] $name (limit ${secs}s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "[session] $name rc=$rc"
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 124 ]; then
        echo "[session] stopping: $name ended with $rc"
        exit $rc
    fi
done
