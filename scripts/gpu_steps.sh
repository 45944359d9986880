#!/bin/bash
# Runs GPU steps in order on the gpurun box; stops at the first step whose
# exit status is not 0/1 (fault, abort, segfault, timeout) -- nothing more
# touches the GPU after that.  Usage: scripts/gpu_steps.sh "name:secs:cmd" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping: $name exited $rc" | tee -a gpurun_out/steps.log
        exit $rc
    fi
done
