#!/bin/bash
# Runs named GPU steps in order on the gpurun box, each under its own time limit.
# A step that exits 0 or 1 (test failures) lets the session continue; any other exit code
# (fault, abort, segfault, timeout) ends the session immediately -- nothing else touches the GPU.
# usage: tools/gpu_session.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    echo "== $name ($secs s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc ($(( $(date +%s) - start )) s)"
    tail -n 15 "gpurun_out/$name.log"
    case $rc in
        0|1) ;;
        *) echo "== STOP: $name exited $rc"; exit $rc ;;
    esac
done
