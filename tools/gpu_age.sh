#!/bin/bash
# usage: tools/gpu_age.sh <tag> [rounds] — kernel trace of an aging 64K mesh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-age}; R=${2:-300}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/prof" -o run --output-format csv -- python3 tools/age_perf.py 65536 $R 25 > gpurun_out/$TAG/age.log 2>&1
rc=$?; cat gpurun_out/$TAG/age.log; exit $rc
