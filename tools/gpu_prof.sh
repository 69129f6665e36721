#!/bin/bash
# usage: tools/gpu_prof.sh <tag> <N> <rounds>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-p}; N=${2:-65536}; R=${3:-10}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG" -o run --output-format csv -- python3 tools/quick_perf.py $N $R > gpurun_out/$TAG/stdout.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -5 gpurun_out/$TAG/stdout.log
find gpurun_out/$TAG -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -40
exit $rc
