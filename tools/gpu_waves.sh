#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/waves
KB_DEBUG_WAVES=1 timeout -k 10 300 python tools/age_perf.py 65536 ${1:-300} 50 > gpurun_out/waves/age.log 2> gpurun_out/waves/waves.log
rc=$?
cat gpurun_out/waves/age.log
grep -E "round (20|270|290) " gpurun_out/waves/waves.log
exit $rc
