#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python tests/parity.py > gpurun_out/parity1.log 2>&1
rc=$?
echo "parity rc=$rc"
tail -20 gpurun_out/parity1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python tools/quick_perf.py 65536 10 > gpurun_out/perf1.log 2>&1
echo "perf rc=$?"
cat gpurun_out/perf1.log
