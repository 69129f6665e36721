#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python tests/parity.py > gpurun_out/parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -14 gpurun_out/parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_prof.sh ${1:-prof2} 65536 10
