#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python tests/parity.py > gpurun_out/parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -14 gpurun_out/parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for ab in 0 1 2 3; do
  KB_ABLATE=$ab timeout -k 10 200 python tools/quick_perf.py 65536 10 > gpurun_out/perf_ab$ab.log 2>&1 || exit 1
  echo "ablate=$ab: $(grep N= gpurun_out/perf_ab$ab.log)"
done
bash tools/gpu_prof.sh ${1:-prof4} 65536 10
