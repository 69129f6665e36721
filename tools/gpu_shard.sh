#!/bin/bash
# usage: tools/gpu_shard.sh <tag> — the sharded-path GPU tests first, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-shard}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "sharded or rccl" > $OUT/pytest_shard.log 2>&1
rc=$?; tail -25 $OUT/pytest_shard.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; exit $rc
