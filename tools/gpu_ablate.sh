#!/bin/bash
# usage: tools/gpu_ablate.sh <tag>   timing experiments on the benched workload: the row pass with parts skipped
# (KB_DEV bits, results are wrong by construction: 1 A3 first chunk only, 2 no Failed group, 4 no Join group,
# 8 no Join-stamp read-back sync) -> gpurun_out/<tag>/ablate.txt (k_rowpass ms per round for each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ablate}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for dev in 0 1 2 4 6; do
  KB_DEV=$dev timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-conv --no-modes --no-replay \
    > $OUT/dev$dev.json 2> $OUT/dev$dev.err || { tail -5 $OUT/dev$dev.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/dev$dev.json'));k=d['kernels'];print('KB_DEV=$dev', 'round', d['round_gpu_ms'], ' '.join(f'{n} {v[\"ms_per_round\"]}' for n,v in k.items() if n!='gaps'))" | tee -a $OUT/ablate.txt
done
