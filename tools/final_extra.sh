#!/bin/bash
# On the GPU box, with the round's final library: SQ counter passes of the benched workload and the configs[4]
# bench-style lines at 4,194,304 peers (sparse rows): the stated scenario (Failed-list drops not counted, the
# default), the same with them counted (k_sp_bfail_sf, VALU-bound), and the long-run mode (loss until round 40).
# tools/final_extra.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-extra}; OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_sq.sh $TAG/sq sim > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
timeout -k 10 300 python -u tools/sparse_big.py --nodes 4194304 --rounds 48 --print-every 1 --fp-every 8 \
  --out $OUT/sparse_4m_bench.json > $OUT/sparse_4m_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sparse_big.py --nodes 4194304 --rounds 24 --print-every 1 --fp-every 8 \
  --count-sf-failed-drops --out $OUT/sparse_4m_bench_counted.json > $OUT/sparse_4m_bench_counted.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/sparse_big.py --nodes 4194304 --rounds 96 --fault-end 40 \
  --print-every 1 --fp-every 8 --out $OUT/sparse_4m_bench_nosf.json > $OUT/sparse_4m_bench_nosf.log 2>&1 || exit $?
python3 -c "
import json
for f in ('sparse_4m_bench', 'sparse_4m_bench_counted', 'sparse_4m_bench_nosf'):
    d = json.load(open('$OUT/' + f + '.json')); print(f, json.dumps(d['bench_line']))"
