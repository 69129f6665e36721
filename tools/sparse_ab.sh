#!/bin/bash
# On the GPU box: sparse-row variant libraries A/B on configs[4]'s scenario at 1M peers (loss until 40, Failed
# drops not counted), 120 rounds each, twice, alternating.  tools/sparse_ab.sh OUTDIR variant...
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    KB_LIB_PATH=kaboodle_amd/variants/$v.so timeout -k 10 200 python3 tools/sparse_big.py --nodes 1048576 --rounds 120 \
      --fault-end 40 --print-every 40 --fp-every 1000 --check-rows 0 --out $OUT/$v.$rep.json > $OUT/$v.$rep.log 2>&1 || { tail -5 $OUT/$v.$rep.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$rep.json')); print('$v.$rep', d['gpu_round_ms_mean'], d['kernels_ms_per_round']['k_sp_handle'])"
  done
done
