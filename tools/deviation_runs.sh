#!/bin/bash
# A3's declared stamp window vs the exact-instant order (KB_VARIANT_EXACT_LRU) on the GPU: quiet rounds to full
# agreement of configs[2]'s workload (faults until round 25) in socket_faithful mode at 8K, 16K and 64K peers.
#   bash tools/deviation_runs.sh <outdir> [budget_s_64k]
set -o pipefail
out=${1:-gpurun_out/dev}; b64=${2:-600}
mkdir -p "$out"
for n in 8192 16384; do
  for lru in window exact; do
    timeout -k 10 400 python -u tools/converge.py --mode sock --nodes $n --lru $lru --cap-factor 4 --every 1024 \
      --out "$out/converge_sock_${n}_${lru}.json" > "$out/converge_sock_${n}_${lru}.log" 2>&1 || exit $?
    tail -1 "$out/converge_sock_${n}_${lru}.log" | cut -c1-300
  done
done
timeout -k 10 $((b64 + 60)) python -u tools/converge.py --mode sock --nodes 65536 --lru exact --cap-factor 2 --every 4096 \
  --budget-s $b64 --out "$out/converge_sock_65536_exact.json" > "$out/converge_sock_65536_exact.log" 2>&1 || exit $?
tail -1 "$out/converge_sock_65536_exact.log" | cut -c1-300
