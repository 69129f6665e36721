#!/bin/bash
# On the GPU box, with the round's final library: the configs[2] quiet tails bench.py attaches
# (tools/converge.py, lib_sha16-matched): the headline's sim_sender and socket_faithful with the exact-instant A3
# order (the bench default since round 6), and socket_faithful with the window order.
# tools/final_conv.sh <tag> -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-conv}; mkdir -p $OUT
timeout -k 10 330 python -u tools/converge.py --mode sock --nodes 65536 --cap-factor 4 --every 4096 \
  --out $OUT/converge_sock.json > $OUT/converge_sock.log 2>&1 || exit $?
timeout -k 10 450 python -u tools/converge.py --mode sim --nodes 65536 --lru exact --cap-factor 3 --every 4096 \
  --out $OUT/converge_sim_exact.json > $OUT/converge_sim_exact.log 2>&1 || exit $?
timeout -k 10 330 python -u tools/converge.py --mode sock --nodes 65536 --lru exact --cap-factor 4 --every 4096 \
  --out $OUT/converge_sock_exact.json > $OUT/converge_sock_exact.log 2>&1 || exit $?
for f in sock sim_exact sock_exact; do tail -1 $OUT/converge_$f.log | cut -c1-240; done
