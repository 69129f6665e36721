set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06n
timeout -k 10 500 python -u tools/ipc_ranks.py --worlds 1 2 4 --steps 20 --warmup 5 --out gpurun_out/r06n/ipc_ranks.json > gpurun_out/r06n/ipc_ranks.log 2>&1
