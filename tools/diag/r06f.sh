set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06f
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --seeds "" > gpurun_out/r06f/bench.json 2> gpurun_out/r06f/bench.err &&
timeout -k 10 300 python -u tools/sparse_big.py --nodes 4194304 --rounds 96 --fault-end 40 --print-every 8 --fp-every 8 --out gpurun_out/r06f/sparse4m_long.json > gpurun_out/r06f/sparse4m_long.log 2>&1 &&
timeout -k 10 300 python -u tools/sparse_big.py --nodes 4194304 --rounds 48 --print-every 8 --fp-every 8 --out gpurun_out/r06f/sparse4m_stated.json > gpurun_out/r06f/sparse4m_stated.log 2>&1
