set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06i
timeout -k 10 1120 python -u tools/sparse_big.py --nodes 4194304 --rounds 400000 --fault-end 40 --until-converged --budget-s 1070 --print-every 500 --fp-every 4000 --out gpurun_out/r06i/sparse_4m_reconv.json > gpurun_out/r06i/sparse_4m_reconv.log 2>&1
