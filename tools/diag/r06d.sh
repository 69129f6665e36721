set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06d
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sparse.py -k "exact or every_round or sparse" -x -q --timeout 300 --timeout-method thread --durations=25 > gpurun_out/r06d/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --a3-order exact --no-cpu --seeds "" > gpurun_out/r06d/bench_exact.json 2> gpurun_out/r06d/bench_exact.err
timeout -k 10 300 python -u tools/sparse_big.py --nodes 4194304 --rounds 96 --fault-end 40 --no-sf-failed-drops --out gpurun_out/r06d/sparse4m_nosf.json > gpurun_out/r06d/sparse4m.log 2>&1
