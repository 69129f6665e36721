set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06j
bash tools/ab_run.sh r06j/ab a3seq a3side > gpurun_out/r06j/ab.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "exact or horizon" > gpurun_out/r06j/pytest.log 2>&1 &&
bash tools/gpu_sq.sh r06j/sq "sim lat exact" > gpurun_out/r06j/sq.log 2>&1 &&
timeout -k 10 120 python -u tools/round_series.py 60 exact > gpurun_out/r06j/series_exact.log 2>&1 &&
timeout -k 10 120 python -u tools/round_series.py 60 window > gpurun_out/r06j/series_window.log 2>&1 &&
timeout -k 10 120 python -u tools/wave_times.py --out gpurun_out/r06j/wave_times.json > gpurun_out/r06j/wave_times.log 2>&1 &&
bash tools/sparse_sq.sh r06j/spsq > gpurun_out/r06j/spsq.log 2>&1
