set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06m
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bigmesh.py tests/test_events.py tests/test_gpu_multiproc.py -m gpu -x -q --timeout 300 --timeout-method thread -k "shard or rccl or union or 140k or processes" > gpurun_out/r06m/pytest.log 2>&1 &&
timeout -k 10 150 python -u tools/xvol.py 65536 8 20 > gpurun_out/r06m/xvol.log 2>&1 &&
timeout -k 10 150 python -u tools/xvol.py 65536 8 20 lists >> gpurun_out/r06m/xvol.log 2>&1 &&
KB_LIB_PATH=kaboodle_amd/variants/base.so timeout -k 10 150 python -u tools/xvol.py 65536 8 20 >> gpurun_out/r06m/xvol.log 2>&1 &&
bash tools/ab_run.sh r06m/ab base union > gpurun_out/r06m/ab.log 2>&1
