set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06s
bash tools/final_conv.sh r06s/conv > gpurun_out/r06s/conv.log 2>&1 &&
bash tools/gpu_sq.sh r06s/sq sim > gpurun_out/r06s/sq.log 2>&1
