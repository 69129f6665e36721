set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06u
bash tools/final_conv.sh r06u/conv > gpurun_out/r06u/conv.log 2>&1 &&
bash tools/gpu_sq.sh r06u/sq sim > gpurun_out/r06u/sq.log 2>&1
