set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06y
bash tools/final_conv.sh r06y/conv > gpurun_out/r06y/conv.log 2>&1 &&
bash tools/final_extra.sh r06y/extra > gpurun_out/r06y/extra.log 2>&1
