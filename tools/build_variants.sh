#!/bin/bash
# Dev A/B builds of the HIP library (timing experiments only): tools/build_variants.sh NAME "FLAGS" ...
# -> kaboodle_amd/variants/NAME.so, run with KB_LIB_PATH=kaboodle_amd/variants/NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p kaboodle_amd/variants
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value -lrccl -pthread \
    $2 -o kaboodle_amd/variants/$1.so kaboodle_amd/csrc/kb_sim.hip &
  shift 2
done
wait
ls -la kaboodle_amd/variants
