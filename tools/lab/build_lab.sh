#!/bin/bash
# Build a GEMM lab kernel file into tools/lab/so/lib<name>.so (run here, on the CPU; the .so travels
# with the tree when the lab is run): bash tools/lab/build_lab.sh gemm_hc_lab.hip gemm_hc
set -e
cd "$(dirname "$0")"
mkdir -p so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../../include "$1" -o so/lib$2.so \
  ${LAB_FLAGS:-}
echo built tools/lab/so/lib$2.so
