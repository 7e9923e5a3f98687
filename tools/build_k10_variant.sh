#!/bin/bash
# build_k10_variant.sh NAME "EXTRA HIPCC FLAGS" -> variants/lib_k10_NAME.so (K10 compile-time knobs / ablations)
set -e
cd "$(dirname "$0")/../classmate-rag_amd"
make -s -j4 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form $2 -I../include -Icsrc -c csrc/cm_gemm.hip -o build/cm_gemm_$1.o
mkdir -p ../variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/lib_k10_$1.so build/cm_api.o build/cm_bm25.o build/cm_dense.o build/cm_fusion.o build/cm_pool.o build/cm_filter.o build/cm_encoder.o build/cm_gemm_$1.o
