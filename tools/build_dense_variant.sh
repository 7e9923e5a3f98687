#!/bin/bash
# build_dense_variant.sh NAME "EXTRA HIPCC FLAGS" -> variants/lib_NAME.so (cm_dense.hip compile-time knobs, A/B probes)
set -e
cd "$(dirname "$0")/../classmate-rag_amd"
make -s -j8 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -amdgpu-mfma-vgpr-form $2 -I../include -Icsrc -c csrc/cm_dense.hip -o build/cm_dense_$1.o
mkdir -p ../variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/lib_$1.so build/cm_api.o build/cm_dense_$1.o build/cm_bm25.o build/cm_fusion.o build/cm_pool.o build/cm_filter.o build/cm_encoder.o build/cm_gemm.o
