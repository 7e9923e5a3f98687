#!/bin/bash
# ASan + UBSan on the host code (SURVEY §5 "sanitizers"; no GPU sanitizers on this pool):
#  1. oracle/cm_oracle.c (the CPU oracle) under a seeded driver, and the C-oracle pytest cases with
#     the sanitized liboracle preloaded into Python (CM_ORACLE_LIB);
#  2. libclassmate_hip's sources with the sanitizers on the host side only (-Xarch_host before each
#     -fsanitize=; the gfx950 device code is built as usual) linked into a driver that walks every
#     entry point's validation / error paths (no GPU needed).
# Outputs under oracle/_asan/ (git-ignored).  Exit 0 = clean.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=oracle/_asan; mkdir -p $OUT
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all -g -O1"
gcc $SAN -fopenmp -ffp-contract=off -std=c11 -Wall -o $OUT/oracle_driver tests/asan/oracle_driver.c oracle/cm_oracle.c -lm
gcc $SAN -fopenmp -ffp-contract=off -std=c11 -Wall -fPIC -shared -o $OUT/liboracle.so oracle/cm_oracle.c -lm
HIPCC=/opt/rocm/bin/hipcc
objs=()
for f in cm_api.cpp cm_dense.hip cm_bm25.hip cm_fusion.hip cm_pool.hip cm_filter.hip cm_encoder.hip cm_gemm.hip; do
  o=$OUT/${f%.*}.o; objs+=($o)
  if [ ! -f $o ] || [ classmate-rag_amd/csrc/$f -nt $o ] || [ include/classmate_hip.h -nt $o ] || [ classmate-rag_amd/csrc/cm_common.h -nt $o ]; then
    $HIPCC --offload-arch=gfx950 -std=c++17 -fPIC -O1 -g -Iinclude -Iclassmate-rag_amd/csrc \
      -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
      -Xarch_host -fno-sanitize-recover=all -c classmate-rag_amd/csrc/$f -o $o &
  fi
done
wait
/opt/rocm/lib/llvm/bin/clang $SAN -Iinclude -c tests/asan/host_driver.c -o $OUT/host_driver.o
$HIPCC --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -g \
  -o $OUT/host_driver $OUT/host_driver.o "${objs[@]}"
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
OMP_NUM_THREADS=4 $OUT/oracle_driver
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 $OUT/host_driver
# the C-oracle pytest cases with the sanitized oracle (LeakSanitizer off: the interpreter itself)
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so) \
  CM_ORACLE_LIB=$PWD/$OUT/liboracle.so OMP_NUM_THREADS=4 \
  python -m pytest -q -p no:cacheprovider tests/test_oracle_c.py -x 2>&1 | tail -1
