#!/bin/bash
# GPU: candidate / band sizes (print variant) + kernel trace of the headline step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
CLASSMATE_HIP_LIB=$PWD/variants/lib_qprint.so timeout -k 10 200 python tools/dense_probe.py --path 5 --reps 1 > gpurun_out/k1qdbg.log 2>&1 || { tail -20 gpurun_out/k1qdbg.log; exit 1; }
grep -E "rerank" gpurun_out/k1qdbg.log | sort | uniq | head -12
bash tools/r4_prof6.sh
