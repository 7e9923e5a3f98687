#!/bin/bash
# GPU: E5 GEMMs default vs TunableOp-tuned; E5 encode probe with the tuned table.  -> gpurun_out/tune/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/tune; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/gemm_probe.py > gpurun_out/tune/gemm_default.log 2>&1 || { tail -20 gpurun_out/tune/gemm_default.log; exit 1; }
cat gpurun_out/tune/gemm_default.log
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_e5.csv
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 400 python -u tools/gemm_probe.py > gpurun_out/tune/gemm_tuning.log 2>&1 || { tail -20 gpurun_out/tune/gemm_tuning.log; exit 1; }
PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 120 python -u tools/gemm_probe.py > gpurun_out/tune/gemm_tuned.log 2>&1 || { tail -20 gpurun_out/tune/gemm_tuned.log; exit 1; }
cat gpurun_out/tune/gemm_tuned.log
PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 200 python -u tools/e5_probe.py > gpurun_out/tune/e5_tuned.log 2>&1 || { tail -20 gpurun_out/tune/e5_tuned.log; exit 1; }
cat gpurun_out/tune/e5_tuned.log
unset PYTORCH_TUNABLEOP_ENABLED
timeout -k 10 200 python -u tools/e5_probe.py > gpurun_out/tune/e5_default.log 2>&1 || { tail -20 gpurun_out/tune/e5_default.log; exit 1; }
cat gpurun_out/tune/e5_default.log
