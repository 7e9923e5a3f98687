#!/bin/bash
# GPU: K1q v6 epilogue split (q64: pre-test only, q128: no epilogue) + kernel trace of the probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/v6abl; export TMPDIR=/tmp
bash tools/k1q_abl2.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v6abl/trace -o probe --output-format csv -- python3 tools/dense_probe.py --path 5 --reps 5 > gpurun_out/v6abl/trace.log 2>&1 || { tail -20 gpurun_out/v6abl/trace.log; exit 1; }
find gpurun_out/v6abl/trace -name '*kernel_stats.csv' | head -1 | xargs -I{} cut -d, -f1-4 {} | head -20
