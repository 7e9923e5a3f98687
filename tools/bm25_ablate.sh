#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for dbg in 0 1 2 3; do
  CM_BM25_DEBUG=$dbg timeout -k 10 300 python tools/bm25_probe.py || exit 1
done
timeout -k 10 300 python tools/bm25_probe.py --head-bytes 0 || exit 1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc1 -o pmc --output-format csv -- python3 tools/bm25_probe.py --reps 2 > gpurun_out/pmc1.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc2 -o pmc --output-format csv -- python3 tools/bm25_probe.py --reps 2 > gpurun_out/pmc2.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3 -o pmc --output-format csv -- python3 tools/bm25_probe.py --reps 2 > gpurun_out/pmc3.log 2>&1 || exit 1
