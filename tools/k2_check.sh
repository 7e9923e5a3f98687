#!/bin/bash
# GPU: BM25 parity tests then the BM25 ablation probe (+ optional variant libraries).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "bm25 or BM25 or hybrid or retrieve or smoke" > gpurun_out/k2_tests.log 2>&1 || { tail -30 gpurun_out/k2_tests.log; exit 1; }
tail -3 gpurun_out/k2_tests.log
for d in ${K2_DBG:-0 1 2 3}; do
  CM_BM25_DEBUG=$d timeout -k 10 300 python tools/bm25_probe.py > gpurun_out/probe_$d.log 2>&1 || { tail -20 gpurun_out/probe_$d.log; exit 1; }
  echo "dbg=$d $(tail -1 gpurun_out/probe_$d.log)"
done
for v in variants/*.so; do
  [ -e "$v" ] || continue
  CLASSMATE_HIP_LIB=$PWD/$v timeout -k 10 300 python tools/bm25_probe.py > gpurun_out/probe_v.log 2>&1 || { tail -20 gpurun_out/probe_v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/probe_v.log)"
done
