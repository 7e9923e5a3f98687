#!/bin/bash
# GPU: BM25 probe (pruned path) per variant library in variants/ (+ the product library), then an
# optional ablation sweep on variants/lib_abl.so.  Timing only; each run under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bm25_probe.py --paths 2 --reps 7 > gpurun_out/k2v_base.log 2>&1 || { tail -5 gpurun_out/k2v_base.log; exit 1; }
echo "base $(tail -1 gpurun_out/k2v_base.log | cut -c1-160)"
for v in ${VARIANTS:-variants/lib_*.so}; do
  n=$(basename $v .so)
  [ "$n" = lib_abl ] && continue
  CLASSMATE_HIP_LIB=$PWD/$v timeout -k 10 300 python -u tools/bm25_probe.py --paths 2 --reps 7 > gpurun_out/k2v_$n.log 2>&1 || { tail -5 gpurun_out/k2v_$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/k2v_$n.log | cut -c1-160)"
done
if [ -n "$DBG" ]; then
  CLASSMATE_HIP_LIB=$PWD/variants/lib_abl.so timeout -k 10 300 python -u tools/bm25_probe.py --paths 2 --reps 7 --dbg $DBG > gpurun_out/k2v_abl.log 2>&1 || { tail -5 gpurun_out/k2v_abl.log; exit 1; }
  grep "docs=" gpurun_out/k2v_abl.log | cut -c1-160
fi
