#!/bin/bash
# round 5 closing check: full GPU suite + smoke + default bench (tools/r5_check.sh), then the batch-1
# encode (tools/e5_b1_probe.py: the padded small-batch graph, key-masked K9s) with the K9s key-mask
# loads issued first vs the previous order (variants/lib_k9s_prev.so), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
bash tools/r5_check.sh || exit 1
mkdir -p gpurun_out/k9s
base=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; prev=$PWD/variants/lib_k9s_prev.so
for r in 1 2; do
  for v in new prev; do
    L=$base; [ $v = prev ] && L=$prev
    CLASSMATE_HIP_LIB=$L timeout -k 10 200 python -u tools/e5_b1_probe.py > gpurun_out/k9s/probe_$v.log 2>&1 || { tail -20 gpurun_out/k9s/probe_$v.log; exit 1; }
    grep "E5 encode" gpurun_out/k9s/probe_$v.log | sed "s/^/$v /"
  done
done
