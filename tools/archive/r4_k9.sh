#!/bin/bash
# GPU: K9s without the LDS O-transpose -- accuracy tests, then headline A/B against variants/lib_k9old.so, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k9; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k9/pytest.log 2>&1 || { tail -40 gpurun_out/k9/pytest.log; exit 1; }
tail -1 gpurun_out/k9/pytest.log
HL="--steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0"
for rep in 1 2; do for v in new old; do
  if [ $v = old ]; then L=$PWD/variants/lib_k9old.so; else L=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; fi
  CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u bench.py $HL --out gpurun_out/k9/b_$v$rep.json > gpurun_out/k9/b.log 2>&1 || { tail -30 gpurun_out/k9/b.log; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/k9/b_$v$rep.json'));print(d['value'],d['ms_per_step'])")" | tee -a gpurun_out/k9/ab.txt
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k9/trace -o hl --output-format csv -- python3 -u bench.py $HL --out gpurun_out/k9/b_tr.json > gpurun_out/k9/tr.log 2>&1 || { tail -30 gpurun_out/k9/tr.log; exit 1; }
find gpurun_out/k9/trace -name "*kernel_stats.csv" | head -1 | xargs grep -E "attention|layernorm" | cut -c1-200
