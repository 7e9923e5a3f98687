#!/bin/bash
# GPU: dense parity tests + K1c/K1s timing of the in-tree library (+ PMC=1: one K1c counter pass).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_scale.py -k dense -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1 || { tail -30 gpurun_out/pytest_dense.log; exit 1; }
tail -1 gpurun_out/pytest_dense.log
for b in 256 16; do
  timeout -k 10 300 python tools/dense_probe.py --reps 9 --batch $b 2>&1 | grep docs= | cut -c1-120
done
[ "${PMC:-0}" = "1" ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_k1c_a -o pmc --output-format csv -- python3 tools/dense_probe.py --reps 3 > gpurun_out/pmc_k1c_a.log 2>&1 || { tail -5 gpurun_out/pmc_k1c_a.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmc_k1c_a/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'dense_coarse_scan_kernelILi12' in r['Kernel_Name'] and 'Lb0E' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    print(f"{k} per_launch={sum(v)/len(v):.4g} launches={len(v)}")
PY
