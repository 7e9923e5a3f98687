#!/bin/bash
# GPU: K1c variants (variants/lib_*.so) at the bench shape, interleaved; PMC=1 adds counter passes.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for f in variants/lib_*.so; do
  v=$(basename $f .so)
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --reps 7 2>&1 | grep docs= | sed "s/^/$v /" | cut -c1-120
done; done
[ "${PMC:-0}" = "1" ] || exit 0
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM" \
           "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc_k1c_$i -o pmc --output-format csv -- python3 tools/dense_probe.py --reps 3 > gpurun_out/pmc_k1c_$i.log 2>&1 || { tail -5 gpurun_out/pmc_k1c_$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmc_k1c_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'dense_coarse_scan_kernelILi12' in r['Kernel_Name'] and 'Lb0E' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
with open('gpurun_out/pmc_k1c.txt', 'w') as out:
    for k, v in sorted(agg.items()):
        line = f"{k} per_launch={sum(v)/len(v):.4g} launches={len(v)}"
        print(line); out.write(line + "\n")
PY
