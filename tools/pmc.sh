#!/bin/bash
# tools/pmc.sh NAME KERNEL_SUBSTR -- CMD...   : three separate rocprofv3 --pmc passes over CMD,
# per-launch averages for kernels whose name contains KERNEL_SUBSTR -> gpurun_out/pmc_NAME.txt
set -o pipefail
name=$1; kern=$2; shift 3
mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
SETS=${PMC_SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS;SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES;FETCH_SIZE GRBM_GUI_ACTIVE"}
IFS=';' read -ra SETARR <<< "$SETS"
for set in "${SETARR[@]}"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set -d gpurun_out/pmc_${name}_$i -o pmc --output-format csv -- "$@" > gpurun_out/pmc_${name}_$i.log 2>&1 || { tail -20 gpurun_out/pmc_${name}_$i.log; exit 1; }
done
python3 - "$name" "$kern" <<'PY'
import csv, glob, sys, collections
name, kern = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f'gpurun_out/pmc_{name}_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
with open(f'gpurun_out/pmc_{name}.txt', 'w') as out:
    for k, v in sorted(agg.items()):
        line = f"{k} per_launch={sum(v)/len(v):.4g} launches={len(v)}"
        print(line); out.write(line + "\n")
PY
