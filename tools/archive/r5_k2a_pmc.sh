#!/bin/bash
# round 5: K2a counters (separate --pmc passes over tools/bm25_probe.py, pruned path, 10M x B=256)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k2apmc; export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set -d gpurun_out/k2apmc/p$i -o pmc --output-format csv -- python3 tools/bm25_probe.py --paths 2 --reps 3 > gpurun_out/k2apmc/p$i.log 2>&1 || { tail -5 gpurun_out/k2apmc/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob('gpurun_out/k2apmc/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'bm25_tail_kernel' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()):
    print(f"{k:32s} {sum(v)/len(v):16.6g}  (n={len(v)})")
PY
