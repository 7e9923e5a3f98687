#!/bin/bash
# GPU: HBM traffic per launch of the dominant kernels (K1c / K1q B=256, K1s B=16, K2a B=256) at the bench
# shape, from separate rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE + TCC hit/miss), each pass its
# own run.  Writes gpurun_out/pmc_traffic_<round>.txt (per-launch averages) and .json.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r02}
run() {  # name kernel-substring cmd...
  local name=$1 kern=$2; shift 2
  local i=0
  for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set -d gpurun_out/pmcT_${name}_$i -o pmc --output-format csv -- "$@" > gpurun_out/pmcT_${name}_$i.log 2>&1 || { tail -5 gpurun_out/pmcT_${name}_$i.log; return 1; }
  done
  python3 - "$name" "$kern" "$R" <<'PY'
import csv, glob, sys, collections, json
name, kern, R = sys.argv[1:4]
agg = collections.defaultdict(list)
for f in glob.glob(f'gpurun_out/pmcT_{name}_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
res = {k: sum(v) / len(v) for k, v in agg.items()}
res["launches"] = len(agg.get("FETCH_SIZE", []))
with open(f'gpurun_out/pmc_traffic_{R}.txt', 'a') as out:
    out.write(f"{name} [{kern}] " + " ".join(f"{k}={v:.6g}" for k, v in sorted(res.items())) + "\n")
try:
    d = json.load(open(f'gpurun_out/pmc_traffic_{R}.json'))
except Exception:
    d = {}
d[name] = res
json.dump(d, open(f'gpurun_out/pmc_traffic_{R}.json', 'w'), indent=1)
print(name, res)
PY
}
rm -f gpurun_out/pmc_traffic_${R}.txt gpurun_out/pmc_traffic_${R}.json
W=${ONLY:-dense_B256 dense_B16 bm25_B256}   # ONLY="bm25_B256 ..." -> a subset
for n in $W; do
  case $n in
    dense_B256) run dense_B256 "dense_coarse_scan_kernelILi12ELi3ELb0" python3 tools/dense_probe.py --reps 3 --batch 256 --path 3 || exit 1 ;;
    dense_q8_B256) run dense_q8_B256 "dense_q8_scan_kernel<false" python3 tools/dense_probe.py --reps 3 --batch 256 --path 5 || exit 1 ;;
    dense_q8s_B16) run dense_q8s_B16 "dense_q8_stream_kernel" python3 tools/dense_probe.py --reps 3 --batch 16 --k 10 || exit 1 ;;
    dense_B16) run dense_B16 "dense_stream_scan_kernelILi12ELi1ELb0" python3 tools/dense_probe.py --reps 3 --batch 16 || exit 1 ;;
    bm25_B256) run bm25_B256 "bm25_tail_kernel" python3 tools/bm25_probe.py --paths 2 --reps 3 || exit 1 ;;
    bm25b_B256) run bm25b_B256 "bm25_block_kernel" python3 tools/bm25_probe.py --paths 2 --reps 3 || exit 1 ;;
  esac
done
