"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel (stdin)."""
import re, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0] + ("S" if "Spill" in m.group(1) else "")] = int(m.group(2))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if pat in r["name"]:
        print(f"{r['name'][:70]:70s} V={r.get('VGPRs')} A={r.get('AGPRs')} spill={r.get('VGPRsS')} occ={r.get('Occupancy')} lds={r.get('LDS')}")
