"""Per-kernel VGPRs / VGPR spills / occupancy from hipcc -Rpass-analysis=kernel-resource-usage
output on stdin (CPU container).  usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 |
python tools/kres_spills.py [--spills-only]"""
import re
import sys

rows, cur = [], {}
for line in sys.stdin:
    m = re.search(r"remark: +([A-Za-z \[\]/]+?): (\S+)", line)
    if not m:
        continue
    key, val = m.group(1).strip(), m.group(2)
    if key == "Function Name":
        if cur:
            rows.append(cur)
        cur = {"name": re.sub(r"EEEvNS.*|^_ZN3cvq\d+", "", val)}
    else:
        cur[key] = val
if cur:
    rows.append(cur)
only = "--spills-only" in sys.argv
for r in rows:
    sp = int(r.get("VGPRs Spill", "0"))
    if only and sp == 0:
        continue
    print(f"{r['name'][:60]:60s} VGPRs {r.get('VGPRs', '?'):>4s} spill {sp:4d} occ {r.get('Occupancy [waves/SIMD]', '?')}")
