"""Per-kernel VGPR / SGPR / spill / occupancy from hipcc -Rpass-analysis=kernel-resource-usage output.
usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/kres.py [name-filter]"""
import re, subprocess, sys
flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"\b(VGPRs|AGPRs|SGPRs|TotalSGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    if flt in r["name"]:
        dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"\(.*", "", dem.replace("(anonymous namespace)::", ""))
        print(f"{dem:60s} vgpr {r.get('VGPRs')} agpr {r.get('AGPRs')} sgpr {r.get('SGPRs')} "
              f"vspill {r.get('VGPRs Spill')} sspill {r.get('SGPRs Spill')} occ {r.get('Occupancy [waves/SIMD]')} "
              f"lds {r.get('LDS Size [bytes/block]')}")
