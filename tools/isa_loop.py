"""Instruction mix of a kernel's hot loops from device assembly (CPU container).
usage: python tools/isa_loop.py <file.s> <mangled-name-prefix> [--min-rcp N | --marker OP --min N]
Prints, for each basic block containing >= N of the marker op, the op histogram and waitcnts,
and the kernel's VGPR / spill / occupancy metadata."""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
marker = sys.argv[sys.argv.index("--marker") + 1] if "--marker" in sys.argv else "ds_read_b128"
mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 8
s = open(path).read().split("\n")
start = [i for i, l in enumerate(s) if l.startswith(name) and l.split(":")[0].startswith(name)]
if not start:
    sys.exit(f"no function {name}")
i0 = start[0]
i1 = i0
while not s[i1].startswith(".Lfunc_end"):
    i1 += 1
f = s[i0:i1]
blocks, cur, lab = [], [], None
for l in f:
    if re.match(r"^\.LBB|^_Z", l):
        if cur:
            blocks.append((lab, cur))
        lab, cur = l.split(";")[0].strip(), []
    elif l.strip() and not l.strip().startswith((";", ".")):
        cur.append(l.strip())
blocks.append((lab, cur))
for lab, b in blocks:
    if sum(x.startswith(marker) for x in b) >= mn:
        ops = {}
        for x in b:
            ops[x.split()[0]] = ops.get(x.split()[0], 0) + 1
        waits = [x for x in b if x.startswith("s_waitcnt")]
        print(lab, len(b), " ".join(f"{k}:{v}" for k, v in sorted(ops.items(), key=lambda t: -t[1])))
        print("   waits:", "; ".join(w[10:] for w in waits))
for l in s[i1:i1 + 400]:
    m = re.search(r"; (NumVgprs|ScratchSize|Occupancy|NumAgprs|TotalNumVgprs): (\d+)", l)
    if m:
        print("  ", m.group(1), m.group(2))
    if "Lfunc_end" in l and l.strip() != s[i1].strip():
        break
