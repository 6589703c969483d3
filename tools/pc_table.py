"""Top instructions of a rocprofv3 PC-sampling CSV (stochastic or host-trap), per kernel.
usage: python tools/pc_table.py <dir with *pc_sampling*.csv> [kernel-substring] [N]"""
import csv
import glob
import sys
from collections import Counter, defaultdict

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else ""
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
files = glob.glob(f"{d}/**/*pc_sampling*.csv", recursive=True)
if not files:
    sys.exit(f"no pc sampling csv under {d}")
per = defaultdict(Counter)
stall = defaultdict(Counter)
tot = Counter()
for f in files:
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name") or r.get("Dispatch_Id", "?")
        if ksub and ksub not in k:
            continue
        ins = r.get("Instruction") or r.get("Instruction_Comment") or r.get("Code_Object_Offset", "?")
        per[k][ins] += 1
        tot[k] += 1
        sr = r.get("Stall_Reason") or r.get("Wave_Issue_Reason") or ""
        if sr:
            stall[k][sr] += 1
for k, c in sorted(per.items(), key=lambda kv: -tot[kv[0]])[:4]:
    print(f"== {k[:100]}  samples {tot[k]}")
    for ins, n in c.most_common(top):
        print(f"{100.0 * n / tot[k]:6.2f}%  {ins[:110]}")
    if stall[k]:
        print("  stall reasons:", ", ".join(f"{s} {100.0 * n / tot[k]:.1f}%" for s, n in stall[k].most_common(8)))
