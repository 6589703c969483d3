"""Per-kernel averages of rocprofv3 --pmc passes (run_counter_collection.csv files) of one
matrix directory: python tools/pmc_table.py gpurun_out/<tag>/<matrix> [--json out.json]
Counters are averaged per dispatch of each kernel name (the sweep makes reps+3 calls)."""
import csv, glob, json, re, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(f"{d}/pmc_*/run_counter_collection.csv")):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (f, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {}
for k, cs in acc.items():
    row = {c: sum(v) / len(v) for c, v in cs.items()}
    row["ms"] = sum(dur[k]) / len(dur[k])
    out[k] = row
for k, row in sorted(out.items(), key=lambda x: -x[1]["ms"]):
    if row["ms"] < 0.05:
        continue
    print(f"{k:45s} {row['ms']:8.3f} ms  " + " ".join(f"{c}={v:.3e}" for c, v in sorted(row.items()) if c != "ms"))
if "--json" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
