"""Best-of-rounds phase table of a tools/ab.sh run.  usage: python tools/ab_table.py <tag>"""
import collections
import glob
import json
import sys

keys = ["Form_mask_matrix_B", "symbolic_binning", "Calculate_C_nnz", "numeric_binning", "Numeric", "total_e2e"]
d = collections.defaultdict(lambda: collections.defaultdict(list))
order = []
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/ab_*.jsonl")):
    v = f.split("ab_", 1)[1].rsplit("_", 1)[0]
    if v not in order:
        order.append(v)
    for line in open(f):
        r = json.loads(line)
        d[r["matrix"]][v].append(r)
print("%-16s %-22s" % ("matrix", "variant") + " ".join("%9s" % k[:9] for k in keys))
for m in d:
    for v in order:
        rs = d[m][v]
        if rs:
            name = v.replace("abvar_", "").replace("mh-spgemm_amd_mhspgemm", "TREE")
            print("%-16s %-22s" % (m[:16], name[:22]) + " ".join("%9.4f" % min(r[k] for r in rs) for k in keys))
