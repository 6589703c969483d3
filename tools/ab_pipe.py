"""Summary of tools/pipe.py A/B files <dir>/<tag>_<round>.jsonl: best ms per (matrix, tag)."""
import glob
import json
import sys

out = sys.argv[1]
res = {}
for f in sorted(glob.glob(out + "/*_?.jsonl")):
    tag = f.split("/")[-1].rsplit("_", 1)[0]
    for line in open(f):
        d = json.loads(line)
        res.setdefault(d["matrix"], {}).setdefault(tag, []).append(d["ms"])
for m, v in res.items():
    tags = sorted(v)
    print(f"{m:18s}", "  ".join(f"{k} {min(x):.4f}" for k, x in sorted(v.items())),
          f"  ({tags[-1]}/{tags[0]} {min(v[tags[-1]]) / min(v[tags[0]]):.3f})" if len(tags) == 2 else "")
