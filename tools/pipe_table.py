"""Table of a tools/gpu.sh ab run: best ms per step (and numeric ms) per matrix and env variant
over the interleaved rounds.  usage: python tools/pipe_table.py <outdir> "<var0>|<var1>|..." """
import collections
import glob
import json
import sys

out, names = sys.argv[1], sys.argv[2].split("|")
d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{out}/v*_*.jsonl")):
    v = int(f.rsplit("/", 1)[1][1:].split("_")[0])
    for line in open(f):
        r = json.loads(line)
        d[r["matrix"]][v].append(r)
print("%-18s" % "matrix" + "".join("%26s" % n[:26] for n in names))
for m, vs in d.items():
    cells = []
    for i in range(len(names)):
        rs = vs.get(i, [])
        cells.append("%14.4f (%8.4f)" % (min(r["ms"] for r in rs), min(r.get("numeric_ms", 0) for r in rs)) if rs else "%26s" % "-")
    print("%-18s" % m[:18] + "".join("%26s" % c for c in cells))
