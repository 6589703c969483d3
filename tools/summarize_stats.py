"""Print a rocprofv3 --stats kernel_stats.csv as a compact table (name, calls, total ms, avg us, %)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    name = r["Name"].replace("void ", "")[:90]
    print(f'{name:90s} {int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e6:9.3f} ms {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):6.2f}%')
