"""Print the kernel timeline of the last full step of a rocprofv3 kernel trace.
usage: python tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [first-kernel-substring]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_mask_"  # k_mask_b or k_mask_lane
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
st, en = idx[-3], idx[-2]
t0 = int(rows[st]["Start_Timestamp"]); prev = t0
busy = 0
for r in rows[st:en]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1000:8.1f} gap {(s - prev) / 1000:6.1f} dur {(e - s) / 1000:7.1f}  {r['Kernel_Name'][:80]}")
    prev = e
step = int(rows[en]["Start_Timestamp"]) - t0
print(f"step {step / 1000:.1f} us, kernels busy {busy / 1000:.1f} us")
