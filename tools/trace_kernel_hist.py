"""Duration histogram of one kernel in a rocprofv3 kernel trace (per-launch rows):
usage: trace_kernel_hist.py run_kernel_trace.csv kernel-substring"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows])
g = np.array([int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) for r in rows])
wg = np.array([int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1) for r in rows])
blocks = g // np.maximum(wg, 1)
print(f"{len(d)} launches, total {d.sum() / 1e3:.1f} ms; duration us p10/50/90/99/max "
      f"{np.percentile(d, 10):.1f} {np.percentile(d, 50):.1f} {np.percentile(d, 90):.1f} {np.percentile(d, 99):.1f} {d.max():.1f}")
for lo, hi in ((0, 8), (8, 32), (32, 64), (64, 128), (128, 1 << 30)):
    m = (blocks >= lo) & (blocks < hi)
    if m.any():
        print(f"  workgroups [{lo}, {hi}): {m.sum()} launches, mean {d[m].mean():.1f} us, total {d[m].sum() / 1e3:.1f} ms")
order = np.argsort(-d)[:8]
print("slowest:", [(round(d[i], 1), int(blocks[i])) for i in order])
print("first 20 in order:", [(round(d[i], 1), int(blocks[i])) for i in range(min(20, len(d)))])
