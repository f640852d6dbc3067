"""Print a window of a rocprofv3 kernel trace (one PC apply in the middle of a
solve): kernel, stream (queue), start and end relative to the window start (us).
usage: trace_window.py run_kernel_trace.csv [anchor-kernel-substring] [skip]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_ilu_blocks_lds"
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 100
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
hits = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
if len(hits) <= skip:
    skip = len(hits) // 2
before = int(sys.argv[5]) if len(sys.argv) > 5 else 4
i0 = max(0, hits[skip] - before)
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + (int(sys.argv[4]) if len(sys.argv) > 4 else 24)]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q}  {r['Kernel_Name'][:90]}")
