"""Timeline of the last bench step from a rocprofv3 kernel trace: kernel, duration and the
idle gap before it (us).  python3 tools/trace_timeline.py <dir with t/**/run_kernel_trace.csv>"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/t/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last step = from the last pool_select launch onward
starts = [i for i, r in enumerate(rows) if "pool_select" in r["Kernel_Name"]]
i0 = starts[-1] if starts else 0
prev = None
tot_k = 0.0
for r in rows[i0 - 3 if i0 >= 3 else 0:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    tot_k += (e - s) / 1e3
    print(f"{(e - s) / 1e3:10.1f} us  gap {gap:8.1f} us  {r['Kernel_Name'][:90]}")
    prev = e
print("kernel time of listed", round(tot_k, 1), "us")
