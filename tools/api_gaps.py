"""Host-side view of one timed bench step from a rocprofv3 --kernel-trace --hip-runtime-trace
--output-format csv run (the gzipped run_kernel_trace / run_hip_api_trace CSVs in <dir>): HIP API time
by function and the host gaps > 100 us (host work while no API call runs).
Usage: python tools/api_gaps.py <dir>"""
import csv, gzip, sys, collections
d = sys.argv[1]
K = list(csv.DictReader(gzip.open(d + '/run_kernel_trace.csv.gz', 'rt')))
A = list(csv.DictReader(gzip.open(d + '/run_hip_api_trace.csv.gz', 'rt')))
print(A[0].keys())
K.sort(key=lambda x: int(x['Start_Timestamp']))
ends = [int(x['End_Timestamp']) for x in K if 'cut_argmax2' in x['Kernel_Name']]
t0, t1 = ends[-3], ends[-2]          # one timed step (x point of step -2)
A = [a for a in A if t0 <= int(a['Start_Timestamp']) < t1]
A.sort(key=lambda a: int(a['Start_Timestamp']))
tot = collections.defaultdict(float); cnt = collections.Counter()
for a in A:
    du = (int(a['End_Timestamp']) - int(a['Start_Timestamp'])) / 1e3
    tot[a['Function']] += du; cnt[a['Function']] += 1
print('step span ms', (t1 - t0) / 1e6, 'api calls', len(A))
for f, v in sorted(tot.items(), key=lambda x: -x[1])[:15]:
    print(f'{f:40s} {cnt[f]:5d} {v/1e3:8.3f} ms')
# long calls and host gaps > 100us
prev = t0
for a in A:
    s, e = int(a['Start_Timestamp']), int(a['End_Timestamp'])
    gap = (s - prev) / 1e3
    if gap > 100 or (e - s) / 1e3 > 200:
        print(f"{(s - t0)/1e6:8.3f} ms  gap {gap:7.1f} us  {a['Function']} {(e - s)/1e3:.1f} us")
    prev = max(prev, e)
