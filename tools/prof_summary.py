"""Summarise a rocprofv3 kernel-stats csv and the per-kernel time of the last factorization/solve."""
import csv, re, sys, collections, glob, os
d = sys.argv[1]
stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(stats)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:20]:
    nm = re.search(r'(k_\w+|__amd\w+)', r['Name']).group(1)
    print(f"{nm:22s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:9.2f}ms {float(r['AverageNs'])/1e3:8.1f}us {float(r['TotalDurationNs'])/tot*100:5.1f}%")
print("total ms", tot / 1e6)
tr = list(csv.DictReader(open(trace)))
tr.sort(key=lambda r: int(r['Start_Timestamp']))
names = [re.search(r'(k_\w+|__amd\w+)', r['Kernel_Name']).group(1) for r in tr]
idx = [i for i, n in enumerate(names) if n == 'k_inertia']
if not idx:  # the fused MPC loop has no separate inertia launch: nothing more to break down
    sys.exit(0)
last = idx[-1]
start = max(i for i in range(last) if names[i] == 'k_status_init')
agg = collections.OrderedDict()
for i in range(start, last + 1):
    dd = (int(tr[i]['End_Timestamp']) - int(tr[i]['Start_Timestamp'])) / 1e3
    a = agg.setdefault(names[i], [0, 0]); a[0] += dd; a[1] += 1
print("last factorization: span %.1f us" % ((int(tr[last]['End_Timestamp']) - int(tr[start]['Start_Timestamp'])) / 1e3))
for k, v in agg.items(): print(f"   {k:20s} {v[1]:5d} {v[0]:9.1f}us")
if len(sys.argv) > 2:
    for i in range(start, last + 1):
        dd = (int(tr[i]['End_Timestamp']) - int(tr[i]['Start_Timestamp'])) / 1e3
        print(f"{names[i]:16s} grid={int(tr[i]['Grid_Size_X'])//256:7d} {dd:8.1f}")
