"""Per-launch timeline of one MPC iteration from a rocprofv3 kernel-trace csv (third-to-last k_term
to second-to-last): kernel, template, workgroups, duration, gap to the previous launch's end (negative:
concurrent launches on two streams), start relative to the iteration's first launch."""
import csv, glob, os, re, sys
d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
tr = list(csv.DictReader(open(f)))
tr.sort(key=lambda r: int(r['Start_Timestamp']))
names = [re.search(r'(k_\w+|__amd\w+)', r['Kernel_Name']).group(1) for r in tr]
idx = [i for i, n in enumerate(names) if n == 'k_term']
a, b = idx[-3], idx[-2]
filt = sys.argv[2] if len(sys.argv) > 2 else None
tot = 0.0
for i in range(a, b):
    r = tr[i]
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    tot += dur
    if filt and filt not in names[i]:
        continue
    gap = (int(r['Start_Timestamp']) - int(tr[i - 1]['End_Timestamp'])) / 1e3
    tm = re.search(r'<(\d+)>', r['Kernel_Name'])
    t = (int(r['Start_Timestamp']) - int(tr[a]['Start_Timestamp'])) / 1e3
    print(f"{names[i]:18s}{'<' + tm.group(1) + '>' if tm else '   ':5s} wg={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):6d} "
          f"{dur:7.1f}us gap {gap:5.1f}  at {t:6.1f}")
print(f"iteration: busy {tot:.1f} us, span {(int(tr[b]['Start_Timestamp']) - int(tr[a]['Start_Timestamp'])) / 1e3:.1f} us")
