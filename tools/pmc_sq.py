"""Per-kernel sums of the counters in a rocprofv3 --pmc collection (SQ cycle counters are in quad-cycles,
MI355X_MICROARCH.md).  usage: python tools/pmc_sq.py <run_counter_collection.csv> [kernel ...]"""
import csv
import sys
from collections import defaultdict


def kname(raw):
    n = raw.replace("(anonymous namespace)", "").split("(")[0].split("<")[0]
    return n.split("::")[-1].split()[-1]


def main(path, kernels):
    acc = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if kernels and k not in kernels:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        d = int(r["Dispatch_Id"])
        if d not in seen[k]:
            seen[k].add(d)
            acc[k]["_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1]["_ns"]):
        n = len(seen[k])
        print(f"{k}: {n} dispatches, {c['_ns'] / n / 1e3:.1f} us avg")
        for name in sorted(c):
            if name != "_ns":
                print(f"   {name:28s} {c[name] / n:16.4g} per dispatch")


if __name__ == "__main__":
    main(sys.argv[1], set(sys.argv[2:]))
