"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports 1/2 of the
bytes of wide coalesced reads on gfx950 -> doubled; WRITE_SIZE (KB) taken as is.  Infinity-Cache
hits are counted by these counters, so the figure is L2->fabric traffic (an upper bound on HBM).
usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json
"""
import csv, glob, json, os, re, sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
        a = acc[m.group(1) if m else r["Kernel_Name"]]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
    return acc


def main():
    fe, wr = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fe) | set(wr)):
        nf, kf = fe.get(k, [0, 0.0])
        nw, kw = wr.get(k, [0, 0.0])
        rd = 2.0 * 1024.0 * kf / max(nf, 1)
        wb = 1024.0 * kw / max(nw, 1)
        out[k] = {"dispatches": max(nf, nw), "read_bytes_per_launch": rd, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": rd + wb}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 3 --warmup 1",
               "kernels": out}, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
