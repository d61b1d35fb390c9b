"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs).

FETCH_SIZE correction, calibrated on this hardware (tools/fetch_calib.hip, profiles/r3_e1_fetch_calib.txt):
  * coalesced reads at 16, 8 AND 4 B per lane: FETCH_SIZE = exactly 1/2 of the bytes read
    (MI355X_MICROARCH.md states it for 16 B/lane; the calibration extends it to 8 and 4 B/lane);
  * random 8-B gathers: FETCH_SIZE = ~64 B per access (one line request tallied at 64 B); the kernel
    time (32 M gathers in 627 us = 3.2 TB/s at 64 B, 6.4 TB/s at 128 B) says the requests move
    ~64 B, so the 2x correction would OVERSTATE gather traffic.
A kernel mixes the two, so both bounds are reported: read_lo = FETCH_SIZE (exact for gathers),
read_hi = 2 FETCH_SIZE (exact for coalesced streams).  hbm_bytes_per_launch is the upper bound
(read_hi + write); hbm_bytes_lo_per_launch the lower.  WRITE_SIZE taken as is (exact for 16-B
streaming stores per the guide).  Infinity-Cache hits are counted by these counters, so the figures
are L2->fabric traffic (an upper bound on HBM).
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
        lo = 1024.0 * kf / max(nf, 1)
        wb = 1024.0 * kw / max(nw, 1)
        out[k] = {"dispatches": max(nf, nw), "read_bytes_per_launch": 2.0 * lo, "read_bytes_lo_per_launch": lo,
                  "write_bytes_per_launch": wb, "hbm_bytes_per_launch": 2.0 * lo + wb,
                  "hbm_bytes_lo_per_launch": lo + wb}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 3 --warmup 1",
               "correction": "read = 2 FETCH_SIZE (coalesced streams, calibrated) .. FETCH_SIZE (8-B gathers); "
                             "profiles/r3_e1_fetch_calib.txt",
               "kernels": out}, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
