"""Summarise a `rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES
GRBM_GUI_ACTIVE` counter collection per kernel: achieved f64 MFMA TF/s (MOPS_F64 are in units of
512 flops) and MFMA pipe utilisation (BUSY / (1024 SIMDs x clock x time), clock = GRBM_GUI_ACTIVE /
8 XCDs / time).  usage: python tools/pmc_mfma.py <run_counter_collection.csv> [kernel ...]"""
import csv
import sys
from collections import defaultdict

PEAK_TF = 78.6


def summarise(path, kernels):
    disp = defaultdict(dict)  # (kernel, dispatch) -> counter -> value, plus the duration
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0].split("<")[0]
        name = name.split("::")[-1].split()[-1]
        if kernels and name not in kernels:
            continue
        d = disp[(name, int(r["Dispatch_Id"]))]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = defaultdict(lambda: defaultdict(float))
    for (name, _), d in disp.items():
        t = tot[name]
        t["n"] += 1
        for k, v in d.items():
            t[k] += v
    out = []
    for name, t in sorted(tot.items(), key=lambda kv: -kv[1]["ns"]):
        sec = t["ns"] * 1e-9
        if sec <= 0 or t.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0) == 0:
            continue
        tf = t["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512 / sec / 1e12
        clk = t["GRBM_GUI_ACTIVE"] / 8 / sec
        util = t["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk * sec)
        out.append(f"  {name:14s} dispatches {int(t['n']):4d}  time {sec * 1e3:9.2f} ms  {tf:8.2f} TF/s "
                   f"({100 * tf / PEAK_TF:5.1f} % of {PEAK_TF})  MFMA pipe util {100 * util:5.1f} %  "
                   f"clock {clk / 1e9:.2f} GHz")
    return out


if __name__ == "__main__":
    print("\n".join(summarise(sys.argv[1], set(sys.argv[2:]))))
