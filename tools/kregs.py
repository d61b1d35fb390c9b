"""Register / spill / LDS summary per kernel from a hipcc -S (gfx950) assembly file.
usage: python tools/kregs.py file.s [substring ...]"""
import re
import sys


def main(path, subs):
    s = open(path).read()
    meta = s[s.find("amdhsa.kernels:"):]
    for ent in re.split(r"\n\s+- \.agpr_count:", meta)[1:]:
        name = re.search(r"\.name:\s+(\S+)", ent).group(1)
        if subs and not any(x in name for x in subs):
            continue
        get = lambda k: (re.findall(r"\.%s:\s+(\d+)" % k, ent) or ["?"])[0]
        print(f"{name[:70]:70s} agpr {ent.split()[0]:>3s} vgpr {get('vgpr_count'):>3s} vspill {get('vgpr_spill_count'):>3s} "
              f"sgpr {get('sgpr_count'):>3s} sspill {get('sgpr_spill_count'):>4s} scratch {get('private_segment_fixed_size'):>4s} "
              f"lds {get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
