"""Register / spill / LDS summary of the kernels in a hipcc -save-temps .s file.
python tools/kstats.py file.s [name-substring]"""
import re
import sys

text = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in text.split("  - .agpr_count:")[1:]:
    name = re.search(r"\n    \.name:\s+(\S+)", blk).group(1)
    if pat not in name:
        continue
    g = lambda k: (re.search(r"\n    \." + k + r":\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
    agpr = blk.split("\n", 1)[0].strip()
    print(f"{name[:70]:70s} vgpr {g('vgpr_count'):>4s} agpr {agpr:>4s} spill {g('vgpr_spill_count'):>3s} "
          f"scratch {g('private_segment_fixed_size'):>3s} sgpr {g('sgpr_count')}")
