"""Print per-kernel resource metadata (VGPRs, SGPRs, LDS, scratch) from a
hipcc -save-temps .s file.  Usage: python tools/kmeta.py file.s [filter]"""
import re
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = txt[txt.find("amdhsa.kernels:"):]
for block in re.split(r"\n  - \.", meta)[1:]:
    block = "." + block
    name = re.search(r"\.name:\s+(\S+)", block)
    if not name or flt not in name.group(1):
        continue
    f = {k: re.search(r"\.%s:\s+(\S+)" % k, block) for k in
         ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size")}
    print(name.group(1)[:70], " ".join("%s=%s" % (k.split("_")[0] if k != "group_segment_fixed_size" else "lds",
                                                   v.group(1)) for k, v in f.items() if v))
