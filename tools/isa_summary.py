"""Static instruction mix of kernels in a gfx950 assembly listing.

usage: python tools/isa_summary.py KERNEL.s NAME [NAME ...]
(make the listing with: hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S
 -I include -I mitsuba3-sunsky_amd/csrc -o KERNEL.s mitsuba3-sunsky_amd/csrc/sunsky_kernels.hip)

Prints, per kernel: instruction count by class (VALU / transcendental / SALU / LDS /
global / branch), the most frequent opcodes, and the register/LDS/spill metadata.
"""
import re
import sys
from collections import Counter

TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32",
         "v_rcp_iflag_f32")


def classify(op):
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def main():
    text = open(sys.argv[1]).read()
    for name in sys.argv[2:]:
        i = re.search(r"^" + re.escape(name) + r":", text, re.M).start()
        j = text.index(".Lfunc_end", i)
        ins = [l.strip() for l in text[i:j].splitlines()
               if l.startswith("\t") and not l.strip().startswith((".", ";"))]
        ops = [x.split()[0] for x in ins]
        cls = Counter(classify(o) for o in ops)
        print(f"== {name}: {len(ops)} instructions  " + "  ".join(f"{k}={v}" for k, v in sorted(cls.items())))
        print("   " + ", ".join(f"{o}:{c}" for o, c in Counter(ops).most_common(30)))
        k = text.find(".amdhsa_kernel " + name)
        meta = text[k:k + 6000] if k >= 0 else ""
        for key in ("vgpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size",
                    "vgpr_spill_count", "sgpr_spill_count"):
            m = re.search(r"\." + key + r":\s+(\d+)", meta)
            if m:
                print(f"   {key} = {m.group(1)}")


if __name__ == "__main__":
    main()
