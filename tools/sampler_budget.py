#!/usr/bin/env python3
"""Instruction budget of the FAST RGB sample_direction per phase.

Compiles tools/sampler_budget.hip (one kernel per phase of sample_one_rgb) to a gfx950 listing
and counts each kernel's VALU / transcendental / SALU / LDS instructions outside the staging
baseline, with the instructions of every loop inside the phase listed per trip (the TGMM sum
runs ceil(live gaussians / 2) pair trips: 5 at the C4 emitter, T = 3).

usage: python tools/sampler_budget.py [--tgmm-trips 5]
"""
import argparse
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from isa_summary import classify  # noqa: E402

KERNELS = ["budget_baseline", "budget_sky_direction", "budget_sky_pdf", "budget_sky_eval", "budget_sky_pick",
           "budget_sun_pick"]


def listing():
    out = "/tmp/sampler_budget.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                           "-DSS_XFORM_IDENTITY", "-I", os.path.join(ROOT, "include"), "-I",
                           os.path.join(ROOT, "mitsuba3-sunsky_amd", "csrc"), "-o", out,
                           os.path.join(HERE, "sampler_budget.hip")])
    return open(out).read().split("\n")


def kernel_lines(lines, name):
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def count(body):
    c = {"valu": 0, "trans": 0, "salu": 0, "lds": 0, "vmem": 0, "branch": 0}
    for l in body:
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        k = classify(t.split()[0])
        if k in c:
            c[k] += 1
    return c


def loops(body):
    """(header label, instruction lines of the innermost loop bodies) by the compiler's loop comments."""
    res, cur, depth_lines = [], None, []
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):.*Inner Loop Header", l) or re.match(r"^(\.LBB\w+):.*=>This Loop Header", l)
        if m:
            cur, depth_lines = m.group(1), []
            continue
        if cur:
            depth_lines.append(l)
            if re.search(r"s_cbranch_\w+\s+" + re.escape(cur) + r"\b", l):
                res.append((cur, depth_lines))
                cur = None
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tgmm-trips", type=int, default=5)
    args = ap.parse_args()
    lines = listing()
    base = count(kernel_lines(lines, "budget_baseline"))
    print(f"{'phase':24s} {'VALU':>6s} {'trans':>6s} {'SALU':>6s} {'LDS':>5s}   loops (per trip)")
    for k in KERNELS[1:]:
        body = kernel_lines(lines, k)
        c = count(body)
        d = {x: c[x] - base[x] for x in c}
        ls = []
        for lab, lb in loops(body):
            lc = count(lb)
            if lc["valu"] + lc["trans"] > 4:
                ls.append(f"{lab}: {lc['valu']} VALU + {lc['trans']} trans + {lc['lds']} LDS")
        print(f"{k:24s} {d['valu']:6d} {d['trans']:6d} {d['salu']:6d} {d['lds']:5d}   " + "; ".join(ls))


if __name__ == "__main__":
    main()
