"""Per-kernel SQ counter ratios from rocprofv3 --pmc CSVs (tools/gpu_sqpmc.sh).
SQ_* cycle counters are quad-cycles on gfx950 (MI355X_MICROARCH.md); ratios are unit-free."""
import csv
import sys
from collections import defaultdict


def main(paths):
    for p in paths:
        acc = defaultdict(lambda: defaultdict(float))
        n = defaultdict(set)
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
        for k, c in acc.items():
            d = len(n[k])
            wc = c["SQ_WAVE_CYCLES"]
            print(f"{k}  dispatches={d}")
            print(f"  per dispatch: VALU insts {c['SQ_INSTS_VALU'] / d:.4g}  LDS insts {c['SQ_INSTS_LDS'] / d:.4g}"
                  f"  wave-cycles {wc / d:.4g}")
            for name in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                         "SQ_WAIT_INST_LDS"):
                print(f"  {name:22s} / WAVE_CYCLES = {c[name] / wc:.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
