"""Per-kernel averages of the counters collected by tools/gpu_spec_pmc.sh (all passes):
counters per dispatch and per wave, plus VALU-active / wave-cycle ratios.
usage: python tools/spmc_summary.py gpurun_out/spmc"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(lambda: defaultdict(float))
    nd = defaultdict(lambda: defaultdict(set))
    for p in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k, c = r["Kernel_Name"], r["Counter_Name"]
            if not k.startswith("sunsky_"):
                continue
            acc[k][c] += float(r["Counter_Value"])
            nd[k][c].add(r["Dispatch_Id"])
    out = {}
    for k, cs in acc.items():
        per = {c: v / len(nd[k][c]) for c, v in cs.items()}
        waves = per.get("SQ_WAVES")
        rec = {"per_dispatch": per}
        if waves:
            rec["per_wave"] = {c: v / waves for c, v in per.items() if c.startswith("SQ_INSTS") or c.startswith("SQ_LDS")}
        if per.get("SQ_WAVE_CYCLES"):
            rec["valu_active_over_wave_cycles"] = per.get("SQ_ACTIVE_INST_VALU", 0) / per["SQ_WAVE_CYCLES"]
        if per.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_bank_conflict_over_active"] = per.get("SQ_LDS_BANK_CONFLICT", 0) / per["SQ_LDS_IDX_ACTIVE"]
        if per.get("SQ_WAIT_ANY"):
            rec["wait_inst_lds_over_wait_any"] = per.get("SQ_WAIT_INST_LDS", 0) / per["SQ_WAIT_ANY"]
        out[k] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
