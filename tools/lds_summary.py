#!/usr/bin/env python3
"""Per-dispatch LDS counters of rocprofv3 --pmc passes over kbench (tools/gpu_cmd_*.sh `lds`):
SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE, SQ_INSTS_LDS, SQ_WAIT_INST_LDS, SQ_WAVE_CYCLES, SQ_WAVES
of the last dispatch of each run (counters summed over the dimension rows).

usage: python tools/lds_summary.py gpurun_out/pmc_lds > profiles/rNN_vM_lds_conflicts.json
"""
import collections
import csv
import glob
import json
import os
import sys

out = {}
for d in sorted(glob.glob(os.path.join(sys.argv[1], "*", ""))):
    name = os.path.basename(os.path.normpath(d))
    files = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not files:
        continue
    byd = collections.defaultdict(lambda: collections.defaultdict(float))
    kern = {}
    for r in csv.DictReader(open(files[0])):
        byd[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        kern[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    last = max(byd)
    out[name] = dict(kernel=kern[last], dispatches=len(byd), **{k: v for k, v in byd[last].items()})
json.dump(out, sys.stdout, indent=1)
print()
