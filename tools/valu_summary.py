"""VALU roofline of kernels from rocprofv3 --pmc CSVs (tools/gpu_valu.sh).

Per dispatch: VALU wave-instructions N (SQ_INSTS_VALU), of which transcendental T
(SQ_INSTS_VALU_TRANS_F32).  A SIMD issues a plain wave64 VALU instruction in 2 cycles and
a transcendental in 8 (tools/valu_probe.hip on MI355X, DESIGN.md §3: ~2.6 / ~8 measured;
MI355X_MICROARCH.md: 32 lanes / cycle), so the VALU-issue floor of a launch is
    t_valu = ((N - T) * 2 + T * 8) / (1024 SIMDs * f_clk),  f_clk = 2.4 GHz,
and frac = t_valu / t_kernel (t_kernel from the kbench run's rocprof kernel trace, or given).
Prints JSON keyed by kernel."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS, CLK = 1024, 2.4e9
PLAIN, TRANS = 2.0, 8.0


def kernel_ms(trace_glob):
    dur = defaultdict(list)
    for p in glob.glob(trace_glob):
        for r in csv.DictReader(open(p)):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return dur


def main(root):
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "*/"))):
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        acc = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for p in files:
            for r in csv.DictReader(open(p)):
                k = r["Kernel_Name"]
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
        for k, c in acc.items():
            nd = len(disp[k])
            if "SQ_WAIT_ANY" in c:   # the stall pass (gpu_valu.sh C2): where the wave cycles go
                wc = c["SQ_WAVE_CYCLES"]
                out.setdefault(k, {}).update({
                    "stall": {"wait_any_frac": c["SQ_WAIT_ANY"] / wc, "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / wc,
                              "active_inst_any_frac": c["SQ_ACTIVE_INST_ANY"] / wc,
                              "wait_inst_lds_frac": c["SQ_WAIT_INST_LDS"] / wc,
                              "active_inst_valu_frac": c["SQ_ACTIVE_INST_VALU"] / wc,
                              "active_inst_lds_frac": c["SQ_ACTIVE_INST_LDS"] / wc,
                              "lds_bank_conflict_per_dispatch": c["SQ_LDS_BANK_CONFLICT"] / nd,
                              "note": "fractions of SQ_WAVE_CYCLES: WAIT_ANY = parked on s_waitcnt / barrier, "
                                      "WAIT_INST_ANY = issue stalls, ACTIVE_INST_ANY = issuing (disjoint, "
                                      "MI355X_MICROARCH.md PMC table)"}})
                continue
            N, T = c["SQ_INSTS_VALU"] / nd, c["SQ_INSTS_VALU_TRANS_F32"] / nd
            waves = c["SQ_WAVES"] / nd
            t_valu = ((N - T) * PLAIN + T * TRANS) / (SIMDS * CLK)
            rec = {"dispatches": nd, "valu_wave_insts": N, "trans_wave_insts": T, "waves": waves,
                   "valu_per_wave": N / waves if waves else None, "trans_per_wave": T / waves if waves else None,
                   "salu_per_wave": c["SQ_INSTS_SALU"] / nd / waves if waves else None,
                   "lds_per_wave": c["SQ_INSTS_LDS"] / nd / waves if waves else None,
                   "valu_active_over_wave_cycles": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"],
                   "valu_issue_floor_ms": t_valu * 1e3,
                   "grbm_gui_active_per_dispatch": c["GRBM_GUI_ACTIVE"] / nd}
            # kernel time from the kbench log of the same pass (first timing line)
            log = d.rstrip("/") + ".log"
            if os.path.exists(log):
                for line in open(log):
                    if line.startswith(k) and " us " in line:
                        us = float(line.split(" us ")[0].split()[-1])
                        rec["kernel_ms"] = us * 1e-3
                        rec["valu_frac"] = t_valu * 1e3 / rec["kernel_ms"]
                        break
            out.setdefault(k, {}).update(rec)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/valu")
