"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM
traffic per kernel (MI355X_MICROARCH.md "HBM": FETCH_SIZE counts 1/2 of the
bytes of a 16-B/lane streaming read on gfx950 -> x2; WRITE_SIZE exact for
16-B/lane streaming stores; both in KiB).

  python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024.0)
    return vals


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) & set(write)):
        if not k.startswith("sunsky_"):
            continue
        # first launch of each kernel runs on cold TLBs / caches: report the steady-state mean
        f = fetch[k][1:] or fetch[k]
        w = write[k][1:] or write[k]
        fr = sum(f) / len(f)
        wr = sum(w) / len(w)
        out[k] = {"launches": len(fetch[k]), "fetch_size_bytes_raw": fr, "fetch_bytes_x2": 2 * fr,
                  "write_bytes": wr, "traffic_bytes": 2 * fr + wr,
                  "correction": "FETCH_SIZE x2 (gfx950 wide streaming read), WRITE_SIZE as is; KiB -> bytes"}
    with open(sys.argv[3], "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in out.items():
        print(f"{k:40s} launches={v['launches']:3d} fetch(x2)={v['fetch_bytes_x2']/1e6:9.2f} MB "
              f"write={v['write_bytes']/1e6:9.2f} MB traffic={v['traffic_bytes']/1e6:9.2f} MB")


if __name__ == "__main__":
    main()
