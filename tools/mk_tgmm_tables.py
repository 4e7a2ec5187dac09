#!/usr/bin/env python3
"""Regenerate the TGMM sampling table from the fitted mixture CSV -- a restatement
of sunsky-testing/mk_sampling_dataset.py:1-27 (which needs pandas + mitsuba):

  * drop the RMSE, MAE, Volume, Normalization and Azimuth columns;
  * sort rows by (Turbidity, Elevation), stable, keeping the 5 gaussians' order;
  * keep (Mean X, Mean Y, Sigma X, Sigma Y, Weight) and turn Mean Y from an
    elevation into a zenith angle (pi/2 - Mean Y);
  * store fp32 with shape (9 turbidities, 30 elevations, 5 gaussians, 5 params)
    through array_to_file (sunsky.h:573-597; here the C ABI's sunsky_array_to_file).

  python tools/mk_tgmm_tables.py <model_hosek.csv> <out.bin>
"""
import csv
import os
import sys

import numpy as np

SHAPE = (9, 30, 5, 5)


def tgmm_from_csv(path):
    with open(path, newline="") as fh:
        rows = list(csv.DictReader(fh))
    keep = ["Turbidity", "Elevation", "Mean X", "Mean Y", "Sigma X", "Sigma Y", "Weight"]
    arr = np.array([[float(r[k]) for k in keep] for r in rows], dtype=np.float64)
    order = np.lexsort([arr[:, 1], arr[:, 0]])          # primary: turbidity, then elevation
    simplified = arr[order, 2:].copy()
    simplified[:, 1] = np.pi / 2 - simplified[:, 1]
    if simplified.size != int(np.prod(SHAPE)):
        raise ValueError(f"{path}: {simplified.shape[0]} rows, expected {int(np.prod(SHAPE[:3]))}")
    return simplified.astype(np.float32).reshape(SHAPE)


def main():
    if len(sys.argv) != 3:
        print(__doc__)
        return 2
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "mitsuba3-sunsky_amd"))
    import sunsky_amd as ss
    table = tgmm_from_csv(sys.argv[1])
    ss.array_to_file(sys.argv[2], table.ravel(), shape=SHAPE)
    print(f"wrote {sys.argv[2]}: shape {SHAPE}, fp32")
    return 0


if __name__ == "__main__":
    sys.exit(main())
