#!/usr/bin/env python3
"""Regenerate the sky / sun dataset files from the Hosek-Wilkie data headers
(ArHosekSkyModelData_{RGB,Spectral}.h, the published model data) -- a restatement
of the reference's generator, include/mitsuba/render/sunsky/sunsky.h:600-932
(write_sky_data, write_sun_data_spectral, write_limb_darkening_data).  Runs in
the build container only (the headers live under /root/reference); the output
is checked bit-exact against the shipped .bin files by tests/test_dataset_tools.py.

Axis reorders (sunsky.h:676-932):
  sky params  [channel][albedo][turbidity][ctrl][param] -> (turbidity, albedo, ctrl, channel, param)
  sky radiance [channel][albedo][turbidity][ctrl]       -> (turbidity, albedo, ctrl, channel)
  solar        [lambda][turbidity][segment][ctrl]       -> (turbidity, segment, lambda, ctrl),
               control points reversed within a segment
  limb darkening [lambda][6]                            -> (lambda, 6)
The RGB sun table (sun_rgb_rad.bin) is a derived product (linear_rgb_rec of the
spectral solar data, sunsky.h:716-770) and is not regenerated here.

  python tools/mk_hw_datasets.py <header dir> <out dir>
"""
import os
import re
import struct
import sys

import numpy as np

NB_TURBIDITY, NB_ALBEDO, NB_CTRL, NB_PARAMS = 10, 2, 6, 9
NB_WAVELENGTHS, NB_SUN_SEGMENTS, NB_SUN_CTRL, NB_LD = 11, 45, 4, 6

_ARRAY = re.compile(r"double\s+(\w+)\s*\[\s*\]\s*=\s*\{(.*?)\}\s*;", re.S)
_PTRS = re.compile(r"double\s*\*\s*(\w+)\s*\[\s*\]\s*=\s*\{(.*?)\}\s*;", re.S)


def parse_header(path):
    """-> (arrays: name -> float64 ndarray, pointer tables: name -> [array names])."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    arrays = {m.group(1): np.array([float(v) for v in m.group(2).replace("\n", " ").split(",") if v.strip()])
              for m in _ARRAY.finditer(text)}
    ptrs = {m.group(1): [v.strip() for v in m.group(2).split(",") if v.strip()] for m in _PTRS.finditer(text)}
    return arrays, ptrs


def sky_table(channels, nb_params):
    """write_sky_data (sunsky.h:878-930)."""
    nch = len(channels)
    out = np.zeros((NB_TURBIDITY, NB_ALBEDO, NB_CTRL, nch, nb_params))
    for c, data in enumerate(channels):
        src = data.reshape(NB_ALBEDO, NB_TURBIDITY, NB_CTRL, nb_params)
        out[:, :, :, c, :] = src.transpose(1, 0, 2, 3)
    return out if nb_params > 1 else out[..., 0]


def solar_table(solar):
    """write_sun_data_spectral (sunsky.h:845-876): control points reversed per segment."""
    out = np.zeros((NB_TURBIDITY, NB_SUN_SEGMENTS, NB_WAVELENGTHS, NB_SUN_CTRL))
    for lam, data in enumerate(solar):
        src = data.reshape(NB_TURBIDITY, NB_SUN_SEGMENTS, NB_SUN_CTRL)
        out[:, :, lam, :] = src[:, :, ::-1]
    return out


def write_bin(path, magic, table):
    """FileStream layout of array_to_file / the writers: char[3], u32 0, u64 ndims, u64 shape, f64 payload."""
    with open(path, "wb") as fh:
        fh.write(magic)
        fh.write(struct.pack("<I", 0))
        fh.write(struct.pack("<Q", table.ndim))
        fh.write(struct.pack(f"<{table.ndim}Q", *table.shape))
        fh.write(np.ascontiguousarray(table, dtype="<f8").tobytes())


def generate(header_dir, out_dir):
    rgb, rgb_p = parse_header(os.path.join(header_dir, "ArHosekSkyModelData_RGB.h"))
    spec, spec_p = parse_header(os.path.join(header_dir, "ArHosekSkyModelData_Spectral.h"))
    pick = lambda arrays, ptrs, name: [arrays[n] for n in ptrs[name]]   # noqa: E731
    os.makedirs(out_dir, exist_ok=True)
    outputs = {
        "sky_rgb_params.bin": (b"SKY", sky_table(pick(rgb, rgb_p, "datasetsRGB"), NB_PARAMS)),
        "sky_rgb_rad.bin": (b"SKY", sky_table(pick(rgb, rgb_p, "datasetsRGBRad"), 1)),
        "sky_spec_params.bin": (b"SKY", sky_table(pick(spec, spec_p, "datasets"), NB_PARAMS)),
        "sky_spec_rad.bin": (b"SKY", sky_table(pick(spec, spec_p, "datasetsRad"), 1)),
        "sun_spec_rad.bin": (b"SUN", solar_table(pick(spec, spec_p, "solarDatasets"))),
        "sun_spec_ld.bin": (b"SUN", np.stack(pick(spec, spec_p, "limbDarkeningDatasets"))),
    }
    for name, (magic, table) in outputs.items():
        write_bin(os.path.join(out_dir, name), magic, table)
    return sorted(outputs)


if __name__ == "__main__":
    if len(sys.argv) != 3:
        print(__doc__)
        sys.exit(2)
    for n in generate(sys.argv[1], sys.argv[2]):
        print("wrote", os.path.join(sys.argv[2], n))
