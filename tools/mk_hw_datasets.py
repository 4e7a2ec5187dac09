#!/usr/bin/env python3
"""Regenerate the sky / sun dataset files from the Hosek-Wilkie data headers
(ArHosekSkyModelData_{RGB,Spectral}.h, the published model data) -- a restatement
of the reference's generator, include/mitsuba/render/sunsky/sunsky.h:600-932
(write_sky_data, write_sun_data_spectral, write_limb_darkening_data,
write_sun_data_rgb).  Runs in the build container only (the headers live under
/root/reference); the output is checked bit-exact against the shipped .bin files by
tests/test_dataset_tools.py.

Axis reorders (sunsky.h:676-932):
  sky params  [channel][albedo][turbidity][ctrl][param] -> (turbidity, albedo, ctrl, channel, param)
  sky radiance [channel][albedo][turbidity][ctrl]       -> (turbidity, albedo, ctrl, channel)
  solar        [lambda][turbidity][segment][ctrl]       -> (turbidity, segment, lambda, ctrl),
               control points reversed within a segment
  limb darkening [lambda][6]                            -> (lambda, 6)
  solar RGB   sum over the 11 nodes of linear_rgb_rec(lambda)[c] x solar x LD_j, / 11
               -> (turbidity, segment, channel, ctrl, LD param)   (write_sun_data_rgb, :716-770)

The RGB sun table needs the ITU-R BT.709 colour matching functions Mitsuba builds at
start-up: CIE 1931 XYZ (src/core/spectrum.cpp:158, fp32) through xyz_to_srgb
(spectrum.h:405-412) in fp32, evaluated by linear_rgb_rec (spectrum.h:333-362) at the node
wavelengths, where the table index is exact (t = (lambda - 360) * 94 / 470 = 8 k) and
320 nm lies outside [360, 830] (rectifier 0).  Two roundings decide the bits:
  * Dr.Jit's matrix x vector is a fused multiply-add chain over the columns,
    r = fma(M2, z, fma(M1, y, M0 * x)), in fp32;
  * the generator's `buffer += rectifier * solar * ld` was compiled with FP contraction:
    buffer = fma(rectifier * solar, ld, buffer) in fp64.
Both are emulated exactly here (fractions), and the result is the shipped file byte for
byte; the plain (uncontracted) forms differ in up to 30 % of the entries by ~1e-16 relative.

  python tools/mk_hw_datasets.py <header dir> <out dir>
"""
import os
import re
import struct
import sys
from fractions import Fraction

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


def fma_exact(a, b, c, dtype):
    """a * b + c rounded once to `dtype` (float32 / float64), elementwise over numpy arrays."""
    a, b, c = np.broadcast_arrays(np.asarray(a, np.float64), np.asarray(b, np.float64), np.asarray(c, np.float64))
    out = np.empty(a.shape, dtype)
    for i, (x, y, z) in enumerate(zip(a.ravel(), b.ravel(), c.ravel())):
        v = Fraction(float(x)) * Fraction(float(y)) + Fraction(float(z))
        out.flat[i] = float(v) if dtype == np.float64 else np.float32(float(v)) if _f32_exact(v) else _round_f32(v)
    return out


def _f32_exact(v):
    return Fraction(float(np.float32(float(v)))) == v


def _round_f32(v):
    """Round the exact rational v to the nearest float32 (ties to even), without the double
    rounding of float() followed by np.float32()."""
    lo = np.float32(float(v))
    if Fraction(float(lo)) > v:
        lo = np.nextafter(lo, np.float32(-np.inf))
    hi = np.nextafter(lo, np.float32(np.inf))
    dl, dh = v - Fraction(float(lo)), Fraction(float(hi)) - v
    if dl != dh:
        return lo if dl < dh else hi
    return lo if (lo.view(np.uint32) & 1) == 0 else hi


XYZ_TO_SRGB = np.array([[3.240479, -1.537150, -0.498535],    # spectrum.h:408-410 (fp32 literals)
                        [-0.969256, 1.875991, 0.041556],
                        [0.055648, -0.204043, 1.057311]], dtype=np.float32)


def cie1931_xyz_table(spectrum_cpp):
    """Mitsuba's 95-sample CIE 1931 XYZ table (src/core/spectrum.cpp:158, Float = float): (3, 95)."""
    src = open(spectrum_cpp).read()
    start = src.index("cie1931_tbl[MI_CIE_SAMPLES * 3]")
    body = src[start:src.index("};", start)]
    vals = [float(v) for v in re.findall(r"Float\(([-0-9.eE+]+)\)", body)]
    assert len(vals) == 95 * 3, len(vals)
    return np.array(vals, dtype=np.float32).reshape(3, 95)


def srgb_tables(xyz):
    """CIE1932Tables::srgb = xyz_to_srgb(xyz) (spectrum.h:179, 405-412): the fp32 matrix x
    vector as Dr.Jit evaluates it, an fma chain over the columns."""
    M = XYZ_TO_SRGB
    rows = []
    for i in range(3):
        r = (M[i, 0] * xyz[0]).astype(np.float32)
        r = fma_exact(M[i, 1], xyz[1], r, np.float32)
        rows.append(fma_exact(M[i, 2], xyz[2], r, np.float32))
    return np.stack(rows)


def linear_rgb_rec_at_nodes(srgb):
    """linear_rgb_rec(lambda) (spectrum.h:333-362) in fp64 at the 11 node wavelengths
    320:40:720: t = (lambda - 360) * 94 / 470 is the integer 8 k at every node >= 360 (the
    fmadd(w0, v0, w1 v1) returns v0), and 320 nm is outside [360, 830] (masked to 0)."""
    rec = np.zeros((NB_WAVELENGTHS, 3))
    for lam_idx, lam in enumerate(range(320, 721, 40)):
        if lam >= 360:
            t = (lam - 360.0) * (94 / (830.0 - 360.0))
            assert t == int(t)
            rec[lam_idx] = srgb[:, int(t)].astype(np.float64)
    return rec


def sun_rgb_table(solar, ld, rec):
    """write_sun_data_rgb (sunsky.h:716-770): per (turbidity, segment, channel, ctrl, LD j)
    the fused accumulation over the 11 nodes of rec[c] * solar * ld[j], then / 11."""
    out = np.zeros((NB_TURBIDITY, NB_SUN_SEGMENTS, 3, NB_SUN_CTRL, NB_LD))
    for lam in range(NB_WAVELENGTHS):
        a = rec[lam][None, None, :, None, None] * solar[:, :, lam, None, :, None]
        out = fma_exact(a, ld[lam][None, None, None, None, :], out, np.float64)
    return out / NB_WAVELENGTHS


def write_bin(path, magic, table):
    """FileStream layout of array_to_file / the writers: char[3], u32 0, u64 ndims, u64 shape, f64 payload."""
    with open(path, "wb") as fh:
        fh.write(magic)
        fh.write(struct.pack("<I", 0))
        fh.write(struct.pack("<Q", table.ndim))
        fh.write(struct.pack(f"<{table.ndim}Q", *table.shape))
        fh.write(np.ascontiguousarray(table, dtype="<f8").tobytes())


def generate(header_dir, out_dir, spectrum_cpp=None):
    """Write the dataset files; the RGB sun table too when Mitsuba's spectrum.cpp (the CIE
    table) is given or found at <header_dir>/../../../../src/core/spectrum.cpp."""
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
    if spectrum_cpp is None:
        spectrum_cpp = os.path.join(header_dir, "..", "..", "..", "..", "src", "core", "spectrum.cpp")
    if os.path.exists(spectrum_cpp):
        rec = linear_rgb_rec_at_nodes(srgb_tables(cie1931_xyz_table(spectrum_cpp)))
        outputs["sun_rgb_rad.bin"] = (b"SUN", sun_rgb_table(outputs["sun_spec_rad.bin"][1],
                                                            outputs["sun_spec_ld.bin"][1], rec))
    for name, (magic, table) in outputs.items():
        write_bin(os.path.join(out_dir, name), magic, table)
    return sorted(outputs)


if __name__ == "__main__":
    if len(sys.argv) != 3:
        print(__doc__)
        sys.exit(2)
    for n in generate(sys.argv[1], sys.argv[2]):
        print("wrote", os.path.join(sys.argv[2], n))
