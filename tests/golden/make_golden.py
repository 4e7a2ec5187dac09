#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the
reference's own test data.  Runs in the build container only (it reads
/root/reference); the GPU box uses the committed .npz files.

Fixtures (data only -- inputs and expected outputs):
  * sun_spectra.npz  -- the 80 ``sun_spectrum_t*_eta*_gamma*.spd`` files of
    resources/sunsky/test_data/spectrum (test04, test_sunsky.py:149-196).
    Inputs are reconstructed exactly as the test builds them:
    turb in linspace(1, 10, 5), eta in linspace(1e-4, pi/2 - 1e-4, 4),
    gamma in linspace(0, deg2rad(0.5388/2) - 1e-4, 4), lambda = linspace(310, 800, 15).
    The values were produced by mi.hosek_sun_rad (sunsky_v.cpp:19 ->
    ArHosekSkyModel.c:686-784), fp64 rounded to fp32.
  * sky_renders.npz  -- the 7 EXR renders of resources/sunsky/test_data/renders
    (test01-03, test_sunsky.py:62-145) decoded to float32 arrays with the same
    channel order as mi.TensorXf(mi.Bitmap(path)) (RGB -> R,G,B; spectral ->
    the 10 bands in ascending wavelength).
"""
import glob
import os
import re
import struct
import zlib

import numpy as np

REF = "/root/reference/resources/sunsky/test_data"
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------- EXR decode
def _read_attrs(buf, pos):
    attrs = {}
    while True:
        end = buf.index(b"\0", pos)
        name = buf[pos:end].decode()
        pos = end + 1
        if not name:
            return attrs, pos
        end = buf.index(b"\0", pos)
        typ = buf[pos:end].decode()
        pos = end + 1
        (size,) = struct.unpack_from("<i", buf, pos)
        pos += 4
        attrs[name] = (typ, buf[pos:pos + size])
        pos += size


def _chlist(data):
    chans, pos = [], 0
    while data[pos] != 0:
        end = data.index(b"\0", pos)
        name = data[pos:end].decode()
        pos = end + 1
        ptype, _plin, _xs, _ys = struct.unpack_from("<iBxxxii", data, pos)
        pos += 16
        chans.append((name, ptype))
    return chans


def decode_exr(path):
    """Minimal OpenEXR reader: single-part scanline, NO/ZIPS/ZIP compression,
    HALF/FLOAT channels.  Returns {channel: (H, W) float32}."""
    buf = open(path, "rb").read()
    magic, version = struct.unpack_from("<ii", buf, 0)
    assert magic == 20000630, "not an OpenEXR file"
    assert (version & 0x200) == 0, "tiled EXR not supported"
    attrs, pos = _read_attrs(buf, 8)
    chans = _chlist(attrs["channels"][1])
    comp = attrs["compression"][1][0]
    xmin, ymin, xmax, ymax = struct.unpack("<iiii", attrs["dataWindow"][1])
    w, h = xmax - xmin + 1, ymax - ymin + 1
    lines_per_block = {0: 1, 2: 1, 3: 16}[comp]
    nblocks = (h + lines_per_block - 1) // lines_per_block
    offsets = struct.unpack_from(f"<{nblocks}Q", buf, pos)
    sizes = {1: 2, 2: 4}
    out = {name: np.zeros((h, w), np.float32) for name, _ in chans}
    for off in offsets:
        y, dsize = struct.unpack_from("<ii", buf, off)
        data = buf[off + 8: off + 8 + dsize]
        nlines = min(lines_per_block, ymax - y + 1)
        expect = nlines * w * sum(sizes[t] for _, t in chans)
        if comp in (2, 3) and dsize < expect:
            raw = np.frombuffer(zlib.decompress(data), np.uint8).astype(np.int32)
            # predictor: t[i] = t[i-1] + t[i] - 128
            t = np.cumsum(np.concatenate([[raw[0]], raw[1:] - 128])) & 0xFF
            t = t.astype(np.uint8)
            half = (len(t) + 1) // 2
            inter = np.empty_like(t)
            inter[0::2] = t[:half]
            inter[1::2] = t[half:]
            data = inter.tobytes()
        p = 0
        for line in range(nlines):
            for name, ptype in chans:
                n = w * sizes[ptype]
                row = np.frombuffer(data[p:p + n], np.float16 if ptype == 1 else np.float32)
                out[name][y - ymin + line] = row.astype(np.float32)
                p += n
    return out


def exr_to_tensor(path):
    ch = decode_exr(path)
    names = list(ch.keys())
    if set(names) >= {"R", "G", "B"}:
        order = ["R", "G", "B"]
    else:
        def wl(n):
            m = re.search(r"([0-9]+(?:\.[0-9]+)?)", n.replace(",", "."))
            return float(m.group(1))
        order = sorted(names, key=wl)
    return np.stack([ch[n] for n in order], axis=-1), order


def main():
    # ---- sun spectra (test04)
    eps = 1e-4
    half = np.deg2rad(0.5388 / 2.0)
    wl = np.linspace(310, 800, 15)
    rows = []
    for turb in np.linspace(1, 10, 5):
        for eta in np.linspace(eps, np.pi / 2 - eps, 4):
            for gamma in np.linspace(0, half - eps, 4):
                fn = os.path.join(REF, "spectrum",
                                  f"sun_spectrum_t{turb:.1f}_eta{eta:.2f}_gamma{gamma:.3e}.spd")
                data = np.loadtxt(fn)
                assert np.allclose(data[:, 0], wl)
                rows.append((turb, eta, gamma, data[:, 1]))
    assert len(rows) == len(glob.glob(os.path.join(REF, "spectrum", "*.spd"))) == 80
    np.savez_compressed(
        os.path.join(OUT, "sun_spectra.npz"),
        turbidity=np.array([r[0] for r in rows]), eta=np.array([r[1] for r in rows]),
        gamma=np.array([r[2] for r in rows]), wavelengths=wl,
        radiance=np.array([r[3] for r in rows], dtype=np.float32))

    # ---- sky renders (test01-03)
    renders = {}
    for fn in sorted(glob.glob(os.path.join(REF, "renders", "*.exr"))):
        key = os.path.splitext(os.path.basename(fn))[0]
        tensor, order = exr_to_tensor(fn)
        renders[key] = tensor
        print(key, tensor.shape, order)
    np.savez_compressed(os.path.join(OUT, "sky_renders.npz"), **renders)
    print("wrote", os.path.join(OUT, "sun_spectra.npz"), os.path.join(OUT, "sky_renders.npz"))


if __name__ == "__main__":
    main()
