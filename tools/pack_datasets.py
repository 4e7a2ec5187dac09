#!/usr/bin/env python3
"""Pack the Hosek-Wilkie sun/sky datasets into one self-describing blob.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box).  The output, ``mitsuba3-sunsky_amd/data/sunsky_datasets.pack``,
is committed and is what the product (C++ staging) and the oracle (C) read at
run time.

Sources (data only, BSD-3 licensed Hosek-Wilkie tables, see DATA_LICENSE.txt):
  * resources/sunsky/datasets/*.bin   -- read with the header layout of
    array_from_file, include/mitsuba/render/sunsky/sunsky.h:516-561
    (char[3] magic, uint32 version, uint64 ndims, uint64 shape[ndims], payload).
  * src/core/spectrum.cpp:158 (cie1931_tbl, Y block) -- CIE 1931 Y at the
    11 model wavelengths 320..720 nm (0 outside [360, 830], spectrum.h:126-127),
    needed by luminance() in estimate_sky_sun_ratio (sunsky.cpp:858-861).

Pack layout (little endian), parsed by csrc/sunsky_dataset.cpp and
oracle/sunsky_oracle.c:
  char  magic[8] = "SSKYPAK1"
  u32   version = 1
  u32   n_entries
  entry[n_entries], 96 bytes each:
      char name[24] (NUL padded), u32 dtype (1 = f32, 2 = f64), u32 ndims,
      u64 shape[6], u64 offset (from file start), u32 nbytes_lo, u32 crc32
  payloads, each 64-byte aligned.
"""
import argparse
import os
import re
import struct
import sys
import zlib

import numpy as np

REF = "/root/reference"
DATASETS = [
    # (entry name, file, expected shape, expected dtype)
    ("sky_rgb_params", "sky_rgb_params.bin", (10, 2, 6, 3, 9), np.float64),
    ("sky_rgb_rad", "sky_rgb_rad.bin", (10, 2, 6, 3), np.float64),
    ("sky_spec_params", "sky_spec_params.bin", (10, 2, 6, 11, 9), np.float64),
    ("sky_spec_rad", "sky_spec_rad.bin", (10, 2, 6, 11), np.float64),
    ("sun_rgb_rad", "sun_rgb_rad.bin", (10, 45, 3, 4, 6), np.float64),
    ("sun_spec_rad", "sun_spec_rad.bin", (10, 45, 11, 4), np.float64),
    ("sun_spec_ld", "sun_spec_ld.bin", (11, 6), np.float64),
    ("tgmm_tables", "tgmm_tables.bin", (9, 30, 5, 5), np.float32),
]
MAGIC = b"SSKYPAK1"
ENTRY_FMT = "<24sII6QQII"
assert struct.calcsize(ENTRY_FMT) == 96


def read_reference_bin(path):
    """Restates array_from_file (sunsky.h:516-561): header then raw payload.

    The reference reads the payload as FileType (Float64 for every table but
    tgmm_tables.bin, which is Float32; sunsky.cpp:182-199); the dtype is
    inferred here from the payload size."""
    raw = open(path, "rb").read()
    magic = raw[:3]
    if magic not in (b"SKY", b"SUN"):
        raise ValueError(f"{path}: bad magic {magic!r}")
    (version,) = struct.unpack_from("<I", raw, 3)
    (ndims,) = struct.unpack_from("<Q", raw, 7)
    shape = struct.unpack_from(f"<{ndims}Q", raw, 15)
    if any(s == 0 for s in shape):
        raise ValueError(f"{path}: zero-sized dimension")
    off = 15 + 8 * ndims
    count = int(np.prod(shape))
    payload = len(raw) - off
    if payload == 8 * count:
        dt = np.float64
    elif payload == 4 * count:
        dt = np.float32
    else:
        raise ValueError(f"{path}: payload {payload} B does not match shape {shape}")
    return magic, version, tuple(int(s) for s in shape), np.frombuffer(raw, dt, count, off).reshape(shape)


def cie_y_at_nodes(spectrum_cpp):
    """CIE 1931 Y (Mitsuba's 95-sample 360..830 nm table, 5 nm step) at 320..720 step 40."""
    src = open(spectrum_cpp).read()
    start = src.index("cie1931_tbl[MI_CIE_SAMPLES * 3]")
    body = src[start:src.index("};", start)]
    vals = [float(v) for v in re.findall(r"Float\(([-0-9.eE+]+)\)", body)]
    assert len(vals) == 95 * 3, len(vals)
    y = np.array(vals[95:190], dtype=np.float32)
    out = np.zeros(11, dtype=np.float32)
    for i, lam in enumerate(range(320, 721, 40)):
        if 360 <= lam <= 830:
            out[i] = y[(lam - 360) // 5]  # lam on the 5 nm grid: exact table entry
    return out


def write_pack(path, entries):
    header = bytearray(MAGIC + struct.pack("<II", 1, len(entries)))
    table_size = len(header) + 96 * len(entries)
    offset = (table_size + 63) // 64 * 64
    blobs = []
    for name, arr in entries:
        arr = np.ascontiguousarray(arr)
        dtype = {np.dtype(np.float32): 1, np.dtype(np.float64): 2}[arr.dtype]
        shape = list(arr.shape) + [0] * (6 - arr.ndim)
        data = arr.astype(arr.dtype.newbyteorder("<")).tobytes()
        crc = zlib.crc32(data) & 0xFFFFFFFF
        header += struct.pack(ENTRY_FMT, name.encode(), dtype, arr.ndim, *shape, offset, len(data), crc)
        blobs.append((offset, data))
        offset = (offset + len(data) + 63) // 64 * 64
    out = bytearray(offset)
    out[: len(header)] = header
    for off, data in blobs:
        out[off: off + len(data)] = data
    with open(path, "wb") as f:
        f.write(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=REF)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..",
                                                  "mitsuba3-sunsky_amd", "data", "sunsky_datasets.pack"))
    args = ap.parse_args()
    ds_dir = os.path.join(args.reference, "resources", "sunsky", "datasets")
    entries = []
    for name, fn, shape, dt in DATASETS:
        _, version, got_shape, arr = read_reference_bin(os.path.join(ds_dir, fn))
        if got_shape != shape or arr.dtype != dt or version != 0:
            sys.exit(f"{fn}: unexpected layout {got_shape} {arr.dtype} v{version}")
        entries.append((name, arr))
    entries.append(("cie_y_nodes", cie_y_at_nodes(os.path.join(args.reference, "src", "core", "spectrum.cpp"))))
    write_pack(os.path.abspath(args.out), entries)
    print(f"wrote {os.path.abspath(args.out)} ({os.path.getsize(args.out)} bytes, {len(entries)} entries)")


if __name__ == "__main__":
    main()
