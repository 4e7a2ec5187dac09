"""Dataset format tooling: the .bin reader/writer and the
TGMM table regeneration of sunsky-testing/mk_sampling_dataset.py.  CPU only."""
import os
import struct
import sys

import numpy as np
import pytest

import sunsky_amd as ss

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
REF = "/root/reference"
CSV = os.path.join(REF, "sunsky-testing/res/datasets/model_hosek.csv")
TGMM_BIN = os.path.join(REF, "resources/sunsky/datasets/tgmm_tables.bin")


def read_pack_entry(name):
    """The SSKYPAK1 layout documented in tools/pack_datasets.py."""
    raw = open(ss.default_dataset_path(), "rb").read()
    assert raw[:8] == b"SSKYPAK1"
    _, n = struct.unpack_from("<II", raw, 8)
    for k in range(n):
        e = struct.unpack_from("<24sII6QQII", raw, 16 + 96 * k)
        if e[0].rstrip(b"\0").decode() == name:
            dtype = {1: np.float32, 2: np.float64}[e[1]]
            shape = tuple(e[3:3 + e[2]])
            return np.frombuffer(raw, dtype, int(np.prod(shape)), e[9]).reshape(shape)
    raise KeyError(name)


@pytest.mark.skipif(not os.path.exists(CSV), reason="reference CSV not present (GPU box)")
def test_tgmm_table_regenerated_from_csv_is_bit_exact(tmp_path):
    from mk_tgmm_tables import SHAPE, tgmm_from_csv
    table = tgmm_from_csv(CSV)
    assert table.shape == SHAPE and table.dtype == np.float32
    np.testing.assert_array_equal(table, read_pack_entry("tgmm_tables"))
    out = tmp_path / "tgmm_tables.bin"
    ss.array_to_file(out, table.ravel(), shape=SHAPE)
    # the same bytes as the reference's shipped file (header + fp32 payload)
    assert out.read_bytes() == open(TGMM_BIN, "rb").read()
    np.testing.assert_array_equal(ss.array_from_file(out).astype(np.float32), table)


def test_pack_tgmm_entry_layout():
    t = read_pack_entry("tgmm_tables")
    assert t.shape == (9, 30, 5, 5)
    # weights of each (turbidity, elevation) mixture are positive, sigmas positive,
    # mean zenith angles within [0, pi/2] (mk_sampling_dataset.py's pi/2 - elevation)
    assert np.all(t[..., 4] > 0) and np.all(t[..., 2:4] > 0)


HW_DIR = os.path.join(REF, "include/mitsuba/render/sunsky")


@pytest.mark.skipif(not os.path.isdir(HW_DIR), reason="Hosek-Wilkie data headers not present (GPU box)")
def test_datasets_regenerated_from_hosek_wilkie_headers_are_bit_exact(tmp_path):
    """tools/mk_hw_datasets.py restates sunsky.h:600-932; its output must be the shipped files
    byte for byte, and the pack's entries must hold the same numbers.  All 7 Hosek-Wilkie
    tables, including the derived RGB sun table behind every RGB sun-disc lane
    (write_sun_data_rgb, sunsky.h:716-770: linear_rgb_rec over the CIE table of
    src/core/spectrum.cpp:158); with the TGMM test above, all 8 shipped files."""
    from mk_hw_datasets import generate
    names = generate(HW_DIR, str(tmp_path))
    assert len(names) == 7 and "sun_rgb_rad.bin" in names
    for name in names:
        assert (tmp_path / name).read_bytes() == open(os.path.join(REF, "resources/sunsky/datasets", name), "rb").read()
        np.testing.assert_array_equal(ss.array_from_file(tmp_path / name), read_pack_entry(name[:-4]))
