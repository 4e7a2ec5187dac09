"""The oracle's fp32-table evaluation modes (oracle/oracle_impl.inc `oracle_round_staged_tables`,
`oracle_adopt_tables`), which split a disc lane's error into table rounding and a kernel's own
arithmetic (tests/test_gpu_disc_literal.py).  CPU only: the product's host-staged tables."""
import numpy as np
import pytest

import oracle as O
import sunsky_amd as ss
from helpers import angles_dict, fp32_sun_input, sun_cone_wo


def _disc_dirs(o32, n, seed):
    inf = o32.info()
    return sun_cone_wo(n, inf["sun_dir_local"], float(np.arccos(inf["cos_cutoff"])), seed=seed, scale=0.999)


@pytest.mark.parametrize("variant", ["rgb", "spectral"])
@pytest.mark.parametrize("elev,turb", [(45.0, 2.0), (8.0, 6.5), (2.5, 10.0)])
def test_rounded_and_adopted_tables(variant, elev, turb):
    d = angles_dict(turb, 0.3, np.deg2rad(90 - elev), 0.3, 1.0, 1.0)
    o32 = O.Oracle(d, variant, "jit", "f32")
    d64 = fp32_sun_input(d, o32)
    o64 = O.Oracle(d64, variant, "jit", "f64")
    o64r = O.Oracle(d64, variant, "jit", "f64")
    o64r.round_staged_tables()
    o64t = O.Oracle(d64, variant, "jit", "f64")
    o64t.adopt_tables(ss.SunskyEmitter(d, variant=variant, device="host"))
    wo = _disc_dirs(o32, 4096, seed=int(elev))
    lam = None if variant == "rgb" else np.repeat(np.arange(320, 721, 40, dtype=np.float32)[:, None], wo.shape[0], 1)
    a, r, t = o64.eval(-wo, lam), o64r.eval(-wo, lam), o64t.eval(-wo, lam)
    den = np.maximum(np.abs(a), 1e-30)
    # fp32 tables move a disc lane by well under the 1e-5 bar (measured <= 1.4e-6)
    assert (np.abs(r - a) / den).max() < 3e-6
    # adopting also takes the product's fp32 local sun direction as is (no fp64 renormalisation,
    # which moves limb lanes by a few 1e-6 here): the frame is the product's, bit for bit
    em = ss.SunskyEmitter(d, variant=variant, device="host")
    assert np.array_equal(o64t.info()["sun_dir_local"], em.info()["sun_dir_local"].astype(np.float64))
    assert o64t.info()["cos_cutoff"] == np.float64(np.float32(em.info()["cos_cutoff"]))
    assert o64t.info()["area_ratio"] == np.float64(np.float32(em.info()["area_ratio"]))
    assert (np.abs(t - r) / np.maximum(np.abs(r), 1e-30)).max() < 2e-5
    # sky lanes: the sky formula on the same tables, at fp32 level in every mode
    ct = np.linspace(0.05, 1, 8)
    sky = -np.stack([np.sqrt(1 - ct * ct), np.zeros(8), ct], 1).astype(np.float32)
    la = None if variant == "rgb" else np.full((1, 8), 500.0, np.float32)
    assert np.allclose(o64r.eval(sky, la), o64.eval(sky, la), rtol=2e-6)
    assert np.allclose(o64t.eval(sky, la), o64.eval(sky, la), rtol=2e-6)


def test_adopt_tables_rejects_the_wrong_variant():
    d = angles_dict(3.0, 0.3, np.deg2rad(45), 0.3, 1.0, 1.0)
    o64 = O.Oracle(d, "rgb", "jit", "f64")
    with pytest.raises(ValueError):
        o64.adopt_tables(ss.SunskyEmitter(d, variant="spectral", device="host"))


def test_adopted_area_ratio_away_from_the_default_aperture():
    """get_area_ratio (sunsky.h:99-101) in fp32 cancels in 1 - cos(half aperture): at a 5 deg
    aperture the fp32 staged ratio is ~2e-3 from the fp64 one, a scale of the whole disc term.
    The adopting oracle takes the staged ratio, so its disc lanes follow the fp32 oracle's
    scale (and the kernels', which are given that ratio)."""
    d = angles_dict(2.5, 0.3, np.deg2rad(70), 0.2, 1.0, 1.0, sun_aperture=5.0)
    o32 = O.Oracle(d, "rgb", "jit", "f32")
    d64 = fp32_sun_input(d, o32)
    o64 = O.Oracle(d64, "rgb", "jit", "f64")
    o64t = O.Oracle(d64, "rgb", "jit", "f64")
    o64t.adopt_tables(ss.SunskyEmitter(d, variant="rgb", device="host"))
    assert abs(o64.info()["area_ratio"] / o32.info()["area_ratio"] - 1) > 1e-3
    wo = _disc_dirs(o32, 2048, seed=4)
    a, b, t = o32.eval(-wo), o64.eval(-wo), o64t.eval(-wo)
    inside = (b > 0).all(axis=1)
    assert inside.sum() > 1000
    rel = lambda x, y: (np.abs(x - y) / np.abs(y))[inside].max()
    assert rel(b, a) > 1e-3            # fp32 vs fp64: the ratio's cancellation
    assert rel(t, a) < 2e-5            # the adopted ratio: fp32 arithmetic only


def test_staged_sun_state_is_the_fp32_references_bit_for_bit():
    """What o64t adopts beyond the tables -- the local sun direction, the disc cutoff and the disc
    area ratio -- is the fp32 reference restatement's own staged state, bit for bit
    (dr::normalize of the fp32 sun_direction and the fp32 frame, sunsky.cpp:923, sunsky.h:99-101),
    over random sun positions, turbidities and apertures: the disc lanes' distance from fp64
    that the staging owns is the reference's, not the product's."""
    rng = np.random.default_rng(1)
    for i in range(24):
        el, ph, turb = rng.uniform(0.2, 89.8), rng.uniform(0, 2 * np.pi), rng.uniform(1, 10)
        ap = (0.5358, 1.0, 5.0, 12.0)[i % 4]
        for variant in ("rgb", "spectral"):
            d = angles_dict(turb, ph, np.deg2rad(90 - el), 0.3, 1.0, 1.0, sun_aperture=ap)
            o = O.Oracle(d, variant, "jit", "f32").info()
            e = ss.SunskyEmitter(d, variant=variant, device="host").info()
            assert np.array_equal(np.float32(o["sun_dir_local"]), np.float32(e["sun_dir_local"])), (variant, el, ap)
            assert np.float32(o["cos_cutoff"]) == np.float32(e["cos_cutoff"]), (variant, el, ap)
            assert np.float32(o["area_ratio"]) == np.float32(e["area_ratio"]), (variant, el, ap)
