"""CPU-side checks of the product boundary: the C-ABI library loads and
exports every symbol include/sunsky_amd.h declares, and the host staging
(no device) matches the oracle's restatement of the reference staging."""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
import sunsky_amd as ss
from helpers import SPECIAL_ALBEDO, angles_dict, hour_dict, sun_cone_wo

REF_DATASETS = "/root/reference/resources/sunsky/datasets"


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(ss.LIB_PATH)
    declared = ss.declared_functions()
    assert len(declared) >= 30
    missing = [f for f in declared if not hasattr(L, f)]
    assert not missing, missing
    assert ss.lib().sunsky_abi_version() == 7
    assert os.path.exists(ss.CODE_OBJECT), "gfx950 code object not built"
    assert os.path.exists(ss.CODE_OBJECT_IDENT), "identity-to_world gfx950 code object not built"


def test_default_dataset_path_resolves_to_bundled_pack():
    p = ss.default_dataset_path()
    assert os.path.exists(p) and p.endswith("sunsky_datasets.pack")


CASES = [
    ("rgb", "jit", hour_dict(3, 11.7753, 0.1, 1.0, 1.0)),
    ("rgb", "jit", angles_dict(2.0, 0.3, np.deg2rad(45), 0.1, 1.0, 1.0)),
    ("rgb", "scalar", angles_dict(6.0, -1.2, np.deg2rad(70), 0.5, 1.0, 1.0)),
    ("rgb", "jit", angles_dict(10.0, 2.0, np.deg2rad(20), [0.1, 0.5, 0.9], 0.7, 1.3)),
    ("spectral", "jit", angles_dict(3.0, 0.0, np.deg2rad(30), 0.3, 1.0, 1.0)),
    ("spectral", "jit", angles_dict(4.2, 0.0, np.deg2rad(30), SPECIAL_ALBEDO, 1.0, 1.0)),
    ("spectral", "scalar", hour_dict(5.2, 9.5, 0.2, 1.0, 1.0)),
    ("rgb", "jit", dict(angles_dict(3.0, 0.5, np.deg2rad(40), 0.3, 1.0, 1.0), sun_aperture=30.0)),
]


@pytest.mark.parametrize("variant,semantics,d", CASES)
def test_host_staging_matches_oracle(variant, semantics, d):
    em = ss.SunskyEmitter(d, variant=variant, semantics=semantics, device="host")
    o = O.Oracle(d, variant, semantics, "f32").info()
    inf = em.info()
    np.testing.assert_allclose(inf["sun_dir_world"], o["sun_dir_world"], rtol=0, atol=2e-7)
    np.testing.assert_allclose(inf["sun_angles"], o["sun_angles"], rtol=0, atol=2e-7)
    nch = 11 if variant == "spectral" else 3
    np.testing.assert_allclose(em.table("sky_params").reshape(nch, 9), o["sky_params"], rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(em.table("sky_radiance"), o["sky_radiance"], rtol=2e-6)
    sun = em.table("sun_radiance")
    np.testing.assert_array_equal(sun, O.Oracle(d, variant, semantics, "f32").sun_table())
    np.testing.assert_allclose(em.table("gaussians").reshape(20, 5), o["gaussians"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(em.table("gaussian_cdf"), o["gauss_cdf"], rtol=1e-6)
    # The sampling weight is a 200x200 fp32 quadrature; the product reduces it as a tree
    # per row then row by row, the oracle adds the fp32 terms exactly (oracle/sunsky_oracle.c
    # g_quad_sum_sequential): measured 2.9e-7 (w_sky) / 5.6e-7 (nodes) apart over 86 emitters
    # (DESIGN.md §6 "Sampling state")
    assert abs(inf["w_sky"] - o["w_sky"]) <= 1e-6 * max(1e-3, abs(o["w_sky"]))
    if variant == "spectral":
        np.testing.assert_allclose(em.table("spectral_pdf"), o["spec_pdf"], rtol=1e-6)
        np.testing.assert_allclose(em.table("spectral_cdf"), o["spec_cdf"], rtol=1e-6)
    assert inf["flags"] == (0x04 | 0x10)


@pytest.mark.parametrize("variant,semantics,d", [c for c in CASES if c[0] == "spectral"])
def test_adopted_spectral_nodes_rebuild_the_products_cdf(variant, semantics, d):
    """The oracle adopts the product's wavelength-distribution nodes (sunsky.cpp:870-885) and
    rebuilds the CDF with its own compute_cdf restatement (distr_1d.h:513-585): the result
    equals the product's staged CDF bit for bit, so the GPU wavelength-sampling tests compare
    the sampling kernels alone."""
    em = ss.SunskyEmitter(d, variant=variant, semantics=semantics, device="host")
    o = O.Oracle(d, variant, semantics, "f32")
    o.override_spectral_distr(em.table("spectral_pdf"))
    inf = o.info()
    np.testing.assert_array_equal(inf["spec_pdf"].astype(np.float32), em.table("spectral_pdf"))
    np.testing.assert_array_equal(inf["spec_cdf"].astype(np.float32), em.table("spectral_cdf"))
    with pytest.raises(ValueError, match="spectral pdf"):
        o.override_spectral_distr(np.array([1.0, -1.0]))
    with pytest.raises(ValueError, match="size"):
        o.override_spectral_distr(np.ones(11))


def test_parameter_errors_match_reference_messages():
    with pytest.raises(ValueError, match="Turbidity value"):
        ss.SunskyEmitter({"turbidity": 0.5}, device="host")
    with pytest.raises(ValueError, match="Invalid sun scale"):
        ss.SunskyEmitter({"sun_scale": -1.0}, device="host")
    with pytest.raises(ValueError, match="Invalid sky scale"):
        ss.SunskyEmitter({"sky_scale": -1.0}, device="host")
    with pytest.raises(ValueError, match="Invalid sun aperture"):
        ss.SunskyEmitter({"sun_aperture": 180.0}, device="host")
    with pytest.raises(ValueError, match="Albedo values must be in"):
        ss.SunskyEmitter({"albedo": 1.5}, device="host")
    with pytest.raises(ValueError, match="Both the 'sun_direction'"):
        ss.SunskyEmitter({"sun_direction": [0, 0, 1], "hour": 12.0}, device="host")
    with pytest.raises(ValueError, match="Unreferenced property"):
        ss.SunskyEmitter({"turbidty": 3.0}, device="host")
    with pytest.raises(FileNotFoundError):
        ss.SunskyEmitter({}, device="host", dataset_path="/nonexistent/sunsky.pack")


def test_parameters_changed_restages_like_construction():
    d = angles_dict(3.0, 0.2, np.deg2rad(50), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, device="host")
    params = em.traverse()
    params["turbidity"] = 7.5
    params["albedo"] = 0.6
    params.update()
    d2 = dict(d, turbidity=7.5, albedo=0.6)
    fresh = ss.SunskyEmitter(d2, device="host")
    np.testing.assert_array_equal(em.table("sky_params"), fresh.table("sky_params"))
    np.testing.assert_array_equal(em.table("sun_radiance"), fresh.table("sun_radiance"))
    assert em.sky_sampling_w == fresh.sky_sampling_w
    with pytest.raises(ValueError, match="Turbidity"):
        params["turbidity"] = 20.0
        params.update()


def test_time_location_parameters_update_sun():
    em = ss.SunskyEmitter(hour_dict(3, 12.0, 0.2, 1.0, 1.0), device="host")
    p = em.traverse()
    p["hour"] = 17.0
    p.update()
    ref = O.sun_coordinates(hour=17.0)
    np.testing.assert_allclose(em.info()["sun_dir_world"], ref, atol=2e-7)


def test_array_file_roundtrip(tmp_path):
    data = np.arange(24, dtype=np.float32) * 0.5
    f = tmp_path / "t.bin"
    ss.array_to_file(f, data, (2, 3, 4))
    back = ss.array_from_file(f)
    assert back.shape == (2, 3, 4)
    np.testing.assert_array_equal(back.reshape(-1), data)
    raw = open(f, "rb").read()
    assert raw[:3] == b"SKY"


@pytest.mark.skipif(not os.path.isdir(REF_DATASETS), reason="reference tree not mounted (GPU box)")
def test_reference_bin_directory_equals_bundled_pack():
    for variant in ("rgb", "spectral"):
        d = angles_dict(4.0, 0.0, np.deg2rad(35), 0.25, 1.0, 1.0)
        a = ss.SunskyEmitter(d, variant=variant, device="host")
        b = ss.SunskyEmitter(d, variant=variant, device="host", dataset_path=REF_DATASETS)
        for t in ("sky_params", "sky_radiance", "sun_radiance", "gaussians"):
            np.testing.assert_array_equal(a.table(t), b.table(t))
        assert a.sky_sampling_w == b.sky_sampling_w
    arr = ss.array_from_file(os.path.join(REF_DATASETS, "sky_rgb_rad.bin"))
    assert arr.shape == (10, 2, 6, 3)


def test_device_entry_points_refuse_host_only_emitter():
    """bake / eval_jvp / eval_vjp on an emitter staged without a device fail with a message."""
    import ctypes
    lib = ss.lib()
    em = ss.SunskyEmitter({"type": "sunsky", "sun_direction": [0.3, 0.2, 0.9]}, "rgb", device="host")
    buf = (ctypes.c_float * 64)()
    assert lib.sunsky_bake_latlong(em._h, 8, 4, 0.0, 3.14, 0.0, 6.28, None, 0, buf, 32, None) != 0
    assert b"host-only" in lib.sunsky_last_error()
    vin = ss._capi.Vec3In(ctypes.addressof(buf), ctypes.addressof(buf), ctypes.addressof(buf))
    assert lib.sunsky_eval_vjp(em._h, vin, None, 0, 0, None, 4, buf, 4, buf, None) != 0
    assert b"host-only" in lib.sunsky_last_error()
    t = (ctypes.c_float * 1)(1.0)
    assert lib.sunsky_eval_jvp(em._h, 0, t, 1, vin, None, 0, 0, None, 4, buf, buf, 4, None) != 0
    assert b"host-only" in lib.sunsky_last_error()
    # argument validation happens before any device work
    assert lib.sunsky_bake_latlong(em._h, 0, 4, 0.0, 3.14, 0.0, 6.28, None, 0, buf, 32, None) != 0
    assert b"image size" in lib.sunsky_last_error()
    assert lib.sunsky_eval_vjp(em._h, vin, None, 0, 0, None, 4, buf, 4, None, None) != 0
    assert b"gradient" in lib.sunsky_last_error()


def test_hosek_sun_rad_reproduces_spd_fixtures(golden_dir):
    """mi.hosek_sun_rad's product counterpart reproduces the reference's 80 .spd fixtures
    (generated by mi.hosek_sun_rad, test_sunsky.py:154-196) bit for bit in fp32."""
    sp = np.load(os.path.join(golden_dir, "sun_spectra.npz"))
    for t, eta, g, rad in zip(sp["turbidity"], sp["eta"], sp["gamma"], sp["radiance"]):
        got = np.array([ss.hosek_sun_rad(t, w, eta, g) for w in sp["wavelengths"]])
        np.testing.assert_array_equal(got.astype(np.float32), rad)
    assert ss.hosek_sun_rad(3.0, 800.0, 0.5, 0.0) == 0.0          # outside [320, 720] nm
    assert ss.lib().plugin_name() == b"sunsky"


@pytest.mark.parametrize("elev,turb", [(2.0, 3.0), (30.0, 3.0), (45.0, 6.5), (80.0, 2.0), (85.0, 9.0), (89.0, 3.0),
                                       (0.3, 3.0)])
def test_sun_pick_sky_pdf_fit_bound(elev, turb):
    """The FAST samplers' sun picks take the sky pdf from the host's quadratic fit over the
    disc (SunskyKArgs::sun_sky_fit, DESIGN.md §3 "Sun-pick sky pdf").  Against the fp64
    oracle's exact sky pdf (pdf_direction at w_sky = 1, sunsky.cpp:711-763) at random disc
    directions: the fit stays within its staged bound, and the total pdf of a sun pick,
    (1 - w) sun_pdf + w sky_pdf, within 1e-7 wherever the fit is on.  Near the zenith or the
    horizon the fit is off (the kernels run the exact TGMM sum)."""
    d = angles_dict(turb, 0.4, np.deg2rad(90.0 - elev), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, "rgb", device="host")
    fit = em.table("sun_sky_fit")
    c, dev, fmin, ok, on = fit[:6].astype(np.float64), float(fit[6]), float(fit[7]), fit[8] == 1, fit[9] == 1
    if elev > 86.0 or elev < 1.0:
        assert not ok and not on
        return
    assert ok and on
    o = O.Oracle(d, "rgb", "jit", "f64")
    o.override_w_sky(1.0)
    inf = o.info()
    half = np.arccos(inf["cos_cutoff"])
    wo = sun_cone_wo(4096, inf["sun_dir_local"], half, seed=int(elev), scale=0.999)
    a, b = wo.astype(np.float64) @ inf["frame_s"], wo.astype(np.float64) @ inf["frame_t"]
    approx = c[0] + a * (c[1] + c[3] * a + c[4] * b) + b * (c[2] + c[5] * b)
    exact = o.pdf_direction(wo).astype(np.float64)
    assert np.abs(approx - exact).max() <= dev, (np.abs(approx - exact).max(), dev)
    assert exact.min() >= fmin
    w = em.sky_sampling_w
    sun_pdf = 1.0 / (2 * np.pi * (1 - inf["cos_cutoff"]))
    rel = w * np.abs(approx - exact) / ((1 - w) * sun_pdf + w * exact)
    assert rel.max() <= 1e-7, rel.max()


def test_sun_segment_thresholds_reproduce_the_reference_decision():
    """render_sun's segment (sunsky.cpp:579-584: floor(cbrt(2 elevation / pi) 45), elevation =
    pi/2 - acos(cos theta), fp32) is taken on the device by counting the staged cos theta
    thresholds a direction passes (SunskyKArgs::sun_seg_z, DESIGN.md §6 "Sun segment index").
    For EVERY fp32 cos theta in [0, 1] (1.07e9 values) the count equals the fp32 oracle's
    decision, so the kernels' index is the reference's bit for bit (VERDICT r04 missing 2)."""
    em = ss.SunskyEmitter(angles_dict(3.0, 0.0, np.deg2rad(45.0), 0.3, 1.0, 1.0), "rgb", device="host")
    t = em.table("sun_segments")
    assert t.shape == (47,)
    z = t[:45]
    assert z[0] == 0.0 and np.all(np.diff(z) > 0) and z[-1] < 1.0
    O.set_threads(os.cpu_count() or 1)
    bad, first = O.check_sun_segment_thresholds(z)
    assert bad == 0, (bad, None if first is None else np.uint32(first).view(np.float32))
    # each threshold is where the decision steps: one fp32 below it the segment is lower
    below = np.nextafter(z[1:], np.float32(0))
    assert np.all(O.sun_segment_f32(z[1:]) == np.arange(1, 45))
    assert np.all(O.sun_segment_f32(below) == np.arange(0, 44))


@pytest.mark.parametrize("elev,aperture", [(0.05, 0.5358), (0.6, 0.5358), (7.9, 0.5358), (21.7, 0.5358),
                                           (58.6, 0.5358), (89.9, 0.5358), (20.0, 30.0), (1.0, 5.0)])
def test_sun_segment_rows_bracket_the_disc(elev, aperture):
    """The kernels count thresholds over (sun_row_lo, sun_row_hi] only: every direction of the
    disc must have its reference segment in [sun_row_lo, sun_row_hi]."""
    d = dict(angles_dict(3.0, 0.3, np.deg2rad(90.0 - elev), 0.3, 1.0, 1.0), sun_aperture=aperture)
    em = ss.SunskyEmitter(d, "rgb", device="host")
    t = em.table("sun_segments")
    lo, hi = int(t[45]), int(t[46])
    o = O.Oracle(d, "rgb", "jit", "f32")
    inf = o.info()
    wo = sun_cone_wo(8192, inf["sun_dir_local"], np.arccos(inf["cos_cutoff"]), seed=int(elev * 10), scale=1.0)
    inside = (wo @ inf["sun_dir_local"] >= inf["cos_cutoff"]) & (wo[:, 2] >= 0)
    pos = O.sun_segment_f32(wo[inside, 2])
    assert inside.sum() > 1000
    assert pos.min() >= lo and pos.max() <= hi, (lo, hi, pos.min(), pos.max())


@pytest.mark.parametrize("variant", ["rgb", "spectral"])
def test_sun_segment_jump_at_every_start_is_below_the_parity_bar(variant):
    """What an index flip at a segment start would cost (DESIGN.md §6 "Sun segment index"):
    the staged sun table is continuous across its 44 starts to ~1e-6, i.e. segment j - 1's
    polynomial at x = start_j - start_{j-1} against segment j's at x = 0, relative to the
    radiance (RGB: over cos psi in [0, 1], floored at 1e-2 of the lane's largest channel as the
    sun-disc tests do; spectral: channels above 1e-3 of the largest).  The kernels now take the
    reference's index exactly; this bounds the effect of Dr.Jit's own acos / cbrt (unvendored,
    parity unpinned) deciding a start one ulp differently: below 5e-6 < 1e-5 at every
    turbidity."""
    starts = np.pi / 2 * (np.arange(46) / 45.0) ** 3
    worst = 0.0
    for turb in (1.0, 1.5, 2.0, 2.5, 3.0, 4.2, 6.0, 7.7, 9.0, 10.0):
        em = ss.SunskyEmitter(angles_dict(turb, 0.0, np.deg2rad(45.0), 0.3, 1.0, 1.0), variant, device="host")
        t = em.table("sun_radiance").astype(np.float64)
        for j in range(1, 45):
            dx = starts[j] - starts[j - 1]
            if variant == "spectral":
                S = t.reshape(45, 11, 4)
                a = sum(S[j - 1, :, k] * dx ** k for k in range(4))
                b = S[j, :, 0]
                ok = np.abs(b) > 1e-3 * np.abs(b).max()
                if not ok.any():
                    continue
                rel = np.abs(a - b)[ok] / np.abs(b)[ok]
            else:
                S = t.reshape(45, 3, 4, 6)
                cp = np.linspace(0.0, 1.0, 41)[:, None] ** np.arange(6)
                a = np.einsum("ckl,k,pl->pc", S[j - 1], dx ** np.arange(4), cp)
                b = np.einsum("cl,pl->pc", S[j, :, 0, :], cp)
                rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-2 * np.abs(b).max(axis=1, keepdims=True))
            worst = max(worst, float(rel.max()))
    print(f"{variant}: largest relative jump at a segment start {worst:.3e}")
    assert worst < 5e-6


def _fit_cases():
    """the sun-pick sky-pdf fit over a wide grid -- azimuth, turbidity 1-10, albedo
    0-1, and sun elevations at the fit's cutoffs (2 rho above the horizon = 0.536 deg, 16 rho from
    the zenith = 85.71 deg) as well as in between; seeded."""
    rng = np.random.default_rng(2024)
    elevs = [0.55, 0.6, 0.75, 1.5, 4.0, 12.0, 27.0, 44.0, 61.0, 75.0, 83.0, 85.5, 85.65, 85.7, 85.75]
    return [(float(e), float(rng.uniform(0, 2 * np.pi)), float(rng.uniform(1, 10)), float(rng.uniform(0, 1)))
            for e in elevs]


@pytest.mark.parametrize("elev,phi,turb,albedo", _fit_cases())
def test_sun_pick_sky_pdf_fit_bound_wide(elev, phi, turb, albedo):
    """test_sun_pick_sky_pdf_fit_bound over the wide grid, with 16384 disc points per case (a
    quarter of them on the rim): wherever the staged fit is usable its bound holds, and
    wherever it is switched on the sun pick's pdf stays within 1e-7 relative."""
    d = angles_dict(turb, phi, np.deg2rad(90.0 - elev), albedo, 1.0, 1.0)
    em = ss.SunskyEmitter(d, "rgb", device="host")
    fit = em.table("sun_sky_fit")
    c, dev, fmin, ok, on = fit[:6].astype(np.float64), float(fit[6]), float(fit[7]), fit[8] == 1, fit[9] == 1
    rho_deg = np.rad2deg(np.deg2rad(0.5358 / 2))
    if elev < np.rad2deg(np.arcsin(2 * np.sin(np.deg2rad(rho_deg)))) or elev > 90.0 - np.rad2deg(
            np.arcsin(16 * np.sin(np.deg2rad(rho_deg)))):
        assert not ok and not on
        return
    if not ok:
        return                 # e.g. a disc across the phi wrap: the kernels run the exact TGMM sum
    o = O.Oracle(d, "rgb", "jit", "f64")
    o.override_w_sky(1.0)
    inf = o.info()
    half = np.arccos(inf["cos_cutoff"])
    wo = np.concatenate([sun_cone_wo(12288, inf["sun_dir_local"], half, seed=int(elev * 100), scale=0.9999),
                         sun_cone_wo(4096, inf["sun_dir_local"], half, seed=7, scale=1.0)])
    # the rim: push the last 4096 points out to the disc edge
    s = inf["sun_dir_local"].astype(np.float64)
    rim = wo[12288:].astype(np.float64)
    t = rim - (rim @ s)[:, None] * s
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    g = half * 0.99999
    wo[12288:] = (np.cos(g) * s + np.sin(g) * t).astype(np.float32)
    a, b = wo.astype(np.float64) @ inf["frame_s"], wo.astype(np.float64) @ inf["frame_t"]
    approx = c[0] + a * (c[1] + c[3] * a + c[4] * b) + b * (c[2] + c[5] * b)
    exact = o.pdf_direction(wo).astype(np.float64)
    assert np.abs(approx - exact).max() <= dev, (np.abs(approx - exact).max(), dev)
    assert exact.min() >= fmin
    if on:
        w = em.sky_sampling_w
        sun_pdf = 1.0 / (2 * np.pi * (1 - inf["cos_cutoff"]))
        rel = w * np.abs(approx - exact) / ((1 - w) * sun_pdf + w * exact)
        assert rel.max() <= 1e-7, rel.max()


@pytest.mark.parametrize("variant,semantics,d", [c for c in CASES if c[1] == "jit"])
def test_quadrature_gap_to_the_sequential_fp32_sum(variant, semantics, d):
    """the reference sums estimate_sky_sun_ratio's 40,000 fp32 terms with
    dr::sum_inner, whose order Dr.Jit leaves to the backend -- agreement with the reference's
    actual reduction is PARITY UNPINNED (no fixture holds w_sky).  The tests hold the product
    to the oracle's exact sum (1e-6); this keeps the distance to the worst-order reduction (the
    terms added one by one in fp32, oracle_set_quadrature_sum(1)) visible: within 2e-5
    relative for w_sky and the wavelength-distribution nodes (5.1e-6 /
    9.6e-6 over 86 emitters)."""
    em = ss.SunskyEmitter(d, variant=variant, semantics=semantics, device="host")
    O.set_quadrature_sum(True)
    try:
        o = O.Oracle(d, variant, semantics, "f32").info()
    finally:
        O.set_quadrature_sum(False)
    gap = abs(em.info()["w_sky"] - o["w_sky"]) / max(1e-3, abs(o["w_sky"]))
    msg = f"w_sky gap to the sequential fp32 sum {gap:.2e}"
    if variant == "spectral":
        a, b = em.table("spectral_pdf").astype(np.float64), o["spec_pdf"].astype(np.float64)
        ng = float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30)))
        msg += f", nodes {ng:.2e}"
        assert ng <= 2e-5, msg
    print(msg)
    assert gap <= 2e-5, msg
