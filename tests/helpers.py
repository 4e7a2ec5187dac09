"""Shared input generators for the parity tests (mirrors the reference tests'
ray layouts, src/emitters/tests/test_sunsky.py)."""
import numpy as np

SPECIAL_ALBEDO = {  # test_sunsky.py:12-16
    "type": "irregular",
    "wavelengths": "320, 360, 400, 440, 480, 520, 560, 600, 640, 680, 720",
    "values": "0.56, 0.21, 0.58, 0.24, 0.92, 0.42, 0.53, 0.75, 0.54, 0.20, 0.46",
}
EXR_WAVELENGTHS = [360 + (830 - 360) / 10 / 2 + i * (830 - 360) / 10 for i in range(10)]  # :88-90


def exr_grid_wi(res=(32, 64)):
    """si.wi of generate_and_compare (test_sunsky.py:93-100): NOT negated."""
    phis, thetas = np.meshgrid(np.linspace(0, 2 * np.pi, res[1], dtype=np.float32),
                               np.linspace(np.pi, 0, res[0], dtype=np.float32))
    phis, thetas = phis.ravel(), thetas.ravel()
    return np.stack([np.cos(phis) * np.sin(thetas), np.sin(phis) * np.sin(thetas), np.cos(thetas)],
                    1).astype(np.float32)


def angles_dict(turb, sun_phi, sun_theta, albedo, sky_scale, sun_scale, **kw):
    """make_emitter_angles (test_sunsky.py:28-39)."""
    d = {"type": "sunsky",
         "sun_direction": [float(np.cos(sun_phi) * np.sin(sun_theta)),
                           float(np.sin(sun_phi) * np.sin(sun_theta)), float(np.cos(sun_theta))],
         "sun_scale": sun_scale, "sky_scale": sky_scale, "turbidity": turb, "albedo": albedo}
    d.update(kw)
    return d


def hour_dict(turb, hour, albedo, sky_scale, sun_scale):
    """make_emitter_hour (test_sunsky.py:18-26)."""
    return {"type": "sunsky", "hour": hour, "sun_scale": sun_scale, "sky_scale": sky_scale,
            "turbidity": turb, "albedo": albedo}


def hemisphere_wo(n, seed=0):
    """Uniform upper-hemisphere directions (cos theta = u1, phi = 2 pi u2), SURVEY.md §8d C2."""
    rng = np.random.default_rng(seed)
    u1 = rng.random(n, dtype=np.float32)
    u2 = rng.random(n, dtype=np.float32)
    ct = u1
    st = np.sqrt(np.maximum(0, 1 - ct * ct))
    ph = np.float32(2 * np.pi) * u2
    return np.stack([st * np.cos(ph), st * np.sin(ph), ct], 1).astype(np.float32)


def sphere_wo(n, seed=0):
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((n, 3)).astype(np.float32)
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def sun_cone_wo(n, sun_dir, half_aperture, seed=0, scale=1.0):
    """Directions inside (scale<1) / around the sun cone, for sun-disc coverage."""
    rng = np.random.default_rng(seed)
    s = np.asarray(sun_dir, dtype=np.float64)
    s = s / np.linalg.norm(s)
    a = np.array([1.0, 0, 0]) if abs(s[0]) < 0.9 else np.array([0, 1.0, 0])
    t1 = np.cross(s, a)
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(s, t1)
    g = half_aperture * scale * np.sqrt(rng.random(n))
    ph = 2 * np.pi * rng.random(n)
    d = (np.cos(g)[:, None] * s + np.sin(g)[:, None] * (np.cos(ph)[:, None] * t1 + np.sin(ph)[:, None] * t2))
    return d.astype(np.float32)


def mean_rel(x, ref, eps):
    return float(np.mean(np.abs(x - ref) / (np.abs(ref) + eps)))


def max_rel(x, ref, floor_frac=1e-6):
    """max |x-ref| / max(|ref|, floor_frac * max|ref|)   (SURVEY.md §8d parity metric)."""
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    floor = floor_frac * max(np.abs(ref).max(), 1e-30)
    return float(np.max(np.abs(x - ref) / np.maximum(np.abs(ref), floor)))


def mask_flip_lanes(o32, o64):
    """Lanes where the fp32 and fp64 oracles take different sides of a mask -- the horizon
    (cos theta >= 0) or the sun disc (s . wo >= cos(alpha / 2)), sunsky.cpp:313-314: one value
    is zero and the other not, or they differ by more than a factor of 2 (the sun term is 1e2-1e6
    times the sky), on any channel.  Ill-conditioned lanes (the limb's cos psi) differ far less."""
    a, b = np.abs(np.asarray(o32, np.float64)), np.abs(np.asarray(o64, np.float64))
    hi, lo = np.maximum(a, b), np.minimum(a, b)
    m = (hi > 1e-6 * max(float(b.max()), 1e-30)) & (hi - lo > 0.5 * hi)
    return m.any(axis=-1) if m.ndim > 1 else m


def parity_stats(gpu, o32, o64, sunlanes, rtol=1e-5):
    """Per-population error figures.  Sky lanes relative to the fp32
    oracle; sun-disc lanes relative to fp64, next to the fp32 oracle's own error there:
    the reference's fp32 arithmetic is the accuracy the sun disc can be held to.
    Lanes where fp32 and fp64 disagree by > 1e-3 (a horizon or disc-edge mask that one
    precision flips, or the limb's ill-conditioned cos psi) are counted, not measured; of
    them, the mask flips (mask_flip_lanes()) and how many the GPU puts on the fp32
    reference's side.  The *_over_1e-5 counts are lanes (any channel) beyond a literal
    rtol of the fp32 / fp64 oracle."""
    st = {"sky_lanes": int((~sunlanes).sum()), "sun_lanes": int(sunlanes.sum())}
    g = np.asarray(gpu, np.float64)
    a = np.asarray(o32, np.float64)
    b = np.asarray(o64, np.float64)
    lane = (lambda m: m.any(axis=-1)) if a.ndim > 1 else (lambda m: m)
    floor = 1e-6 * max(np.abs(b).max(), 1e-30)
    den = np.maximum(np.abs(b), floor)
    den_a = np.maximum(np.abs(a), 1e-6 * max(np.abs(a).max(), 1e-30))
    flip = lane(np.abs(a - b) / den > 1e-3)
    mflip = mask_flip_lanes(a, b)
    st["deviant_lanes"] = int(flip.sum())
    st["mask_flip_lanes"] = int(mflip.sum())
    st["mask_flip_lanes_on_o32_side"] = int((mflip & ~lane(np.abs(g - a) / den_a > 1e-3)).sum())
    over32 = lane(np.abs(g - a) / den_a > rtol)
    st["sky_lanes_over_1e-5_vs_o32"] = int((over32 & ~sunlanes).sum())
    st["sun_lanes_over_1e-5_vs_o32"] = int((over32 & sunlanes).sum())
    sky, sun = ~sunlanes & ~flip, sunlanes & ~flip
    if sky.any():
        st["sky_max_rel_vs_o32"] = max_rel(g[sky], a[sky])
        st["sky_max_rel_vs_o64"] = float((np.abs(g[sky] - b[sky]) / den[sky]).max())
    if sun.any():
        rg, ra = np.abs(g[sun] - b[sun]) / den[sun], np.abs(a[sun] - b[sun]) / den[sun]
        st["sun_max_rel_vs_o64"] = float(rg.max())
        st["sun_o32_max_rel_vs_o64"] = float(ra.max())
        st["sun_lanes_over_1e-5_vs_o64"] = int(lane(rg > rtol).sum())
        st["sun_o32_lanes_over_1e-5_vs_o64"] = int(lane(ra > rtol).sum())
    return st


SUN_SLACK = {"fast": 1.25, "reference": 4.0}


def assert_parity(gpu, o32, o64, sunlanes, rtol=1e-5, precision="fast", sun_k=None, sun_rtol=None):
    """gpu/o32/o64: (n, c).  sky lanes: rel to o32; sun lanes: conditioning-aware vs o64,
    |gpu - o64| <= rtol |o64| + k |o32 - o64| per lane with k = 1.25 for the fast kernels
    (their cos psi comes from fp64 chord terms: more accurate than the reference's fp32) and
    k = 4 for the reference-precision kernels, which repeat the reference's fp32 operations
    with the GPU's libm (an ulp of sin(gamma) next to the limb moves a lane by ~1e-5); those
    must also be as accurate as the fp32 reference overall (max over the sun lanes within
    1.25 x the fp32 oracle's max).  sun_k overrides k (the aggregate check then applies when
    k > 1.25).  sun_rtol overrides rtol on the sun lanes.  Returns parity_stats()."""
    k = SUN_SLACK[precision] if sun_k is None else sun_k
    sun_rtol = rtol if sun_rtol is None else sun_rtol
    sky = ~sunlanes
    if sky.any():
        g, a, b = gpu[sky].astype(np.float64), o32[sky].astype(np.float64), o64[sky]
        floor = 1e-6 * np.abs(a).max()
        strict = np.abs(g - a) <= rtol * np.maximum(np.abs(a), floor)
        bound = rtol * np.maximum(np.abs(a), floor) + np.abs(a - b)
        bad = np.abs(g - a) > bound
        assert not bad.any(), (f"sky lanes: {bad.sum()} over bound, worst {np.max(np.abs(g - a) / bound):.2f}x; "
                               f"strict max rel {max_rel(gpu[sky], o32[sky]):.3e}")
        assert strict.mean() >= 0.9999, f"sky lanes: only {strict.mean():.6f} within plain {rtol:g}"
    if sunlanes.any():
        g, a, b = gpu[sunlanes].astype(np.float64), o32[sunlanes].astype(np.float64), o64[sunlanes]
        bound = sun_rtol * np.abs(b) + k * np.abs(a - b) + 1e-30
        bad = np.abs(g - b) > bound
        assert not bad.any(), f"sun lanes: {bad.sum()} over bound, worst {np.max(np.abs(g - b) / bound):.2f}x"
    # Lanes where the two precisions take different sides of a mask (horizon, disc edge): the
    # bounds above admit anything between the sides there.  The kernels make the reference's
    # own fp32 tests (cos theta >= 0, the fp32 dot s . wo >= cos(alpha / 2) in the oracle's fma
    # order), so each mask flip must sit on the fp32 reference's side: within 1e-3 of o32 on
    # every channel.  Other lanes where o32 and o64 differ by > 1e-3 (the limb's
    # ill-conditioned cos psi, where the fp32 reference itself is off by up to 1.5e-4 and the
    # FAST kernels are closer to fp64) must sit within 1e-3 of one of them.
    g, a, b = (np.asarray(x, np.float64) for x in (gpu, o32, o64))
    den_a = np.maximum(np.abs(a), 1e-6 * max(np.abs(a).max(), 1e-30))
    den_b = np.maximum(np.abs(b), 1e-6 * max(np.abs(b).max(), 1e-30))
    lane = (lambda m: m.any(axis=-1)) if a.ndim > 1 else (lambda m: m)
    side_a = ~lane(np.abs(g - a) / den_a > 1e-3)
    side_b = ~lane(np.abs(g - b) / den_b > 1e-3)
    mflip = mask_flip_lanes(a, b)
    off32 = mflip & ~side_a
    assert not off32.any(), (f"{int(off32.sum())} of {int(mflip.sum())} mask-flip lanes not on the fp32 reference's "
                             f"side (its fp32 horizon / disc test)")
    flip = lane(np.abs(a - b) / den_b > 1e-3) & ~mflip
    off = flip & ~side_a & ~side_b
    assert not off.any(), f"{int(off.sum())} of {int(flip.sum())} ill-conditioned lanes on neither side"
    st = parity_stats(gpu, o32, o64, sunlanes, rtol=rtol)
    if k > 1.25 and "sun_max_rel_vs_o64" in st:
        assert st["sun_max_rel_vs_o64"] <= 1.25 * max(st["sun_o32_max_rel_vs_o64"], rtol), st
    print("parity", {k: (f"{v:.3e}" if isinstance(v, float) else v) for k, v in st.items()})
    return st


def lambda_pdf(o, lam):
    """ContinuousDistribution::eval_pdf_normalized (distr_1d.h:428-446) of the oracle's
    wavelength distribution over [360, 720] at lam, in fp64 (nodes and integral from the
    oracle, after it adopted the product's nodes)."""
    inf = o.info()
    y = inf["spec_pdf"].astype(np.float64)
    x = (np.asarray(lam, np.float64) - 360.0) / (360.0 / (y.size - 1))
    i = np.clip(np.floor(x).astype(int), 0, y.size - 2)
    t = x - i
    return (y[i] + t * (y[i + 1] - y[i])) / inf["spec_integral"]


def assert_lambda_parity(lam_g, lam_o):
    """Same sample, same wavelength: every lane within 1e-5 relative of the fp32 oracle that
    adopted the product's nodes (the product and the oracle invert the same CDF with the same
    fp32 operations, so in practice the wavelengths are equal bit for bit)."""
    rel = np.abs(lam_g.astype(np.float64) - lam_o) / np.abs(lam_o)
    assert rel.max() <= 1e-5, (rel.max(), np.argmax(rel))
    same = float(np.mean(lam_g == lam_o.astype(np.float32)))
    print(f"lambda: max rel {rel.max():.3e}, bitwise equal {same:.6f}")
    return same


def disc_lanes(d, info, band=1e-6):
    """Sun-disc lanes for the parity bars: directions within `band` of the disc edge count
    as disc lanes too.  The kernel's (and the fp32 reference's) disc test is an fp32 dot
    against the fp32 cos(half aperture); a lane the fp64 test puts just outside may carry
    the sun term, at the limb where the fp32 reference's own cos psi error is largest."""
    return (np.asarray(d, np.float64) @ info["sun_dir_local"]) >= info["cos_cutoff"] - band


def fp32_sun_input(d, o32):
    """The emitter dict with sun_direction replaced by the fp32-normalised direction the
    reference computes from it (dr::normalize(props.get<ScalarVector3f>("sun_direction")),
    sunsky.cpp:923) -- the product and the fp32 oracle use those bits -- for the fp64 oracle,
    so that it evaluates exactly what an fp32 implementation was given.  From the unrounded
    direction the disc moves by up to ~1e-8 rad, which next to the limb (d cos psi / d gamma
    unbounded) moves disc lanes by up to 3.6e-4 (measured at 8 deg elevation / 200 deg)."""
    if "sun_direction" not in d:
        return d
    return dict(d, sun_direction=[float(x) for x in o32.info()["sun_dir_world"]])
