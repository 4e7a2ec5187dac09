"""Sun-disc lanes of the FAST eval kernels at the literal 1e-5 bar.

The error of a disc lane splits in two (oracle/oracle_impl.inc `oracle_round_staged_tables`,
`oracle_adopt_tables`):
* table rounding: the reference stages its tables in fp32 (array_from_file<Float64, Float>,
  sunsky.cpp:182-195).  The fp64 evaluation of the fp32-rounded tables ("o64r") against the
  fp64 tables ("o64") is measured in tests/test_oracle_table_modes.py (<= 1.4e-6 on its disc lanes);
* the kernel's own arithmetic: the kernel against the fp64 evaluation of the exact fp32
  tables, local sun direction and disc cutoff it was given ("o64t", the oracle adopting the
  product's staged state) -- the exact value of the fp32-staged algorithm on those inputs.
  (The fp64 oracle renormalises the fp32 sun direction in fp64, which moves it by ~1e-8; at
  the limb, where d cos psi / d gamma is unbounded, that alone moves a lane by up to ~5e-5.)
The FAST eval kernels evaluate the disc term in fp64 (sunsky_kernels.hip `SunDisc64`), so
every disc lane must sit within a plain 1e-5 of o64t on every channel.  Lanes where the
fp32 and fp64 disc / horizon tests disagree (the mask flips of tests/helpers.py) take the
fp32 reference's side, as in every other parity test.
"""
import numpy as np
import pytest
import torch

import oracle as O
import sunsky_amd as ss
from helpers import angles_dict, fp32_sun_input, hemisphere_wo, mask_flip_lanes, sun_cone_wo

pytestmark = pytest.mark.gpu

RTOL = 1e-5
NODES = [float(x) for x in range(320, 721, 40)]
EXR_LAMBDAS = [383.5 + 47.0 * i for i in range(10)]   # test_sunsky.py:88-90, off the nodes


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def soa(a):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float32).T)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def disc_heavy_wo(info, n_disc, seed):
    """Uniform over the disc, a band within 1e-4 of the limb (where cos psi cancels), a little
    outside it, and random sky directions."""
    s, ha = info["sun_dir_local"], float(np.arccos(info["cos_cutoff"]))
    rng = np.random.default_rng(seed)
    limb = sun_cone_wo(n_disc, s, ha, seed=seed + 1, scale=1.0)
    # directions at gamma in [ha (1 - 1e-4), ha (1 + 1e-5)]: rebuild from the cone axis
    g = ha * (1 - 1e-4 * rng.random(n_disc) + 1e-5 * rng.random(n_disc) * (rng.random(n_disc) < 0.1))
    ph = 2 * np.pi * rng.random(n_disc)
    s64 = np.asarray(s, np.float64)
    a = np.array([1.0, 0, 0]) if abs(s64[0]) < 0.9 else np.array([0, 1.0, 0])
    t1 = np.cross(s64, a)
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(s64, t1)
    edge = (np.cos(g)[:, None] * s64 + np.sin(g)[:, None] * (np.cos(ph)[:, None] * t1 + np.sin(ph)[:, None] * t2))
    return np.concatenate([limb, edge.astype(np.float32), hemisphere_wo(4 * n_disc, seed=seed + 2)]).astype(np.float32)


def check(out, o32, o64t, o64, disc, label):
    """out / o32 / o64t / o64: (n, c); disc: lanes inside the fp32 disc test."""
    g, a, b, c = (np.asarray(x, np.float64) for x in (out, o32, o64t, o64))
    flip = mask_flip_lanes(a, b)
    den_a = np.maximum(np.abs(a), 1e-6 * np.abs(a).max())
    assert not (flip & (np.abs(g - a) / den_a > 1e-3).any(axis=-1)).any(), f"{label}: mask flip off o32's side"
    lanes = disc & ~flip
    assert lanes.sum() > 100, label
    den = np.maximum(np.abs(b[lanes]), 1e-30)
    rel = (np.abs(g[lanes] - b[lanes]) / den).max(axis=-1)
    tab = (np.abs(np.asarray(c)[lanes] - b[lanes]) / den).max(axis=-1)    # fp32 staged state vs fp64
    rel32 = (np.abs(a[lanes] - b[lanes]) / den).max(axis=-1)
    print(f"{label}: {int(lanes.sum())} disc lanes: kernel vs o64t max {rel.max():.2e} "
          f"(over 1e-5: {int((rel > RTOL).sum())}); o32 vs o64t max {rel32.max():.2e} "
          f"(over 1e-5: {int((rel32 > RTOL).sum())}); o64 vs o64t (fp32 tables and sun frame) max {tab.max():.2e}")
    assert (rel <= RTOL).all(), f"{label}: {int((rel > RTOL).sum())} disc lanes over 1e-5 of o64t, worst {rel.max():.3e}"
    return rel.max()


def oracles(d, variant, em):
    o32 = O.Oracle(d, variant, "jit", "f32")
    d64 = fp32_sun_input(d, o32)
    o64 = O.Oracle(d64, variant, "jit", "f64")
    o64t = O.Oracle(d64, variant, "jit", "f64")
    o64t.adopt_tables(em)
    return o32, o64t, o64


CASES = [(45.0, 2.0), (45.0, 10.0), (30.0, 3.0), (8.0, 6.0), (2.5, 1.5)]


@pytest.mark.parametrize("elev,turb", CASES)
def test_fast_eval_rgb_disc_lanes_literal_bar(elev, turb):
    """eval() and eval_direction() (sunsky.cpp:303-352, 453-461), RGB."""
    d = angles_dict(turb, 0.3, np.deg2rad(90 - elev), 0.1, 1.0, 1.0)
    em = ss.SunskyEmitter(d, "rgb", precision="fast")
    o32, o64t, o64 = oracles(d, "rgb", em)
    inf = o32.info()
    wo = disc_heavy_wo(inf, 8192, seed=int(elev * 10))
    disc = (wo @ inf["sun_dir_local"].astype(np.float32) >= np.float32(inf["cos_cutoff"])) & (wo[:, 2] >= 0)
    a, b, c = o32.eval(-wo), o64t.eval(-wo), o64.eval(-wo)
    out = host(em.eval(ss.SurfaceInteraction3f(wi=soa(-wo)))).T
    check(out, a, b, c, disc, f"eval rgb {elev} deg T {turb}")
    ds = ss.DirectionSample3f(d=soa(wo))
    outd = host(em.eval_direction(ss.Interaction3f(), ds)).T
    assert np.array_equal(outd, out)
    # the VEC = 1 kernel (planes at a 4-byte offset) gives the same bits
    n = wo.shape[0]
    flat = torch.empty(3 * n + 1, dtype=torch.float32, device="cuda")
    wi_odd = flat[1:].view(3, n)
    wi_odd.copy_(soa(-wo))
    assert wi_odd.data_ptr() % 16 != 0
    out1 = host(em.eval(ss.SurfaceInteraction3f(wi=wi_odd))).T
    assert np.array_equal(out1, out)


@pytest.mark.parametrize("elev,turb", CASES)
@pytest.mark.parametrize("kind", ["nodes", "broadcast", "rays4"])
def test_fast_eval_spectral_disc_lanes_literal_bar(kind, elev, turb):
    """Spectral eval (sunsky.cpp:325-348): the C3 node kernel, a broadcast list off the nodes,
    and per-ray wavelengths (Mitsuba's Spectrum<Float, 4>)."""
    d = angles_dict(turb, 0.3, np.deg2rad(90 - elev), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, "spectral", precision="fast")
    o32, o64t, o64 = oracles(d, "spectral", em)
    inf = o32.info()
    wo = disc_heavy_wo(inf, 4096, seed=int(elev * 10) + 7)
    n = wo.shape[0]
    disc = (wo @ inf["sun_dir_local"].astype(np.float32) >= np.float32(inf["cos_cutoff"])) & (wo[:, 2] >= 0)
    if kind == "rays4":
        rng = np.random.default_rng(5)
        lam = (360 + 360 * rng.random((4, n))).astype(np.float32)
        out = host(em.eval(ss.SurfaceInteraction3f(wi=soa(-wo), wavelengths=torch.from_numpy(lam).cuda())))
    else:
        ls = NODES if kind == "nodes" else EXR_LAMBDAS
        lam = np.repeat(np.asarray(ls, np.float32)[:, None], n, 1)
        out = host(em.eval_spectral_broadcast(soa(-wo), ls))
    a, b, c = o32.eval(-wo, lam), o64t.eval(-wo, lam), o64.eval(-wo, lam)
    check(out.T, a.T, b.T, c.T, disc, f"{kind} {elev} deg T {turb}")


def test_fast_bake_disc_pixels_match_eval():
    """The lat-long bake evaluates the disc term in line (kSunF64) on directions it generates
    on the device: its disc pixels against eval() of the host-generated grid (a 30 deg
    aperture so the grid resolves the disc), away from the limb and the horizon where the
    directions' rounding dominates (tests/test_bake.py compares the rest)."""
    import math
    from test_bake import grid_dirs
    d = angles_dict(3.0, 0.4, np.deg2rad(50), 0.2, 1.0, 1.0, sun_aperture=30.0)
    for variant in ("rgb", "spectral"):
        em = ss.SunskyEmitter(d, variant, precision="fast")
        w, h = 256, 128
        img = em.bake_latlong(w, h) if variant == "rgb" else em.bake_latlong(w, h, wavelengths=NODES)
        img = host(img).reshape(3 if variant == "rgb" else len(NODES), -1)
        dirs, theta = grid_dirs(w, h)
        wi = torch.from_numpy(-dirs).cuda()
        ref = host(em.eval(ss.SurfaceInteraction3f(wi=wi)) if variant == "rgb" else em.eval_spectral_broadcast(wi, NODES))
        inf = O.Oracle(d, variant, "jit", "f32").info()
        gam = np.arccos(np.clip(dirs.T.astype(np.float64) @ inf["sun_dir_local"], -1, 1))
        ha = math.radians(15.0)
        disc = (gam < ha - 1e-3) & (np.abs(theta - np.pi / 2) > np.radians(2))
        assert disc.sum() > 100
        rel = np.abs(img[:, disc] - ref[:, disc]) / np.abs(ref[:, disc])
        assert rel.max() < 1e-4, rel.max()


# Beyond the five positions above: the sun at the zenith and just above the horizon (the disc
# then spans the elevation range where the segment index and the horizon mask change), and
# wider apertures (more disc lanes, cos psi over a wider chord range).
EXTRA = [(89.0, 3.0, 0.5358), (0.6, 4.0, 0.5358), (20.0, 2.5, 5.0), (60.0, 7.0, 12.0)]


@pytest.mark.parametrize("elev,turb,aperture", EXTRA)
def test_fast_eval_disc_lanes_literal_bar_extremes(elev, turb, aperture):
    """RGB eval and the C3 node kernel at the extra sun positions / apertures."""
    base = angles_dict(turb, 0.3, np.deg2rad(90 - elev), 0.2, 1.0, 1.0, sun_aperture=aperture)
    for variant in ("rgb", "spectral"):
        em = ss.SunskyEmitter(base, variant, precision="fast")
        o32, o64t, o64 = oracles(base, variant, em)
        inf = o32.info()
        wo = disc_heavy_wo(inf, 4096, seed=int(elev * 10) + 11)
        disc = (wo @ inf["sun_dir_local"].astype(np.float32) >= np.float32(inf["cos_cutoff"])) & (wo[:, 2] >= 0)
        if variant == "rgb":
            out = host(em.eval(ss.SurfaceInteraction3f(wi=soa(-wo)))).T
            check(out, o32.eval(-wo), o64t.eval(-wo), o64.eval(-wo), disc, f"rgb {elev} deg ap {aperture}")
        else:
            lam = np.repeat(np.asarray(NODES, np.float32)[:, None], wo.shape[0], 1)
            out = host(em.eval_spectral_broadcast(soa(-wo), NODES))
            check(out.T, o32.eval(-wo, lam).T, o64t.eval(-wo, lam).T, o64.eval(-wo, lam).T, disc,
                  f"nodes {elev} deg ap {aperture}")
