"""Forward-mode derivatives of eval() (sunsky_eval_jvp) against central finite
differences of the fp64 oracle -- the reference differentiates turbidity,
albedo and sun_direction (sunsky.cpp:220-240; sunsky-testing/traversal_test.py:
94-145).  Bar: |jvp - fd| <= 2e-3 |fd| + 1e-4 max|fd| per lane (FD truncation
and fp32 rounding), on the lanes where the quantity is differentiable."""
import ctypes
import math

import numpy as np
import pytest
import torch

import oracle as O
import sunsky_amd as ss
from helpers import angles_dict, assert_parity, hemisphere_wo, sun_cone_wo

ETA = math.radians(40)


def scene(turb=3.4, albedo=0.3, sun=None):
    d = angles_dict(turb, 0.6, math.pi / 2 - ETA, albedo, 1.0, 1.0)
    if sun is not None:
        d["sun_direction"] = [float(v) for v in sun]
    return d


def rays(o):
    inf = o.info()
    wo = np.concatenate([hemisphere_wo(1 << 14, seed=11),
                         sun_cone_wo(1024, inf["sun_dir_local"], np.arccos(inf["cos_cutoff"]), seed=12, scale=0.9)])
    return wo.astype(np.float32)


def check(jvp, fd, mask):
    j, f = jvp[mask].astype(np.float64), fd[mask]
    bound = 2e-3 * np.abs(f) + 1e-4 * np.abs(f).max()
    bad = np.abs(j - f) > bound
    assert not bad.any(), f"{bad.sum()} lanes over bound, worst {np.max(np.abs(j - f) / bound):.2f}x"


def test_jvp_argument_validation_host():
    em = ss.SunskyEmitter(scene(), "rgb", device="host")
    lib = ss.lib()
    t = (ctypes.c_float * 3)(1, 0, 0)
    vin = ss._capi.Vec3In(None, None, None)
    # n = 0: the tangent is still staged and validated
    assert lib.sunsky_eval_jvp(em._h, 0, t, 1, vin, None, 0, 0, None, 0, None, None, 0, None) == 0
    assert lib.sunsky_eval_jvp(em._h, 0, t, 2, vin, None, 0, 0, None, 0, None, None, 0, None) != 0
    assert b"turbidity tangent" in lib.sunsky_last_error()
    assert lib.sunsky_eval_jvp(em._h, 1, t, 3, vin, None, 0, 0, None, 0, None, None, 0, None) == 0
    assert lib.sunsky_eval_jvp(em._h, 7, t, 1, vin, None, 0, 0, None, 0, None, None, 0, None) != 0
    hour = ss.SunskyEmitter({"type": "sunsky", "hour": 12.0}, "rgb", device="host")
    assert lib.sunsky_eval_jvp(hour._h, 2, t, 3, vin, None, 0, 0, None, 0, None, None, 0, None) != 0
    assert b"time/location" in lib.sunsky_last_error()
    with pytest.raises(ValueError):
        em.eval_jvp(ss.SurfaceInteraction3f(wi=torch.zeros(3, 1)), "sky_scale", 1.0)


def _gpu(a):
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float32).T)).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["rgb", "spectral"])
@pytest.mark.parametrize("param", ["turbidity", "albedo", "sun_direction"])
def test_eval_jvp_matches_finite_differences(variant, param):
    d = scene()
    em = ss.load_dict(d, variant=variant)
    o32 = O.Oracle(d, variant, "jit", "f32")
    wo = rays(o32)
    wi = -wo
    lam = np.random.default_rng(3).uniform(330, 710, (4, wo.shape[0])).astype(np.float32)
    si = ss.SurfaceInteraction3f(wi=_gpu(wi), wavelengths=torch.from_numpy(lam).cuda() if variant == "spectral" else None)
    inf = o32.info()
    s = np.array(d["sun_direction"], np.float64)
    if param == "turbidity":
        tangent, h = [1.0], 1e-3
        plus, minus = scene(turb=3.4 + h), scene(turb=3.4 - h)
    elif param == "albedo":
        tangent, h = [1.0], 1e-3
        plus, minus = scene(albedo=0.3 + h), scene(albedo=0.3 - h)
    else:
        t = np.cross(s, [0.0, 0.0, 1.0])
        t /= np.linalg.norm(t)
        t = 0.6 * t + 0.8 * np.cross(s, t)            # a tangent mixing azimuth and elevation
        tangent, h = list(t), 1e-4
        plus, minus = scene(sun=(s + h * t) / np.linalg.norm(s + h * t)), scene(sun=(s - h * t) / np.linalg.norm(s - h * t))
    val, dval = em.eval_jvp(si, param, tangent)
    torch.cuda.synchronize()
    val, dval = val.cpu().numpy().T, dval.cpu().numpy().T
    lam_o = lam if variant == "spectral" else None
    ev = lambda dd: O.Oracle(dd, variant, "jit", "f64").eval(wi, lam_o)   # noqa: E731
    fd = (ev(plus) - ev(minus)) / (2 * h)
    fd = fd.T if variant == "spectral" else fd
    # value: the reference-order eval
    ref32 = o32.eval(wi, lam_o)
    ref64 = O.Oracle(d, variant, "jit", "f64").eval(wi, lam_o)
    ref32, ref64 = (ref32.T, ref64.T) if variant == "spectral" else (ref32, ref64)
    cosg = wo @ inf["sun_dir_local"]
    sun = (cosg >= inf["cos_cutoff"]) & (wo[:, 2] >= 0)
    assert_parity(val, ref32, ref64, sun, precision="reference")   # the AD kernels keep full precision
    mask = np.ones(wo.shape[0], bool)
    if param == "sun_direction":
        # the disc test flips under the perturbation and d gamma is singular at gamma = 0
        mask &= cosg < math.cos(math.radians(1.0))
    # finite differences straddle no discontinuity: keep lanes away from the horizon
    mask &= wo[:, 2] > 1e-3
    check(dval, fd, mask[:, None].repeat(dval.shape[1], 1))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["rgb", "spectral"])
def test_eval_vjp_matches_jvp_contractions(variant):
    """Reverse mode (sunsky_eval_vjp) against the forward mode: for a random cotangent,
    grad[p] = sum(d_out * jvp(e_p)) for every basis parameter; deterministic and accumulating."""
    grad, cot, si, view, em = _vjp_vs_jvp(scene(), variant)
    # deterministic, and accumulating into a given buffer
    grad2, _ = em.eval_vjp(si, cot)
    assert torch.equal(grad, grad2)
    em.eval_vjp(si, cot, grad=grad2)
    assert torch.allclose(grad2, 2 * grad, rtol=1e-6, atol=0)
    assert view["albedo"].numel() == (11 if variant == "spectral" else 3)


def _vjp_vs_jvp(d, variant, sun_axes=True):
    """eval_vjp's 15 gradients against the contractions of eval_jvp along each basis tangent
    (1e-4 of the contraction's magnitude); without sun axes (time/location mode) the three
    sun_direction gradients must be 0."""
    em = ss.load_dict(d, variant=variant)
    o32 = O.Oracle(d, variant, "jit", "f32")
    wo = rays(o32)
    rng = np.random.default_rng(5)
    lam = rng.uniform(330, 710, (4, wo.shape[0])).astype(np.float32)
    si = ss.SurfaceInteraction3f(wi=_gpu(-wo), wavelengths=torch.from_numpy(lam).cuda() if variant == "spectral" else None)
    k = 4 if variant == "spectral" else 3
    cot = torch.from_numpy(rng.standard_normal((k, wo.shape[0])).astype(np.float32)).cuda()
    grad, view = em.eval_vjp(si, cot)
    g = grad.cpu().numpy().astype(np.float64)
    c = cot.cpu().numpy().astype(np.float64)
    nch = 11 if variant == "spectral" else 3

    def contract(param, tangent):
        _, dv = em.eval_jvp(si, param, tangent)
        terms = c * dv.cpu().numpy().astype(np.float64)
        return terms.sum(), np.abs(terms).sum()

    checks = [(0, "turbidity", [1.0])]
    checks += [(1 + ch, "albedo", list(np.eye(nch)[ch])) for ch in range(nch)]
    if sun_axes:
        checks += [(12 + ax, "sun_direction", list(np.eye(3)[ax])) for ax in range(3)]
    else:
        assert np.all(g[12:15] == 0.0), g[12:15]
    for idx, param, tangent in checks:
        ref, mag = contract(param, tangent)
        assert abs(g[idx] - ref) <= 1e-4 * mag + 1e-12, (param, tangent, g[idx], ref, mag)
    return grad, cot, si, view, em


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["rgb", "spectral"])
@pytest.mark.parametrize("case", ["low_sun", "high_sun", "rotated", "time_mode"])
def test_eval_vjp_sun_axes_across_elevations_and_frames(variant, case):
    """The VJP reaches the sun axes through one unit-elevation sky tangent scaled by d eta_k
    plus the gamma part (sunsky_kernels.hip eval_vjp_*_body): the same contractions as the
    forward mode near the horizon, near the zenith, under a rotated to_world, and with no
    sun axes at all in time/location mode (sunsky.cpp:220-240: sun_direction is not exposed)."""
    if case == "time_mode":
        d = {"type": "sunsky", "hour": 15.5, "turbidity": 4.2, "albedo": 0.25}
        _vjp_vs_jvp(d, variant, sun_axes=False)
        return
    if case == "low_sun":
        d = scene(sun=[0.8 * math.cos(math.radians(4)), 0.6 * math.cos(math.radians(4)), math.sin(math.radians(4))])
    elif case == "high_sun":
        d = scene(sun=[0.3 * math.cos(math.radians(82)), -0.95 * math.cos(math.radians(82)), math.sin(math.radians(82))])
    else:
        d = scene(sun=[0.4, 0.3, 0.8])
        c, s = math.cos(0.7), math.sin(0.7)
        d["to_world"] = np.array([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]], np.float32)
    _vjp_vs_jvp(d, variant)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["rgb", "spectral"])
def test_ad_tables_restaged_after_parameter_change(variant):
    """The C ABI caches the AD tangent tables between calls (restaged on a state change or,
    for eval_jvp, a new tangent).  After params.update() -- and across JVP tangents, and
    across streams -- the results equal those of a freshly created emitter, bit for bit."""
    d = scene()
    em = ss.load_dict(d, variant=variant)
    o32 = O.Oracle(d, variant, "jit", "f32")
    wo = rays(o32)
    rng = np.random.default_rng(9)
    lam = rng.uniform(330, 710, (4, wo.shape[0])).astype(np.float32)
    si = ss.SurfaceInteraction3f(wi=_gpu(-wo), wavelengths=torch.from_numpy(lam).cuda() if variant == "spectral" else None)
    k = 4 if variant == "spectral" else 3
    cot = torch.from_numpy(rng.standard_normal((k, wo.shape[0])).astype(np.float32)).cuda()
    em.eval_vjp(si, cot)
    em.eval_jvp(si, "turbidity", [1.0])
    p = em.traverse()
    p["turbidity"] = 6.5
    p.update()
    fresh = ss.load_dict(scene(turb=6.5), variant=variant)
    g_new, _ = em.eval_vjp(si, cot)
    g_ref, _ = fresh.eval_vjp(si, cot)
    assert torch.equal(g_new, g_ref)
    nch = 11 if variant == "spectral" else 3
    for param, tan in (("turbidity", [1.0]), ("albedo", list(np.eye(nch)[1])), ("turbidity", [0.5]),
                       ("sun_direction", [0.0, 1.0, 0.0])):
        a = em.eval_jvp(si, param, tan)[1]
        b = fresh.eval_jvp(si, param, tan)[1]
        assert torch.equal(a, b), (param, tan)
    # another stream: ordered after the previous AD call on the default stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g_s, _ = em.eval_vjp(si, cot)
    s.synchronize()
    assert torch.equal(g_s, g_ref)


@pytest.mark.parametrize("variant", ["rgb", "spectral"])
@pytest.mark.parametrize("param,tangent", [("turbidity", [1.0]), ("albedo", [0.7]),
                                           ("sun_direction", [0.3, -0.2, 0.5])])
def test_host_tangent_tables_match_finite_differences_of_the_staging(variant, param, tangent):
    """CPU: the staging tangent (sunsky_staging.h radiance_param_tangent / sun_param_tangent,
    through sunsky_emitter_tangent_tables on the host) against central differences of the
    host-staged tables themselves (compute_radiance_params / compute_sun_params,
    sunsky.h:158-231, 404-419) at a step of 1e-3 along the tangent."""
    base = scene(turb=3.4, sun=[math.sin(math.pi / 2 - ETA) * math.cos(0.6), math.sin(math.pi / 2 - ETA) * math.sin(0.6),
                                math.cos(math.pi / 2 - ETA)])
    em = ss.SunskyEmitter(base, variant, device="host")
    t = em.tangent_tables(param, tangent, on_device=False)
    h = 1e-3

    def staged(sign):
        # through traverse() + update(), as Dr.Jit differentiates: m_sun_dir is used as set
        # (parameters_changed, sunsky.cpp:242-285), not renormalised like the constructor's
        e = ss.SunskyEmitter(base, variant, device="host")
        p = e.traverse()
        if param == "turbidity":
            p["turbidity"] = base["turbidity"] + sign * h * tangent[0]
        elif param == "albedo":
            p["albedo"] = base["albedo"] + sign * h * tangent[0]
        else:
            p["sun_direction"] = [s + sign * h * v for s, v in zip(np.asarray(p["sun_direction"], np.float64), tangent)]
        p.update()
        nch = e.info()["nb_channels"]
        sky = np.concatenate([e.table("sky_params").reshape(nch, 9), e.table("sky_radiance")[:, None]], axis=1)
        return sky.astype(np.float64), e.table("sun_radiance").astype(np.float64)

    (sp, up), (sm, um) = staged(1), staged(-1)
    fd_sky, fd_sun = (sp - sm) / (2 * h), (up - um) / (2 * h)
    scale = np.abs(fd_sky).max(axis=1, keepdims=True) + 1e-12
    # fp32 tables differenced at h = 1e-3: ~1e-4 of each channel's largest entry
    assert np.all(np.abs(t["dsky"] - fd_sky) <= 2e-2 * np.abs(fd_sky) + 2e-3 * scale), \
        np.max(np.abs(t["dsky"] - fd_sky) / (2e-2 * np.abs(fd_sky) + 2e-3 * scale))
    assert np.all(np.abs(t["dsun"] - fd_sun) <= 2e-2 * np.abs(fd_sun) + 2e-3 * (np.abs(fd_sun).max() + 1e-12))
    if param == "sun_direction":
        assert np.abs(t["dsun_local"]).max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["rgb", "spectral"])
@pytest.mark.parametrize("rotated", [False, True])
def test_device_tangent_staging_is_the_host_tangent_bitwise(variant, rotated):
    """f2: the tangent tables eval_jvp / eval_vjp read are staged by the device kernel
    sunsky_stage_tangent (sunsky_staging.h, fp64), bit for bit the host model's
    eval_tangent for every differentiable parameter, after a parameter update too."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = scene()
    d["sun_direction"] = [0.4, 0.3, 0.8]
    if rotated:
        c, s = math.cos(0.5), math.sin(0.5)
        d["to_world"] = np.array([[c, -s, 0, 0], [s, c, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]], np.float32)
    em = ss.SunskyEmitter(d, variant)
    cases = [("turbidity", [1.0]), ("turbidity", [-2.5]), ("albedo", [1.0]), ("albedo", [0.3] * em.info()["nb_channels"]),
             ("sun_direction", [1.0, 0.0, 0.0]), ("sun_direction", [0.1, -0.7, 0.2])]
    for step in range(2):
        for param, tan in cases:
            dev = em.tangent_tables(param, tan, on_device=True)
            hst = em.tangent_tables(param, tan, on_device=False)
            for k in dev:
                assert np.array_equal(dev[k].view(np.uint32), hst[k].view(np.uint32)), (param, tan, k)
        p = em.traverse()
        p["turbidity"] = 7.25
        p["albedo"] = 0.55
        p.update()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["rgb", "spectral"])
def test_sun_disc_tangent_along_sun_direction(variant):
    """the sun-disc part of the sun_direction tangent -- d cos(psi) / d s in the
    limb darkening (sunsky.cpp:631-650) and, for RGB, in the cos(psi) powers of render_sun
    (:572-614), through gamma = unit_angle(s, wo) (:311) -- on lanes well inside the disc,
    alpha/8 <= gamma <= alpha/4 (alpha/2 = the half aperture), which the sun_direction check
    above masks out.  Steps of up to 2h = 4e-4 along tangents orthogonal to s cannot flip
    the disc test there (alpha/4 = 2.3e-3), and the disc radiance is a smooth function of
    cos(gamma) on the scale of the aperture, so the 4-point central differences of the fp64
    oracle are accurate to ~(h / (alpha/4))^4 / 30 ~ 2e-6; their noise is the fp32 rounding
    of the perturbed sun direction the oracle takes (~3e-8 / h).  Below alpha/8 the fp32
    chord wo . ds of the kernel's d gamma cancels (6e-8 / gamma relative), as in the
    reference's own fp32 AD.  JVP per lane and the VJP's sun-axis gradient projected on the
    tangent (sum over the disc lanes with a random cotangent) against them."""
    d = scene()
    em = ss.load_dict(d, variant=variant)
    o32 = O.Oracle(d, variant, "jit", "f32")
    inf = o32.info()
    half = math.acos(inf["cos_cutoff"])
    wo = sun_cone_wo(16384, inf["sun_dir_local"], half, seed=21, scale=0.5)
    gam = np.arccos(np.clip(wo.astype(np.float64) @ inf["sun_dir_local"], -1.0, 1.0))
    wo = wo[gam >= half / 4]
    n = wo.shape[0]
    wi = -wo
    rng = np.random.default_rng(22)
    lam = rng.uniform(330, 710, (4, n)).astype(np.float32)
    lam_o = lam if variant == "spectral" else None
    si = ss.SurfaceInteraction3f(wi=_gpu(wi), wavelengths=torch.from_numpy(lam).cuda() if variant == "spectral" else None)
    s = np.array(d["sun_direction"], np.float64)
    t1 = np.cross(s, [0.0, 0.0, 1.0])
    t1 /= np.linalg.norm(t1)
    t2 = np.cross(s, t1)
    k = 4 if variant == "spectral" else 3
    cot = rng.standard_normal((k, n))
    grad, view = em.eval_vjp(si, torch.from_numpy(cot.astype(np.float32)).cuda())
    g_sun = view["sun_direction"].cpu().numpy().astype(np.float64)
    h = 2e-4
    ev = lambda k, t: O.Oracle(scene(sun=(s + k * h * t) / np.linalg.norm(s + k * h * t)), variant, "jit",  # noqa: E731
                               "f64").eval(wi, lam_o)
    for t in (t1, t2, 0.6 * t1 + 0.8 * t2):
        fd = (8 * (ev(1, t) - ev(-1, t)) - (ev(2, t) - ev(-2, t))) / (12 * h)
        fd = fd.T if variant == "spectral" else fd
        _, dval = em.eval_jvp(si, "sun_direction", list(t))
        dval = dval.cpu().numpy().T.astype(np.float64)
        assert np.abs(fd).max() > 0
        worst = np.max(np.abs(dval - fd) / (2e-3 * np.abs(fd) + 1e-4 * np.abs(fd).max()))
        print(f"{variant} t={np.round(t, 3)}: {n} disc lanes, JVP vs FD worst {worst:.2f}x of the bound")
        check(dval, fd, np.ones_like(dval, bool))
        proj, ref = float(g_sun @ t), float((cot.T * fd).sum())
        mag = float(np.abs(cot.T * fd).sum())
        assert abs(proj - ref) <= 1e-3 * mag, (proj, ref, mag)
