"""chi^2 sampling tests of the reference (test_sunsky.py:227-293, test06/07)
on the GPU kernels, plus CPU self-checks of the chi^2 harness (tests/chi2.py)."""
import math

import numpy as np
import pytest
import torch

import sunsky_amd as ss
from chi2 import ChiSquareTest, SphericalDomain, emitter_adapter, pool_chi2

SIN_OFFSET = 0.00775                     # test_sunsky.py:9
PHI_SUN = -4 * math.pi / 5               # test_sunsky.py:241, :270


def sky_dict(turb, sun_theta, **kw):
    st, ct = math.sin(sun_theta), math.cos(sun_theta)
    d = {"type": "sunsky", "sun_direction": [math.cos(PHI_SUN) * st, math.sin(PHI_SUN) * st, ct],
         "turbidity": turb, "albedo": 0.5}
    d.update(kw)
    return d


# ------------------------------------------------------------ harness (CPU)
def _uniform_sphere(u):
    z = 1 - 2 * u[0]
    r = torch.sqrt(torch.clamp(1 - z * z, min=0))
    phi = 2 * math.pi * u[1]
    return torch.stack([r * torch.cos(phi), r * torch.sin(phi), z])


def test_harness_accepts_matching_pdf():
    t = ChiSquareTest(SphericalDomain(), _uniform_sphere, lambda d: torch.full((d.shape[1],), 1 / (4 * math.pi)),
                      sample_count=400_000, res=31, ires=4, device="cpu")
    assert t.run(), t.messages


def test_harness_rejects_wrong_pdf():
    # cos-weighted claim for uniform samples
    t = ChiSquareTest(SphericalDomain(), _uniform_sphere,
                      lambda d: torch.clamp(d[2], min=0) / math.pi + 0.0 * d[0],
                      sample_count=400_000, res=31, ires=4, device="cpu")
    assert not t.run()


def test_pool_chi2_matches_reference_rules():
    # math.h:325-352 by hand: cells 0/0 skipped, cells < 5 pooled until > 5
    obs = np.array([0, 1, 2, 3, 10, 20], float)
    exp = np.array([0, 2, 2, 2, 10, 20], float)
    chsq, dof, n_in, n_out = pool_chi2(obs, exp, 5)
    assert (n_in, n_out) == (3, 1)
    assert dof == 3 - 1
    assert chsq == pytest.approx((6 - 6) ** 2 / 6)


# ------------------------------------------------------------ GPU kernels
CASES = [(t, th) for t in (2.2, 4.8, 6.0) for th in (math.radians(20), math.radians(50))]


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("turb,sun_theta", CASES)
def test06_sky_sampling(turb, sun_theta):
    em = ss.load_dict(sky_dict(turb, sun_theta, sun_scale=0.0))
    sample, pdf = emitter_adapter(em)
    t = ChiSquareTest(SphericalDomain(SIN_OFFSET), sample, pdf, sample_count=100_000_000, res=215, ires=32)
    ok = t.run()
    print(t.messages)
    assert ok, t.messages


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("turb,sun_theta", CASES)
def test07_sun_and_sky_sampling(turb, sun_theta):
    # sun_aperture 30 deg, as test_sunsky.py:275-276, to resolve the sun at chi^2's resolution
    em = ss.load_dict(sky_dict(turb, sun_theta, sun_aperture=30.0))
    sample, pdf = emitter_adapter(em)
    t = ChiSquareTest(SphericalDomain(SIN_OFFSET), sample, pdf, sample_count=100_000_000, res=215, ires=32)
    ok = t.run()
    print(t.messages)
    assert ok, t.messages


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("semantics", ["jit", "scalar"])
def test07_spectral_and_scalar_variants(semantics):
    """The same chi^2 bar for the spectral variant and the scalar variants' w_sky = 0.5."""
    em = ss.load_dict(sky_dict(3.0, math.radians(35), sun_aperture=30.0), variant="spectral", semantics=semantics)

    def sample_func(u):
        wl = torch.full((4, u.shape[1]), 550.0, device=u.device)
        ds, _ = em.sample_direction(ss.Interaction3f(wavelengths=wl), u)
        return ds.d

    def pdf_func(d):
        return em.pdf_direction(ss.Interaction3f(), ss.DirectionSample3f(d=d))

    t = ChiSquareTest(SphericalDomain(SIN_OFFSET), sample_func, pdf_func, sample_count=50_000_000, res=215, ires=32)
    ok = t.run()
    print(t.messages)
    assert ok, t.messages


def test_two_sample_chi2_self_check():
    from chi2 import two_sample_chi2
    rng = np.random.default_rng(4)
    p = rng.dirichlet(np.ones(400))
    a = rng.multinomial(2_000_000, p)
    b = rng.multinomial(300_000, p)
    assert two_sample_chi2(a, b)[2] > 0.01
    q = p * (1 + 0.05 * np.sin(np.arange(400)))
    c = rng.multinomial(300_000, q / q.sum())
    assert two_sample_chi2(a, c)[2] < 1e-6
