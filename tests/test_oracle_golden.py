"""Pin the CPU oracle against every fixture the reference's own tests hold
for this path.  CPU only."""
import os

import numpy as np
import pytest

import oracle as O
from helpers import (EXR_WAVELENGTHS, SPECIAL_ALBEDO, angles_dict, exr_grid_wi, hemisphere_wo,
                     hour_dict, max_rel, mean_rel)


@pytest.fixture(scope="module")
def spectra(golden_dir):
    return np.load(os.path.join(golden_dir, "sun_spectra.npz"))


@pytest.fixture(scope="module")
def renders(golden_dir):
    return np.load(os.path.join(golden_dir, "sky_renders.npz"))


def test_hw_sun_restatement_reproduces_spd_fixtures(spectra):
    """fp64 restatement of ArHosekSkyModel.c:686-784 == mi.hosek_sun_rad fixtures, bit for bit in fp32."""
    o64 = O.Oracle({"sun_direction": [0, 0, 1], "albedo": 0.0}, "spectral", "jit", "f64")
    o32 = O.Oracle({"sun_direction": [0, 0, 1], "albedo": 0.0}, "spectral", "jit", "f32")
    worst32 = 0.0
    for t, eta, g, rad in zip(spectra["turbidity"], spectra["eta"], spectra["gamma"], spectra["radiance"]):
        got = np.array([o64.hw_sun_radiance(t, w, eta, g) for w in spectra["wavelengths"]])
        np.testing.assert_array_equal(got.astype(np.float32), rad)
        got32 = np.array([o32.hw_sun_radiance(t, w, eta, g) for w in spectra["wavelengths"]])
        worst32 = max(worst32, max_rel(got32, rad))
    assert worst32 < 1e-5


@pytest.mark.parametrize("precision", ["f32", "f64"])
def test04_sun_radiance_through_eval(spectra, precision):
    """test_sunsky.py:154-196 restated on the oracle's eval(): mean rel <= 1e-2 per case."""
    phi = np.pi / 5
    worst = 0.0
    for t, eta, g, rad in zip(spectra["turbidity"], spectra["eta"], spectra["gamma"], spectra["radiance"]):
        theta_ray = np.pi / 2 - eta
        sun_theta = theta_ray - g
        if sun_theta < 0:
            sun_theta = theta_ray + g
        o = O.Oracle(angles_dict(t, phi, sun_theta, 0.0, 0.0, 1.0), "spectral", "jit", precision)
        wl = spectra["wavelengths"].astype(np.float32)
        n = wl.size
        wi = -np.array([[np.cos(phi) * np.sin(theta_ray), np.sin(phi) * np.sin(theta_ray),
                         np.cos(theta_ray)]] * n, dtype=np.float32)
        res = o.eval(wi, wl)
        err = float(np.mean(np.abs(res - rad) / (rad + 1e-6)))
        worst = max(worst, err)
        assert err <= 1e-2, (t, eta, g, err)
    print(f"test04 worst mean-rel ({precision}) = {worst:.3e}")


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("params", [(9.5, 2, 0.2), (12.25, 5.2, 0.0), (18.3, 9.8, 0.5)])
def test01_sky_radiance_rgb(renders, params, precision):
    hour, turb, albedo = params
    o = O.Oracle(hour_dict(turb, hour, albedo, 1.0, 0.0), "rgb", "jit", precision)
    img = o.eval(exr_grid_wi()).reshape(32, 64, 3)
    ref = renders[f"sky_rgb_hour{hour:.2f}_t{turb:.3f}_a{albedo:.3f}"]
    assert mean_rel(img, ref, 0.001) <= 0.017


SPEC_CASES = [
    (np.deg2rad(2), 2, 0.0, "sky_spec_eta0.035_t2.000_a0.000", 0.037),
    (np.deg2rad(20), 5.2, 0.0, "sky_spec_eta0.349_t5.200_a0.000", 0.037),
    (np.deg2rad(45), 9.8, 0.0, "sky_spec_eta0.785_t9.800_a0.000", 0.037),
    (np.deg2rad(60), 4.2, SPECIAL_ALBEDO, "sky_spectrum_special", 0.03),
]


@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("case", SPEC_CASES, ids=[c[3] for c in SPEC_CASES])
def test02_03_sky_radiance_spectral(renders, case, precision):
    eta, turb, albedo, key, tol = case
    o = O.Oracle(angles_dict(turb, 0.0, np.pi / 2 - eta, albedo, 1.0, 0.0), "spectral", "jit", precision)
    wi = exr_grid_wi()
    lam = np.array([np.full(wi.shape[0], w, np.float32) for w in EXR_WAVELENGTHS])
    img = o.eval(wi, lam).T.reshape(32, 64, 10)
    assert mean_rel(img, renders[key], 0.001) <= tol


@pytest.mark.parametrize("variant", ["rgb", "spectral"])
@pytest.mark.parametrize("turb", [2.0, 6.0, 10.0])
def test_oracle_fp32_tracks_fp64_sky(variant, turb):
    """The fp32 restatement stays within 3e-6 relative of fp64 on the sky."""
    d = angles_dict(turb, 0.3, np.deg2rad(45), 0.1, 1.0, 0.0)
    o32 = O.Oracle(d, variant, "jit", "f32")
    o64 = O.Oracle(d, variant, "jit", "f64")
    wo = hemisphere_wo(20000, seed=int(turb))
    if variant == "rgb":
        a, b = o32.eval(-wo), o64.eval(-wo)
    else:
        lam = np.repeat(np.arange(320, 721, 40, dtype=np.float32)[:, None], wo.shape[0], 1)
        a, b = o32.eval(-wo, lam), o64.eval(-wo, lam)
    assert max_rel(a, b) < 3e-6


def test_gauss_legendre_matches_numpy():
    x, w = O.gauss_legendre(200)
    xr, wr = np.polynomial.legendre.leggauss(200)
    np.testing.assert_allclose(x, xr, atol=1e-14)
    np.testing.assert_allclose(w, wr, rtol=1e-10)


def test_sun_coordinates_solar_noon():
    """Default Tokyo record at hour 11.7753: elevation ~76.57 deg."""
    s = O.sun_coordinates(hour=11.7753)
    assert abs(np.linalg.norm(s) - 1) < 1e-6
    elev = np.degrees(np.arcsin(s[2]))
    assert abs(elev - 76.57) < 0.05


def test_invalid_parameters_raise():
    with pytest.raises(ValueError, match="Turbidity"):
        O.Oracle({"turbidity": 11.0})
    with pytest.raises(ValueError, match="sun_direction"):
        O.Oracle({"sun_direction": [0, 0, 1], "hour": 3.0})
    with pytest.raises(ValueError, match="Albedo"):
        O.Oracle({"albedo": 1.5})
