"""The sky sampling density against the environment map built from the sky (SURVEY.md §8f
row 4; sunsky-testing/sky_data_test.py:43-79 `plot_pdf`): the sky (sun_scale 0) is baked
to a lat-long image over helpers.py get_spherical_rays, an `envmap` emitter is built from it,
and its pdf_direction is compared with the emitter's tGMM pdf_direction over
get_north_hemisphere_rays(eps = 0.15) with relative_error = |pdf_ref - pdf_tgmm| /
(pdf_ref + 0.01).

The reference script only plots the two; the gates here were measured on the oracle
(mean relative error 0.044-0.065, correlation 0.988-0.998 over three skies) and sit above
them with margin.  Parity of the product path: the GPU bake (sunsky_bake_latlong) and the GPU
pdf_direction give the same envmap pdf / tGMM pdf as the oracle, and so the same statistics.

`envmap_pdf` restates the envmap plugin's pdf (src/emitters/envmap.cpp:145-233 construction,
:461-477 pdf_direction) over Hierarchical2D<0> (include/mitsuba/core/distr_2d.h:380-455
normalisation, :665-700 eval) in the z-up frame of the bake: the reference hands the envmap
ds.d = (d.y, d.z, -d.x), so its (atan2(d.x, -d.z), acos(d.y)) are (phi, theta) of d here.
Test infrastructure only."""
import math

import numpy as np
import pytest

import oracle as O

LUM = (np.float32(0.212671), np.float32(0.715160), np.float32(0.072169))   # spectrum.h:431-434
H, W = 256, 512                      # temp_shape = (render_shape[0] * 2, render_shape[1])
SKIES = [(6.5, 0.5), (3.0, 0.2), (2.0, 0.8)]   # (turbidity, albedo); the first is plot_pdf's


def envmap_pdf(img, d):
    """pdf_direction of an envmap built from img (H, W, 3) RGB lat-long, at unit d (n, 3)."""
    h, w, _ = img.shape
    lum = (img[..., 0] * LUM[0] + img[..., 1] * LUM[1] + img[..., 2] * LUM[2]).astype(np.float32)
    theta_scale = np.float32(1.0 / (h - 1) * np.pi)
    lum = lum * np.sin(np.arange(h, dtype=np.float32) * theta_scale)[:, None]
    lum = np.concatenate([lum, lum[:, :1]], axis=1).astype(np.float64)     # last column mirrors the first
    avg = 0.25 * (lum[:-1, :-1] + lum[:-1, 1:] + lum[1:, :-1] + lum[1:, 1:])
    scale = w * (h - 1) / avg.sum()                                          # n_patches / sum
    d = np.asarray(d, dtype=np.float64)
    u = np.arctan2(d[:, 1], d[:, 0]) / (2 * np.pi) - 0.5 / w                 # uv.x -= .5 / (shape(1) - 1)
    v = np.arccos(np.clip(d[:, 2], -1, 1)) / np.pi
    u -= np.floor(u)
    v -= np.floor(v)
    px, py = np.clip(u, 0, 1) * w, np.clip(v, 0, 1) * (h - 1)
    ox, oy = np.minimum(px.astype(np.int64), w - 1), np.minimum(py.astype(np.int64), h - 2)
    fx, fy = px - ox, py - oy
    val = ((1 - fx) * (1 - fy) * lum[oy, ox] + fx * (1 - fy) * lum[oy, ox + 1] + (1 - fx) * fy * lum[oy + 1, ox]
           + fx * fy * lum[oy + 1, ox + 1]) * scale
    inv_sin = 1.0 / np.sqrt(np.maximum(d[:, 0] ** 2 + d[:, 1] ** 2, np.finfo(np.float32).eps ** 2))
    return val * inv_sin / (2 * np.pi ** 2)


def _sph(phi, theta):
    return np.stack([np.cos(phi) * np.sin(theta), np.sin(phi) * np.sin(theta), np.cos(theta)], -1)


def sky_dict(t, a):
    eta, phi_sun = math.radians(45), math.pi / 2
    st, ct = math.sin(math.pi / 2 - eta), math.cos(math.pi / 2 - eta)
    return {"type": "sunsky", "sun_direction": [math.cos(phi_sun) * st, math.sin(phi_sun) * st, ct],
            "sun_scale": 0.0, "turbidity": t, "albedo": a}


def hemisphere_dirs():
    """get_north_hemisphere_rays((128, 512), eps=0.15)"""
    p, t = np.meshgrid(np.linspace(0, 2 * np.pi, 512, dtype=np.float32),
                       np.linspace(0.15, np.pi / 2 - 0.15, 128, dtype=np.float32))
    return _sph(p, t).reshape(-1, 3).astype(np.float32)


def spherical_dirs():
    """get_spherical_rays((H, W)): theta = linspace(0, pi, H) rows, phi = linspace(0, 2 pi, W)"""
    p, t = np.meshgrid(np.linspace(0, 2 * np.pi, W, dtype=np.float32), np.linspace(0, np.pi, H, dtype=np.float32))
    return _sph(p, t).reshape(-1, 3).astype(np.float32)


def stats(ref, tgmm):
    rel = np.abs(ref - tgmm) / (ref + 0.01)
    return {"mean_rel": rel.mean(), "p99_rel": np.quantile(rel, 0.99), "corr": np.corrcoef(ref, tgmm)[0, 1]}


def check(s):
    assert s["mean_rel"] < 0.09 and s["p99_rel"] < 0.3 and s["corr"] > 0.98, s


def test_envmap_restatement_is_a_density():
    """The restated envmap pdf integrates to 1 over the sphere (any positive image)."""
    rng = np.random.default_rng(1)
    img = rng.uniform(0.1, 2.0, (64, 128, 3)).astype(np.float32)
    mu, wmu = np.polynomial.legendre.leggauss(400)
    phi = (np.arange(800) + 0.5) * (2 * np.pi / 800)
    M, P = np.meshgrid(mu, phi, indexing="ij")
    st = np.sqrt(1 - M * M)
    d = np.stack([st * np.cos(P), st * np.sin(P), M], -1).reshape(-1, 3)
    total = (envmap_pdf(img, d).reshape(M.shape) * wmu[:, None]).sum() * (2 * np.pi / 800)
    assert abs(total - 1) < 2e-3, total


@pytest.mark.parametrize("sky", SKIES)
def test_tgmm_pdf_tracks_envmap_pdf_oracle(sky):
    em = O.Oracle(sky_dict(*sky), "rgb", "jit", "f32")
    img = em.eval(-spherical_dirs()).reshape(H, W, 3).astype(np.float32)
    hd = hemisphere_dirs()
    check(stats(envmap_pdf(img, hd), em.pdf_direction(hd).astype(np.float64)))


@pytest.mark.gpu
@pytest.mark.parametrize("sky", SKIES)
def test_tgmm_pdf_tracks_envmap_pdf_gpu(sky):
    """Product path: sunsky_bake_latlong -> envmap pdf, sunsky_pdf_direction -> tGMM pdf.
    Both agree with the oracle's pipeline, and pass the same gates."""
    import torch
    import sunsky_amd as ss
    em = ss.SunskyEmitter(sky_dict(*sky), "rgb")
    img = em.bake_latlong(W, H).permute(1, 2, 0).cpu().numpy()          # (H, W, 3)
    hd = hemisphere_dirs()
    ds = ss.DirectionSample3f(d=torch.from_numpy(hd.T.copy()).cuda())
    tgmm = em.pdf_direction(ss.Interaction3f(), ds).cpu().numpy().astype(np.float64)
    ref = envmap_pdf(img, hd)
    o = O.Oracle(sky_dict(*sky), "rgb", "jit", "f32")
    o.override_w_sky(em.sky_sampling_w)
    o_img = o.eval(-spherical_dirs()).reshape(H, W, 3).astype(np.float32)
    o_ref, o_tgmm = envmap_pdf(o_img, hd), o.pdf_direction(hd).astype(np.float64)
    assert np.max(np.abs(ref - o_ref) / o_ref) < 1e-4
    assert np.max(np.abs(tgmm - o_tgmm) / np.maximum(o_tgmm, 1e-6)) < 1e-5
    s, so = stats(ref, tgmm), stats(o_ref, o_tgmm)
    check(s)
    assert abs(s["mean_rel"] - so["mean_rel"]) < 1e-4, (s, so)
