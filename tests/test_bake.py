"""Lat-long bake (sunsky_bake_latlong), the envmap construction of
sunsky-testing/sky_data_test.py:58-79 over helpers.py get_spherical_rays:
compared with eval() of the same directions generated on the host."""
import math

import numpy as np
import pytest
import torch

import sunsky_amd as ss
from helpers import angles_dict

pytestmark = pytest.mark.gpu


def grid_dirs(w, h, theta=(0.0, math.pi), phi=(0.0, 2 * math.pi)):
    """dr.meshgrid(linspace(phi), linspace(theta)) -> to_spherical (helpers.py:4-9, 27-36)."""
    dt = np.float32((theta[1] - theta[0]) / (h - 1)) if h > 1 else np.float32(0)
    dp = np.float32((phi[1] - phi[0]) / (w - 1)) if w > 1 else np.float32(0)
    th = (np.arange(h, dtype=np.float32) * dt + np.float32(theta[0])).astype(np.float32)
    ph = (np.arange(w, dtype=np.float32) * dp + np.float32(phi[0])).astype(np.float32)
    P, T = np.meshgrid(ph, th)
    d = np.stack([np.cos(P) * np.sin(T), np.sin(P) * np.sin(T), np.cos(T)], 0).reshape(3, -1).astype(np.float32)
    return d, T.reshape(-1)


def compare(bake, ref, theta):
    keep = np.abs(theta - np.pi / 2) > np.radians(2)          # horizon: direction-rounding sensitive
    b, r = bake[:, keep].astype(np.float64), ref[:, keep].astype(np.float64)
    rel = np.abs(b - r) / np.maximum(np.abs(r), 1e-6 * np.abs(r).max())
    assert rel.max() < 1e-4, rel.max()
    below = theta > np.pi / 2 + 1e-3
    assert np.all(bake[:, below] == 0)


@pytest.mark.parametrize("size", [(512, 256), (37, 13)])
def test_bake_rgb_matches_eval(size):
    w, h = size
    d = angles_dict(4.0, 0.3, math.radians(50), 0.2, 1.0, 1.0)
    em = ss.load_dict(d)
    img = em.bake_latlong(w, h)
    torch.cuda.synchronize()
    dirs, theta = grid_dirs(w, h)
    ref = em.eval(ss.SurfaceInteraction3f(wi=torch.from_numpy(-dirs).cuda()))
    compare(img.reshape(3, -1).cpu().numpy(), ref.cpu().numpy(), theta)


def test_bake_spectral_matches_broadcast_eval():
    d = angles_dict(3.0, -0.5, math.radians(30), 0.3, 1.0, 1.0)
    em = ss.load_dict(d, variant="spectral")
    lam = [400.0, 550.0, 700.0, 720.0]
    img = em.bake_latlong(256, 128, theta=(0.0, math.pi / 2), wavelengths=lam)
    torch.cuda.synchronize()
    dirs, theta = grid_dirs(256, 128, theta=(0.0, math.pi / 2))
    ref = em.eval_spectral_broadcast(torch.from_numpy(-dirs).cuda(), lam)
    compare(img.reshape(4, -1).cpu().numpy(), ref.cpu().numpy(), theta)


def test_bake_argument_errors():
    em = ss.load_dict(angles_dict(4.0, 0.3, math.radians(50), 0.2, 1.0, 1.0))
    with pytest.raises(ValueError):
        em.bake_latlong(0, 10)
    spec = ss.load_dict(angles_dict(4.0, 0.3, math.radians(50), 0.2, 1.0, 1.0), variant="spectral")
    with pytest.raises(ValueError):
        spec.bake_latlong(8, 8)
