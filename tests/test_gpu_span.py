"""Batches beyond one step per lane.  The parity tests run at sizes where every lane of the grid
takes one step; past ~16.8M directions (64 workgroups x 256 lanes x 4 directions per CU on 256
CUs) the per-ray spectral eval and the node kernel walk two or more steps of a contiguous span
per workgroup (`span_steps`) and the other kernels loop grid-stride.  A 25M batch
(two steps, ragged tail) must give the bits of the same inputs evaluated in 4M chunks (one step
each): a size-independent property of the work split, checked bitwise."""
import numpy as np
import pytest
import torch

import sunsky_amd as ss
from helpers import angles_dict

pytestmark = pytest.mark.gpu

N = 3 * (1 << 23) + 3     # 25,165,827: two steps per lane, a 3-direction tail
CHUNK = 1 << 22           # one step per lane


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _emitter(variant, rotated):
    d = angles_dict(3.0, 0.7, np.deg2rad(50.0), 0.3, 1.0, 1.0)
    if rotated:
        c, s = np.cos(0.4), np.sin(0.4)
        d["to_world"] = np.array([[c, -s, 0, 0], [s, c, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]], np.float32)
    return ss.SunskyEmitter(d, variant)


def _wi(n, g):
    """-wo for wo uniform over the upper hemisphere (cos theta = u1), (3, n) on the device."""
    u = torch.rand((2, n), generator=g, device="cuda")
    st = torch.sqrt(torch.clamp(1 - u[0] * u[0], min=0))
    ph = 2 * np.pi * u[1]
    return (-torch.stack([st * torch.cos(ph), st * torch.sin(ph), u[0]])).contiguous()


def _chunked(fn, n):
    return torch.cat([fn(a, min(a + CHUNK, n)) for a in range(0, n, CHUNK)], dim=-1)


def _same_bits(full, part):
    assert full.shape == part.shape
    same = (full.view(torch.int32) == part.view(torch.int32)) | (torch.isnan(full) & torch.isnan(part))
    assert bool(same.all()), f"{int((~same).sum())} lanes differ"


@pytest.mark.parametrize("rotated", [False, True])
def test_per_ray_spectral_eval_beyond_one_step(rotated):
    em = _emitter("spectral", rotated)
    g = torch.Generator(device="cuda").manual_seed(3)
    wi = _wi(N, g)
    lam = 360.0 + 360.0 * torch.rand((4, N), generator=g, device="cuda")
    full = em.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam))
    part = _chunked(lambda a, b: em.eval(ss.SurfaceInteraction3f(wi=wi[:, a:b].contiguous(),
                                                                 wavelengths=lam[:, a:b].contiguous())), N)
    _same_bits(full, part)


@pytest.mark.parametrize("rotated", [False, True])
def test_node_kernel_beyond_one_step(rotated):
    em = _emitter("spectral", rotated)
    g = torch.Generator(device="cuda").manual_seed(4)
    wi = _wi(N, g)
    lams = [float(x) for x in range(320, 721, 40)]
    full = em.eval_spectral_broadcast(wi, lams)
    part = _chunked(lambda a, b: em.eval_spectral_broadcast(wi[:, a:b].contiguous(), lams), N)
    _same_bits(full, part)


def test_rgb_eval_sampling_and_pdf_beyond_one_step():
    em = _emitter("rgb", False)
    g = torch.Generator(device="cuda").manual_seed(5)
    wi = _wi(N, g)
    _same_bits(em.eval(ss.SurfaceInteraction3f(wi=wi)),
               _chunked(lambda a, b: em.eval(ss.SurfaceInteraction3f(wi=wi[:, a:b].contiguous())), N))
    u = torch.rand((2, N), generator=g, device="cuda")
    ds, w = em.sample_direction(ss.Interaction3f(), u)
    parts = [em.sample_direction(ss.Interaction3f(), u[:, a:min(a + CHUNK, N)].contiguous())
             for a in range(0, N, CHUNK)]
    _same_bits(ds.d, torch.cat([p[0].d for p in parts], dim=-1))
    _same_bits(ds.pdf, torch.cat([p[0].pdf for p in parts], dim=-1))
    _same_bits(w, torch.cat([p[1] for p in parts], dim=-1))
    pdf = em.pdf_direction(ss.Interaction3f(), ds)
    _same_bits(pdf, torch.cat([em.pdf_direction(ss.Interaction3f(), p[0]) for p in parts], dim=-1))
