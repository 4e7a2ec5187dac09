"""Empty and tiny batches.  A Mitsuba wavefront can hold any number of rays, including none;
the reference computes every lane the same way whatever the wavefront's size.  Here a batch
of k rays (k = 0: an empty call that must succeed and write nothing; k = 1..7: the 16-byte
vector kernels' scalar tails only) must give the bits of the same rays inside a larger batch,
for every batch entry point of both variants."""
import numpy as np
import pytest
import torch

import sunsky_amd as ss
from helpers import angles_dict, sphere_wo

pytestmark = pytest.mark.gpu

N = 4099
SIZES = [0, 1, 2, 3, 5, 7]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _inputs(variant, n, seed=21):
    g = torch.Generator(device="cuda").manual_seed(seed)
    wi = torch.from_numpy(np.ascontiguousarray(-sphere_wo(n, seed=seed).T)).cuda()
    u = torch.rand((2, n), generator=g, device="cuda")
    u3 = torch.rand((2, n), generator=g, device="cuda")
    ws = torch.rand(n, generator=g, device="cuda")
    lam = 360.0 + 360.0 * torch.rand((4, n), generator=g, device="cuda") if variant == "spectral" else None
    return dict(wi=wi, u=u, u3=u3, ws=ws, lam=lam)


def _head(x, k):
    return None if x is None else x[..., :k].contiguous()


def _run(em, variant, inp):
    spec = variant == "spectral"
    wi, u, u3, ws, lam = inp["wi"], inp["u"], inp["u3"], inp["ws"], inp["lam"]
    out = {"eval": em.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam))}
    ds, w = em.sample_direction(ss.Interaction3f(wavelengths=lam), u)
    out.update(sample_d=ds.d, sample_pdf=ds.pdf, sample_w=w)
    out["pdf_direction"] = em.pdf_direction(ss.Interaction3f(), ds)
    out["eval_direction"] = em.eval_direction(ss.Interaction3f(wavelengths=lam), ds)
    ray, rw = em.sample_ray(0.0, ws if spec else None, u, u3)
    out.update(ray_o=ray.o, ray_d=ray.d, ray_w=rw)
    lam_s, lw = em.sample_wavelengths(ss.SurfaceInteraction3f(wi=wi), ws)
    out.update(wl=lam_s, wl_w=lw)
    if spec:
        out["nodes"] = em.eval_spectral_broadcast(wi, [float(x) for x in range(320, 721, 40)])
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("variant", ["rgb", "spectral"])
@pytest.mark.parametrize("precision", ["fast", "reference"])
def test_tiny_and_empty_batches_match_the_large_batch(variant, precision):
    d = angles_dict(3.0, 0.7, np.deg2rad(55.0), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, variant, precision=precision)
    inp = _inputs(variant, N)
    big = _run(em, variant, inp)
    for k in SIZES:
        small = _run(em, variant, {key: _head(v, k) for key, v in inp.items()})
        for name, a in small.items():
            b = big[name][..., :k]
            assert a.shape == b.shape, (k, name, tuple(a.shape), tuple(b.shape))
            same = (a.view(torch.int32) == b.view(torch.int32)) | (torch.isnan(a) & torch.isnan(b))
            assert bool(same.all()), f"k={k} {name}: {int((~same).sum())} lanes differ"
