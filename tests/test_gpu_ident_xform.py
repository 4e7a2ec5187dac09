"""The identity-to_world code object (sunsky_kernels_ident.hsaco, DESIGN.md §3 "Identity
to_world"): for an emitter whose to_world is the identity the C ABI launches the same kernels
compiled with to_world / to_local as the identity, which is what the general kernels' runtime
test returns there.  Every entry point must give the general code object's bits
(SUNSKY_AMD_GENERAL_XFORM=1 forces the general one), in both precisions; an emitter with a
rotated to_world keeps the general code object."""
import numpy as np
import pytest
import torch

import sunsky_amd as ss
from helpers import angles_dict, sphere_wo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _run(em, variant, n, seed):
    """The entry points on one set of seeded inputs; a dict of output tensors."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    wi = torch.from_numpy(np.ascontiguousarray(-sphere_wo(n, seed=seed).T)).cuda()
    u = torch.rand((2, n), generator=g, device="cuda")
    u3 = torch.rand((2, n), generator=g, device="cuda")
    spec = variant == "spectral"
    lam = 360.0 + 360.0 * torch.rand((4, n), generator=g, device="cuda") if spec else None
    out = {"eval": em.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam))}
    ds, w = em.sample_direction(ss.Interaction3f(wavelengths=lam), u)
    out.update(sample_d=ds.d, sample_pdf=ds.pdf, sample_w=w)
    out["pdf_direction"] = em.pdf_direction(ss.Interaction3f(), ds)
    out["eval_direction"] = em.eval_direction(ss.Interaction3f(wavelengths=lam), ds)
    ws = torch.rand(n, generator=g, device="cuda") if spec else None
    ray, rw = em.sample_ray(0.0, ws, u, u3)
    out.update(ray_o=ray.o, ray_d=ray.d, ray_w=rw)
    lam_s, lw = em.sample_wavelengths(ss.SurfaceInteraction3f(wi=wi), torch.rand(n, generator=g, device="cuda"))
    out.update(wl=lam_s, wl_w=lw)
    if spec:
        out["nodes"] = em.eval_spectral_broadcast(wi, [float(x) for x in range(320, 721, 40)])
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("precision", ["fast", "reference"])
@pytest.mark.parametrize("variant", ["rgb", "spectral"])
def test_identity_code_object_bitwise_general(variant, precision, monkeypatch):
    d = angles_dict(3.0, 0.7, np.deg2rad(55.0), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, variant, precision=precision)
    n = (1 << 18) + 13   # ragged: the v1 tails as well
    ident = _run(em, variant, n, 5)
    monkeypatch.setenv("SUNSKY_AMD_GENERAL_XFORM", "1")
    general = _run(em, variant, n, 5)
    for k in ident:
        a, b = ident[k], general[k]
        assert a.shape == b.shape, k
        same = (a.view(torch.int32) == b.view(torch.int32)) | (torch.isnan(a) & torch.isnan(b))
        assert bool(same.all()), f"{k}: {int((~same).sum())} lanes differ"


def test_rotated_to_world_keeps_general_code_object(monkeypatch):
    """A rotated emitter never takes the identity code object: forcing the general one is a
    no-op for it, bit for bit."""
    c, s = np.cos(0.4), np.sin(0.4)
    d = dict(angles_dict(3.0, 0.7, np.deg2rad(55.0), 0.3, 1.0, 1.0),
             to_world=np.array([[c, -s, 0, 0], [s, c, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]], np.float32))
    em = ss.SunskyEmitter(d, "rgb")
    n = 1 << 16
    a = _run(em, "rgb", n, 9)
    monkeypatch.setenv("SUNSKY_AMD_GENERAL_XFORM", "1")
    b = _run(em, "rgb", n, 9)
    for k in a:
        assert torch.equal(a[k].view(torch.int32), b[k].view(torch.int32)), k


@pytest.mark.parametrize("var,obj,msg", [
    ("SUNSKY_AMD_CODE_OBJECT", "sunsky_kernels_ident.hsaco", "is an identity-to_world build"),
    ("SUNSKY_AMD_CODE_OBJECT_IDENT", "sunsky_kernels.hsaco", "is not an identity-to_world build")])
def test_code_object_override_of_the_wrong_form_is_refused(var, obj, msg):
    """An identity build (it exports sunsky_xform_identity_marker) named as the general code
    object would drop every rotated to_world without an error: the C ABI refuses it at load,
    and a general build named as the identity object too."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, **{var: os.path.join(os.path.dirname(ss.CODE_OBJECT), obj)})
    code = ("import sys, torch; sys.path.insert(0, %r); import sunsky_amd as ss\n"
            "em = ss.load_dict({'type': 'sunsky', 'sun_direction': [0.3, 0.4, 0.866]})\n"
            "em.eval(ss.SurfaceInteraction3f(wi=-torch.ones((3, 64), device='cuda') / 3 ** 0.5))\n"
            "torch.cuda.synchronize()\n" % os.path.dirname(os.path.dirname(ss.__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0, "the wrong-form code object was accepted"
    assert msg in r.stderr, r.stderr[-2000:]


def test_general_code_object_override_alone_names_the_identity_module():
    """with only SUNSKY_AMD_CODE_OBJECT set, identity-to_world emitters still run the
    installed identity module; the C ABI says so once on stderr, so an A/B of a probe build
    cannot silently time the installed kernels."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, SUNSKY_AMD_CODE_OBJECT=ss.CODE_OBJECT)
    env.pop("SUNSKY_AMD_CODE_OBJECT_IDENT", None)
    code = ("import sys, torch; sys.path.insert(0, %r); import sunsky_amd as ss\n"
            "em = ss.load_dict({'type': 'sunsky', 'sun_direction': [0.3, 0.4, 0.866]})\n"
            "em.eval(ss.SurfaceInteraction3f(wi=-torch.ones((3, 64), device='cuda') / 3 ** 0.5))\n"
            "torch.cuda.synchronize()\n" % os.path.dirname(os.path.dirname(ss.__file__)))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "SUNSKY_AMD_CODE_OBJECT is set but SUNSKY_AMD_CODE_OBJECT_IDENT is not" in r.stderr, r.stderr[-2000:]
    assert "sunsky_kernels_ident.hsaco" in r.stderr
