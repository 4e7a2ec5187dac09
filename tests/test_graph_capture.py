"""The hot-path entry points are stream-ordered, allocate nothing on the device and make
no host-synchronous calls, so a caller can capture them into a hipGraph
(include/sunsky_amd.h).  Captured with torch.cuda.graph (hipStreamBeginCapture on ROCm):
replays equal the eager calls bit for bit, and a replay after the inputs change in place
equals an eager call on the new inputs."""
import numpy as np
import pytest
import torch

import sunsky_amd as ss
from helpers import angles_dict, hemisphere_wo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _inputs(n, seed):
    wo = np.ascontiguousarray(hemisphere_wo(n, seed).T.astype(np.float32))
    u = np.random.default_rng(seed + 100).random((2, n), dtype=np.float32)
    return torch.from_numpy(-wo).cuda(), torch.from_numpy(u).cuda()


@pytest.mark.parametrize("variant", ["rgb", "spectral"])
def test_eval_and_sampling_replay_bitwise(variant):
    em = ss.SunskyEmitter(angles_dict(3.0, 0.3, np.deg2rad(50), 0.3, 1.0, 1.0), variant)
    n = 1 << 16
    wi, u = _inputs(n, 1)
    lam = torch.full((4, n), 550.0, device="cuda") + torch.arange(4, device="cuda").view(4, 1) * 37.0

    def step():
        si = ss.SurfaceInteraction3f(wi=wi, wavelengths=lam if variant == "spectral" else None)
        it = ss.Interaction3f(wavelengths=lam if variant == "spectral" else None)
        e = em.eval(si)
        ds, w = em.sample_direction(it, u)
        p = em.pdf_direction(it, ds)
        dl, wl = em.sample_direction(it, u, positions=False)   # the LEAN (RGB: wave-sorted) kernel
        return e, ds.d, ds.pdf, w, p, dl.d, dl.pdf, wl

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()                                   # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        captured = step()
    g.replay()
    torch.cuda.synchronize()
    eager = step()
    torch.cuda.synchronize()
    for a, b in zip(captured, eager):
        assert torch.equal(a, b)
    wi2, u2 = _inputs(n, 2)
    wi.copy_(wi2)
    u.copy_(u2)
    g.replay()
    torch.cuda.synchronize()
    eager2 = step()
    torch.cuda.synchronize()
    for a, b, old in zip(captured, eager2, eager):
        assert torch.equal(a, b)
        assert not torch.equal(a, old)


def test_replay_reads_the_updated_emitter_state():
    """Kernels read the emitter state from device memory (include/sunsky_amd.h), so a graph
    captured before params.update() replays with the new parameters: equal to an eager call
    after the update, different from the pre-update result."""
    em = ss.SunskyEmitter(angles_dict(3.0, 0.3, np.deg2rad(50), 0.3, 1.0, 1.0), "rgb")
    n = 1 << 14
    wi, _ = _inputs(n, 3)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        em.eval(ss.SurfaceInteraction3f(wi=wi))
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        captured = em.eval(ss.SurfaceInteraction3f(wi=wi))
    g.replay()
    torch.cuda.synchronize()
    before = captured.clone()
    params = em.traverse()
    params["turbidity"] = 6.5
    params.update()
    g.replay()
    torch.cuda.synchronize()
    eager = em.eval(ss.SurfaceInteraction3f(wi=wi))
    torch.cuda.synchronize()
    assert torch.equal(captured, eager)
    assert not torch.equal(captured, before)


@pytest.mark.parametrize("variant", ["rgb", "spectral"])
def test_replay_after_a_to_world_update(variant):
    """An emitter with the identity to_world launches the identity code object eagerly
    (DESIGN.md §3), but a captured launch takes the general one: a graph captured before an
    update to a rotated to_world replays with the rotation, equal to an eager call after the
    update (which takes the general code object), and eager calls before the update equal
    the captured replay before it."""
    em = ss.SunskyEmitter(angles_dict(3.0, 0.3, np.deg2rad(50), 0.3, 1.0, 1.0), variant)
    n = 1 << 14
    wi, u = _inputs(n, 5)
    lam = torch.full((4, n), 500.0, device="cuda") + torch.arange(4, device="cuda").view(4, 1) * 41.0
    spec = variant == "spectral"

    def step():
        e = em.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam if spec else None))
        ds, w = em.sample_direction(ss.Interaction3f(wavelengths=lam if spec else None), u, positions=False)
        p = em.pdf_direction(ss.Interaction3f(), ds)
        return e, ds.d, ds.pdf, w, p

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        captured = step()
    g.replay()
    torch.cuda.synchronize()
    eager = step()
    torch.cuda.synchronize()
    for a, b in zip(captured, eager):
        assert torch.equal(a, b)
    c, s_ = np.cos(0.5), np.sin(0.5)
    params = em.traverse()
    params["to_world"] = np.array([[c, 0, s_, 0], [0, 1, 0, 0], [-s_, 0, c, 0], [0, 0, 0, 1]], np.float32)
    params.update()
    g.replay()
    torch.cuda.synchronize()
    eager = step()
    torch.cuda.synchronize()
    for a, b in zip(captured, eager):
        assert torch.equal(a, b)
    assert not torch.equal(captured[0], eager[0].new_zeros(eager[0].shape))


def test_direct_diffuse_with_visibility_replays_bitwise():
    """The occluded caller pair (rays, then shading with the tracer's verdicts) captures too."""
    em = ss.SunskyEmitter(angles_dict(3.0, 0.3, np.deg2rad(50), 0.3, 1.0, 1.0), "rgb")
    n, spp = 1 << 14, 2
    nrm = torch.nn.functional.normalize(torch.rand((3, n), device="cuda") + 0.2, dim=0)

    def step():
        e_d, b_d = em.direct_diffuse_rays(nrm, 4, spp)
        vis = ((e_d[2] >= 0.4).to(torch.uint8) + 2 * (b_d[2] >= 0.4).to(torch.uint8))
        return em.direct_diffuse(nrm, 4, spp, visibility=vis)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        captured = step()
    g.replay()
    torch.cuda.synchronize()
    eager = step()
    torch.cuda.synchronize()
    assert torch.equal(captured, eager)


def test_update_is_refused_inside_a_capture():
    """parameters_changed_async is a host + stream operation (include/sunsky_amd.h): on a
    capturing stream it raises and changes nothing -- the parameter keeps its committed value,
    the captured eval replays the old state, and the same update outside the capture works."""
    d = angles_dict(3.0, 0.3, np.deg2rad(50), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, "rgb")
    n = 1 << 12
    wi, _ = _inputs(n, 5)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        em.eval(ss.SurfaceInteraction3f(wi=wi))
    torch.cuda.current_stream().wait_stream(side)
    before = em.eval(ss.SurfaceInteraction3f(wi=wi)).clone()
    params = em.traverse()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        captured = em.eval(ss.SurfaceInteraction3f(wi=wi))
        params["turbidity"] = 6.5
        with pytest.raises(ValueError, match="hipGraph"):
            params.update()
    assert em.get_param("turbidity") == 3.0 and params["turbidity"] == 3.0
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(captured, before)
    params["turbidity"] = 6.5
    params.update()
    fresh = ss.SunskyEmitter(dict(d, turbidity=6.5), "rgb")
    assert torch.equal(em.eval(ss.SurfaceInteraction3f(wi=wi)), fresh.eval(ss.SurfaceInteraction3f(wi=wi)))


def _inject(em, count):
    ss._capi.check(ss.lib().sunsky_emitter_inject_staging_fault(em._h, count))


def test_update_rejected_by_the_device_staging_restores_the_previous_state():
    """A negative wavelength-distribution node found by the device staging (the check of
    ContinuousDistribution's constructor, distr_1d.h) rejects the update as the reference's
    parameters_changed does: the next read-back raises once, the previous parameters are
    restored and restaged on the device, and later calls see the old state.  The status is
    forced with the test-only sunsky_emitter_inject_staging_fault."""
    d = angles_dict(3.0, 0.3, np.deg2rad(50), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, "spectral")
    n = 1 << 12
    wi, _ = _inputs(n, 6)
    lam = torch.full((4, n), 550.0, device="cuda")
    before = em.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)).clone()
    params = em.traverse()
    params["turbidity"] = 6.5
    _inject(em, 1)
    params.update()                        # async: nothing waits for the device
    with pytest.raises(ValueError, match="non-negative"):
        em.info()
    assert em.info()["turbidity"] == 3.0 and em.get_param("turbidity") == 3.0
    assert torch.equal(em.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)), before)
    np.testing.assert_array_equal(em.table("sky_params"), ss.SunskyEmitter(d, "spectral").table("sky_params"))
    params = em.traverse()
    params["turbidity"] = 6.5
    params.update()
    fresh = ss.SunskyEmitter(dict(d, turbidity=6.5), "spectral")
    assert torch.equal(em.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)),
                       fresh.eval(ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)))


@pytest.mark.parametrize("second", ["accepted", "rejected"])
def test_two_queued_updates_with_a_rejection(second):
    """two async updates queued before a read-back.  The rejection status is
    sticky across stagings, so a rejected update followed by an accepted one still reports
    the error, and two rejected ones revert to the last ACCEPTED state (not to the first
    rejected snapshot); the emitter then evaluates exactly as a fresh one at that state,
    and later updates work."""
    d = angles_dict(3.0, 0.3, np.deg2rad(50), 0.3, 1.0, 1.0)
    em = ss.SunskyEmitter(d, "spectral")
    n = 1 << 12
    wi, _ = _inputs(n, 7)
    lam = torch.full((4, n), 610.0, device="cuda")
    si = ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)
    params = em.traverse()
    params["turbidity"] = 5.0
    params.update()
    assert em.info()["turbidity"] == 5.0           # read back: this state is accepted
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):                    # batch work queued on a caller stream
        em.eval(si)
    _inject(em, 1 if second == "accepted" else 2)
    params = em.traverse()
    params["turbidity"] = 6.0
    params.update()                                # rejected
    params["albedo"] = 0.45                        # (traverse() would read the state back)
    params.update()                                # accepted or rejected
    with pytest.raises(ValueError, match="non-negative"):
        em.info()
    assert em.get_param("turbidity") == 5.0 and np.allclose(em.get_param("albedo"), 0.3, rtol=0, atol=1e-7)
    fresh = ss.SunskyEmitter(dict(d, turbidity=5.0), "spectral")
    assert torch.equal(em.eval(si), fresh.eval(si))
    np.testing.assert_array_equal(em.table("spectral_pdf"), fresh.table("spectral_pdf"))
    assert em.info()["turbidity"] == 5.0           # reported once
    params = em.traverse()
    params["turbidity"] = 7.0
    params.update()
    assert torch.equal(em.eval(si), ss.SunskyEmitter(dict(d, turbidity=7.0), "spectral").eval(si))
