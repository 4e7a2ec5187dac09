"""Argument checks of the Python face: malformed batch inputs raise
ValueError before any pointer reaches the C ABI, so a wrong shape can never become an
out-of-bounds device access.  Runs on CPU: a host-only emitter (staging, no kernels)
goes through the same validation as a GPU one."""
import numpy as np
import pytest
import torch

import sunsky_amd as ss


@pytest.fixture(scope="module")
def rgb():
    return ss.SunskyEmitter({"turbidity": 3.0}, "rgb", device="host")


@pytest.fixture(scope="module")
def spec():
    return ss.SunskyEmitter({"turbidity": 3.0}, "spectral", device="host")


def wi(n):
    return torch.zeros((3, n))


def test_vectors_must_be_soa(rgb):
    with pytest.raises(ValueError, match=r"\(3, n\)"):
        rgb.eval(ss.SurfaceInteraction3f(wi=torch.zeros((8, 3))))


def test_mask_length(rgb):
    with pytest.raises(ValueError, match="active mask"):
        rgb.eval(ss.SurfaceInteraction3f(wi=wi(8)), active=torch.ones(7, dtype=torch.bool))
    with pytest.raises(ValueError, match="active mask"):
        rgb.pdf_direction(ss.Interaction3f(), ss.DirectionSample3f(d=wi(8)), active=torch.ones((2, 8)))


@pytest.mark.parametrize("shape", [(4, 1), (4, 7), (17, 8), (8,)[:0] + (9,)])
def test_wavelength_planes(spec, shape):
    with pytest.raises(ValueError, match="wavelengths"):
        spec.eval(ss.SurfaceInteraction3f(wi=wi(8), wavelengths=torch.full(shape, 500.0)))


def test_spectral_needs_wavelengths(spec):
    with pytest.raises(ValueError):
        spec.eval(ss.SurfaceInteraction3f(wi=wi(8)))


def test_sample_direction_inputs(rgb):
    with pytest.raises(ValueError, match=r"\(2, n\)"):
        rgb.sample_direction(ss.Interaction3f(), torch.zeros((3, 8)))
    with pytest.raises(ValueError, match="it.p"):
        rgb.sample_direction(ss.Interaction3f(p=wi(7)), torch.zeros((2, 8)))


def test_sample_ray_inputs(spec):
    with pytest.raises(ValueError, match="sample3"):
        spec.sample_ray(None, torch.zeros(8), torch.zeros((2, 8)), torch.zeros((2, 9)))
    with pytest.raises(ValueError, match="wavelength_sample"):
        spec.sample_ray(None, torch.zeros(5), torch.zeros((2, 8)), torch.zeros((2, 8)))
    with pytest.raises(ValueError, match="wavelength sample"):
        spec.sample_ray(None, None, torch.zeros((2, 8)), torch.zeros((2, 8)))


def test_sample_wavelengths_inputs(spec):
    with pytest.raises(ValueError, match="sample"):
        spec.sample_wavelengths(ss.SurfaceInteraction3f(wi=wi(8)), torch.zeros(3))


def test_eval_vjp_gradient_buffer(rgb):
    si = ss.SurfaceInteraction3f(wi=wi(8))
    with pytest.raises(ValueError, match="d_out"):
        rgb.eval_vjp(si, torch.zeros((3, 7)))
    for bad in (torch.zeros(12), torch.zeros(16, dtype=torch.float64), torch.zeros(32)[::2]):
        with pytest.raises(ValueError, match="grad"):
            rgb.eval_vjp(si, torch.zeros((3, 8)), grad=bad)


def test_outputs_checked(rgb, spec):
    with pytest.raises(ValueError, match="out"):
        rgb.bake_latlong(16, 8, out=torch.zeros((3, 8, 15)))
    with pytest.raises(ValueError, match="out"):
        spec.eval_spectral_broadcast(wi(8), [400.0, 500.0], out=torch.zeros((2, 7)))
    with pytest.raises(ValueError, match="reflectance"):
        rgb.direct_diffuse(wi(8), reflectance=torch.zeros(4))


def test_numpy_inputs_are_accepted_up_to_the_launch(rgb):
    """Well-formed inputs pass validation; the host-only emitter then refuses to launch."""
    with pytest.raises(Exception) as e:
        rgb.eval(ss.SurfaceInteraction3f(wi=np.zeros((3, 8), np.float32)))
    assert not isinstance(e.value, ValueError) or "host-only" in str(e.value)
