"""traverse() / parameters_changed() semantics on the host: a rejected
update restores the last committed values (the reference validates in
parameters_changed, sunsky.cpp:242-285, and the scene keeps its previous state), and
traverse() reads the emitter's current values back through the C ABI."""
import numpy as np
import pytest

import sunsky_amd as ss
from helpers import angles_dict, hour_dict


def test_rejected_update_rolls_back():
    em = ss.SunskyEmitter(angles_dict(3.0, 0.2, np.deg2rad(50), 0.3, 1.0, 1.0), "rgb", device="host")
    w0 = em.sky_sampling_w
    tab0 = em.table("sky_params")
    p = em.traverse()
    p["turbidity"] = 12.0
    p["sky_scale"] = 2.0
    with pytest.raises(ValueError, match="out of range"):
        p.update()
    assert em.get_param("turbidity") == 3.0 and em.get_param("sky_scale") == 1.0
    assert p["turbidity"] == 3.0 and p["sky_scale"] == 1.0
    assert em.info()["turbidity"] == 3.0 and em.sky_sampling_w == w0
    assert np.array_equal(em.table("sky_params"), tab0)
    # a valid update after the rejected one starts from the committed state
    p["sun_scale"] = 0.5
    p.update()
    assert em.get_param("sun_scale") == 0.5 and em.get_param("turbidity") == 3.0
    assert np.array_equal(em.table("sky_params"), tab0)


def test_rejected_albedo_update_rolls_back():
    em = ss.SunskyEmitter(angles_dict(4.0, 0.2, np.deg2rad(40), 0.3, 1.0, 1.0), "spectral", device="host")
    p = em.traverse()
    p["albedo"] = np.full(11, 1.5, np.float32)
    with pytest.raises(ValueError, match="Albedo"):
        p.update()
    assert np.allclose(em.get_param("albedo"), 0.3)


def test_traverse_reads_current_time_location():
    em = ss.SunskyEmitter(hour_dict(3.0, 10.0, 0.2, 1.0, 1.0), "rgb", device="host")
    p = em.traverse()
    assert p["hour"] == 10.0 and p["year"] == 2010 and p["latitude"] == pytest.approx(35.6894)
    sun0 = em.info()["sun_dir_world"].copy()
    p["hour"] = 14.5
    p["latitude"] = 10.0
    p.update()
    q = em.traverse()
    assert q["hour"] == 14.5 and q["latitude"] == pytest.approx(10.0)
    assert not np.allclose(em.info()["sun_dir_world"], sun0)


def test_traverse_to_world_and_sun_direction():
    M = np.array([[0, 0, 1, 0], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1]], np.float32)
    d = dict(angles_dict(3.0, 0.2, np.deg2rad(50), 0.3, 1.0, 1.0), to_world=M)
    em = ss.SunskyEmitter(d, "rgb", device="host")
    p = em.traverse()
    assert np.array_equal(p["to_world"], M)
    assert np.allclose(p["sun_direction"], d["sun_direction"], atol=1e-6)
    with pytest.raises(KeyError):
        p["hour"] = 3.0
