"""Timing of the entry points bench.py does not report (sample_ray, sample_wavelengths,
eval_direction, the general sample_direction with it.p), 64M items, HIP events over bursts.
Developer tool: python tools/entry_bench.py > gpurun_out/entry_bench.json"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mitsuba3-sunsky_amd"))
import sunsky_amd as ss  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = 1 << 26
    th = np.deg2rad(60.0)
    d = {"type": "sunsky", "turbidity": 3.0, "albedo": 0.3, "sun_direction": [float(np.sin(th)), 0.0, float(np.cos(th))]}
    g = torch.Generator(device="cuda").manual_seed(5)
    out = {}
    for variant in ("rgb", "spectral"):
        em = ss.SunskyEmitter(d, variant)
        u2 = torch.rand((2, n), generator=g, device="cuda")
        u3 = torch.rand((2, n), generator=g, device="cuda")
        wl = torch.rand(n, generator=g, device="cuda")
        out[f"sample_ray_{variant}_ms"] = timed(lambda: em.sample_ray(None, wl, u2, u3))
        wi = -torch.nn.functional.normalize(torch.randn((3, n), generator=g, device="cuda"), dim=0)
        si = ss.SurfaceInteraction3f(wi=wi)
        out[f"sample_wavelengths_{variant}_ms"] = timed(lambda: em.sample_wavelengths(si, wl))
        p = torch.randn((3, n), generator=g, device="cuda")
        lam = (360.0 + 360.0 * torch.rand((4, n), generator=g, device="cuda")) if variant == "spectral" else None
        it = ss.Interaction3f(p=p, wavelengths=lam)
        out[f"sample_direction_general_{variant}_ms"] = timed(lambda: em.sample_direction(it, u2))
        del u2, u3, wl, wi, si, p, lam, it
        torch.cuda.empty_cache()
    out["items"] = n
    print(json.dumps(out))


if __name__ == "__main__":
    main()
