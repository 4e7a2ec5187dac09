"""AD kernel timing helper (run under rocprofv3 --kernel-trace --stats): eval_vjp and
eval_jvp over 16M upper-hemisphere directions, RGB and spectral (4 lambda per ray)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mitsuba3-sunsky_amd"))
import sunsky_amd as ss  # noqa: E402

n = 1 << 24
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
v = torch.randn((3, n), device=dev, generator=g)
v[2] = v[2].abs()
wi = -(v / v.norm(dim=0, keepdim=True)).contiguous()
d = {"type": "sunsky", "sun_direction": [0.3, 0.4, 0.866], "turbidity": 3.0, "albedo": 0.2}
for variant, k in (("rgb", 3), ("spectral", 4)):
    em = ss.load_dict(dict(d), variant=variant)
    lam = 360 + 360 * torch.rand((4, n), device=dev, generator=g) if variant == "spectral" else None
    si = ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)
    cot = torch.ones((k, n), device=dev)
    grad = em.eval_vjp(si, cot)[0]
    for _ in range(10):
        em.eval_vjp(si, cot, grad=grad)
    for _ in range(10):
        em.eval_jvp(si, "turbidity", [1.0])
    torch.cuda.synchronize()
print("ad_bench done")
