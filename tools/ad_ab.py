"""A/B timing of eval_vjp (RGB and spectral 4 lambda, 16M rays) for one code object.

usage: SUNSKY_AMD_CODE_OBJECT=<x.hsaco> python tools/ad_ab.py <label>
Prints one JSON line: the label, the mean launch time of each VJP call (torch events on the
stream the C ABI launches on, 20 timed calls after 5 warm-up calls) and the gradient bits,
so that interleaved runs of several code objects can be compared for speed and equality.
"""
import json
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
res = {"label": sys.argv[1], "code_object": os.environ.get("SUNSKY_AMD_CODE_OBJECT", "default")}
for variant, k in (("rgb", 3), ("spectral", 4)):
    em = ss.load_dict(dict(d), variant=variant)
    lam = 360 + 360 * torch.rand((4, n), device=dev, generator=g) if variant == "spectral" else None
    si = ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)
    cot = 0.5 + torch.rand((k, n), device=dev, generator=g)
    grad = torch.zeros(16, device=dev)
    for _ in range(5):
        grad.zero_()
        em.eval_vjp(si, cot, grad=grad)
    torch.cuda.synchronize()
    bits = grad.cpu().view(torch.int32).tolist()
    s = torch.cuda.current_stream()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(s)
    for _ in range(20):
        em.eval_vjp(si, cot, grad=grad)
    t1.record(s)
    torch.cuda.synchronize()
    res[variant] = {"ms": t0.elapsed_time(t1) / 20, "grad_bits": bits}
print(json.dumps(res), flush=True)
