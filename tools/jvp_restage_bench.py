"""JVP / VJP restage latency: a params.update() then eval_jvp / eval_vjp on a
small batch, so every call restages the tangent tables (sunsky_stage_tangent on the device).
Reports the host time of the AD call and the wall time of update + call + synchronize,
median of 200; run under rocprofv3 --kernel-trace --stats for the staging kernel's own time.
usage: python tools/jvp_restage_bench.py [out.json] [package parent dir (default: the repo's)]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..",
                                                                     "mitsuba3-sunsky_amd"))
import sunsky_amd as ss  # noqa: E402

dev = torch.device("cuda", 0)
n = 4096
v = torch.randn((3, n), device=dev)
v[2] = v[2].abs()
wi = -(v / v.norm(dim=0, keepdim=True)).contiguous()
res = {}
for variant, k in (("rgb", 3), ("spectral", 4)):
    em = ss.load_dict({"type": "sunsky", "sun_direction": [0.3, 0.4, 0.866], "turbidity": 3.0, "albedo": 0.2},
                      variant=variant)
    lam = (360 + 360 * torch.rand((4, n), device=dev)) if variant == "spectral" else None
    si = ss.SurfaceInteraction3f(wi=wi, wavelengths=lam)
    cot = torch.ones((k, n), device=dev)
    p = em.traverse()
    for mode in ("jvp", "vjp"):
        host, wall = [], []
        for it in range(220):
            p["turbidity"] = 3.0 + 0.01 * (it % 7)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.update()
            t1 = time.perf_counter()
            if mode == "jvp":
                em.eval_jvp(si, "sun_direction", [0.1, 0.2, 0.3])
            else:
                em.eval_vjp(si, cot)
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            if it >= 20:
                host.append((t2 - t1) * 1e6)
                wall.append((t3 - t0) * 1e6)
        res[f"{variant}_{mode}"] = {"ad_call_host_us": float(np.median(host)), "update_call_sync_us": float(np.median(wall)),
                                    "rays": n}
res["package"] = ss.__file__
print(json.dumps(res, indent=1))
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as fh:
        json.dump(res, fh, indent=1)
