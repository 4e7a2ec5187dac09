"""Child process of tests/test_profiler_ranges.py (run under rocprofv3 --marker-trace):
one call of each batch entry point family on cuda:0."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-sunsky_amd"))

import torch  # noqa: E402

import sunsky_amd as ss  # noqa: E402

torch.cuda.set_device(0)
em = ss.SunskyEmitter({"type": "sunsky", "turbidity": 3.0, "albedo": 0.2}, "rgb")
n = 4096
u = torch.rand((2, n), device="cuda")
wi = -torch.nn.functional.normalize(torch.rand((3, n), device="cuda") + 0.1, dim=0)
em.eval(ss.SurfaceInteraction3f(wi=wi))
ds, w = em.sample_direction(ss.Interaction3f(), u)
em.pdf_direction(ss.Interaction3f(), ds)
em.eval_direction(ss.Interaction3f(), ds)
em.direct_diffuse(-wi, 1, 2)
torch.cuda.synchronize()
print("worker ok")
