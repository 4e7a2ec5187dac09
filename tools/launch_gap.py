"""Where do bench.py's inter-kernel gaps come from?  Times the headline launch
pattern several ways (HIP events on the launch stream)."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mitsuba3-sunsky_amd")]
import sunsky_amd as ss
from bench import sun_dict, hemisphere_dirs

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
n = 1 << 24
wi = -hemisphere_dirs(n, 1234, dev)
ems = [ss.SunskyEmitter(sun_dict(t), "rgb", device=dev) for t in (2.0, 6.0, 10.0)]
outs = [torch.empty((3, n), device=dev) for _ in ems]
lib = ss.lib()
vin = ss._capi.Vec3In(wi[0].data_ptr(), wi[1].data_ptr(), wi[2].data_ptr())
stream = torch.cuda.current_stream(dev).cuda_stream


def call(em, out):
    rc = lib.sunsky_eval(em._h, vin, None, 0, 0, None, n, out.data_ptr(), n, stream)
    assert rc == 0


def timed(fn, launches, reps=3):
    best = 1e9
    for _ in range(reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        e0.record()
        fn()
        e1.record()
        h1 = time.perf_counter()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / launches)
    return best * 1e3, (h1 - h0) / launches * 1e6


print("one emitter x60      : %.2f us/launch (host %.2f us/launch)" % timed(lambda: [call(ems[0], outs[0]) for _ in range(60)], 60))
print("three emitters x20   : %.2f us/launch (host %.2f us/launch)" % timed(lambda: [call(e, o) for _ in range(20) for e, o in zip(ems, outs)], 60))
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    stream = s.cuda_stream
    call(ems[0], outs[0])
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for e, o in zip(ems, outs):
            call(e, o)
torch.cuda.synchronize()
print("graph of 3, x20      : %.2f us/launch (host %.2f us/launch)" % timed(lambda: [g.replay() for _ in range(20)], 60))
