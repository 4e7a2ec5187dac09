"""params.update() latency on the GPU: host time of the stream-ordered C-ABI call, the
Python update() around it, and the device time of one staging (events around a single
update on an idle stream).  Compares with the host-only staging (host C++/OpenMP).
Run under rocprofv3 --kernel-trace --stats for the staging kernels' own durations."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mitsuba3-sunsky_amd"))
import sunsky_amd as ss  # noqa: E402


def main():
    d = {"type": "sunsky", "turbidity": 3.0, "albedo": 0.3, "sun_direction": [0.5, 0.1, 0.86]}
    res = {}
    L = ss.lib()
    for variant in ("rgb", "spectral"):
        em = ss.SunskyEmitter(d, variant)
        stream = torch.cuda.current_stream().cuda_stream
        torch.cuda.synchronize()
        reps = 200
        # raw C ABI: set_param + parameters_changed_async
        t0 = time.perf_counter()
        for k in range(reps):
            v = (C.c_float * 1)(3.0 + 0.001 * k)
            L.sunsky_emitter_set_param(em._h, b"turbidity", v, 1)
            L.sunsky_emitter_parameters_changed_async(em._h, C.c_void_p(stream))
        capi_us = (time.perf_counter() - t0) / reps * 1e6
        torch.cuda.synchronize()
        # Python Parameters.update()
        p = em.traverse()
        t0 = time.perf_counter()
        for k in range(reps):
            p["turbidity"] = 3.0 + 0.001 * k
            p.update()
        py_us = (time.perf_counter() - t0) / reps * 1e6
        torch.cuda.synchronize()
        # device time of one staging on an idle stream
        dev = []
        for k in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            v = (C.c_float * 1)(4.0 + 0.01 * k)
            L.sunsky_emitter_set_param(em._h, b"turbidity", v, 1)
            L.sunsky_emitter_parameters_changed_async(em._h, C.c_void_p(stream))
            e1.record()
            torch.cuda.synchronize()
            dev.append(e0.elapsed_time(e1) * 1e3)
        # blocking form (+ read back of w_sky etc.)
        t0 = time.perf_counter()
        for k in range(20):
            v = (C.c_float * 1)(5.0 + 0.01 * k)
            L.sunsky_emitter_set_param(em._h, b"turbidity", v, 1)
            L.sunsky_emitter_parameters_changed(em._h)
        block_us = (time.perf_counter() - t0) / 20 * 1e6
        hs = ss.SunskyEmitter(d, variant, device="host")
        t0 = time.perf_counter()
        for k in range(10):
            v = (C.c_float * 1)(3.0 + 0.01 * k)
            L.sunsky_emitter_set_param(hs._h, b"turbidity", v, 1)
            L.sunsky_emitter_parameters_changed(hs._h)
        host_us = (time.perf_counter() - t0) / 10 * 1e6
        res[variant] = {"capi_async_host_us": capi_us, "python_update_host_us": py_us,
                        "device_staging_us_median": float(np.median(dev)), "blocking_call_us": block_us,
                        "host_only_staging_us": host_us, "host_threads": int(os.environ.get("OMP_NUM_THREADS", "0"))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
