"""Diagnostic: error of the GPU eval vs the fp32 / fp64 oracle, by lane class."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "mitsuba3-sunsky_amd")]
import oracle as O
import sunsky_amd as ss
from helpers import angles_dict, hemisphere_wo, sun_cone_wo, sphere_wo

torch.cuda.set_device(0)
for prec in ["fast", "reference"]:
    for turb in [1.0, 2.0, 6.0, 10.0]:
        d = angles_dict(turb, 0.7, np.deg2rad(45), 0.1, 1.0, 1.0)
        em = ss.SunskyEmitter(d, "rgb", precision=prec)
        o32, o64 = O.Oracle(d, "rgb", "jit", "f32"), O.Oracle(d, "rgb", "jit", "f64")
        inf = o32.info()
        wo = np.concatenate([hemisphere_wo(1 << 16, seed=3),
                             sun_cone_wo(4096, inf["sun_dir_local"], np.arccos(inf["cos_cutoff"]), seed=4, scale=1.3),
                             sphere_wo(4096, seed=5)])
        wi = -wo
        t = torch.from_numpy(np.ascontiguousarray(wi.T.astype(np.float32))).cuda()
        out = em.eval(ss.SurfaceInteraction3f(wi=t)); torch.cuda.synchronize()
        g = out.cpu().numpy().T.astype(np.float64)
        a, b = o32.eval(wi).astype(np.float64), o64.eval(wi)
        s = inf["sun_dir_local"]
        sun = (wo @ s >= inf["cos_cutoff"]) & (wo[:, 2] >= 0)
        sky = ~sun
        fl = 1e-6 * np.abs(b).max()
        rg32 = np.abs(g - a) / np.maximum(np.abs(a), fl)
        rg64 = np.abs(g - b) / np.maximum(np.abs(b), fl)
        r3264 = np.abs(a - b) / np.maximum(np.abs(b), fl)
        i = np.unravel_index(np.argmax(np.where(sky[:, None], rg32, 0)), rg32.shape)
        gam = np.degrees(np.arccos(np.clip(wo @ s, -1, 1)))
        print(f"{prec:9s} T={turb:4.1f} sky: gpu-o32 max {rg32[sky].max():.2e} mean {rg32[sky].mean():.2e} | "
              f"gpu-o64 max {rg64[sky].max():.2e} mean {rg64[sky].mean():.2e} | o32-o64 max {r3264[sky].max():.2e} "
              f"mean {r3264[sky].mean():.2e} | worst lane gamma {gam[i[0]]:.3f} deg theta {np.degrees(np.arccos(wo[i[0],2])):.2f} "
              f"o32-o64 there {r3264[i]:.2e}", flush=True)
