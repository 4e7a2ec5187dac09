import sys, os, numpy as np, torch
sys.path.insert(0, 'mitsuba3-sunsky_amd'); sys.path.insert(0, 'oracle'); sys.path.insert(0, '.')
import bench, oracle as O, sunsky_amd as ss
torch.cuda.set_device(0)
for t in (2.0,):
    d = bench.sun_dict(t)
    em = ss.SunskyEmitter(d, "rgb")
    o32 = O.Oracle(d, "rgb", "jit", "f32")
    o64 = bench.oracle64(O, d, "rgb", "jit", o32); o64t = bench.oracle64(O, d, "rgb", "jit", o32, em)
    inf = o32.info()
    cone = -bench.sun_cone_dirs(inf["sun_dir_local"], inf["cos_cutoff"], 1 << 14, seed=int(t))
    g = em.eval(ss.SurfaceInteraction3f(wi=torch.from_numpy(cone.T.copy()).cuda())).T.cpu().numpy().astype(np.float64)
    a, b, c = o32.eval(cone), o64.eval(cone), o64t.eval(cone)
    sun = (-cone @ inf["sun_dir_local"] >= inf["cos_cutoff"]) & (cone[:, 2] <= 0)
    rel = (np.abs(g - c) / np.abs(c)).max(1)
    rel32 = (np.abs(a - b) / np.abs(b)).max(1)
    wo = -cone.astype(np.float64)
    gam = np.arccos(np.clip(wo @ inf["sun_dir_local"], -1, 1)); ha = np.arccos(inf["cos_cutoff"])
    idx = np.argsort(-np.where(sun & (rel32 < 1e-3), rel, 0))[:12]
    for i in idx:
        print(i, f"rel_vs_o64t {rel[i]:.2e} o32err {rel32[i]:.2e} gamma/ha {gam[i]/ha:.9f}", g[i], c[i], a[i])
    print("sun lanes", sun.sum(), "dot32 in", (np.float32(wo.astype(np.float32) @ inf['sun_dir_local'].astype(np.float32)) >= np.float32(inf['cos_cutoff'])).sum())
