"""Python face of the MI355X sun/sky emitter: the method names, arguments and
errors of the reference `sunsky` plugin (src/emitters/sunsky.cpp) as exposed to
Python by mitsuba (src/render/python/emitter_v.cpp:102-137), over the C ABI.

Every batch method takes and returns torch tensors on the emitter's GPU in SoA
layout ((3, n) vectors, (k, n) spectra) and runs on the current torch stream.
"""
import ctypes as C
import math

import numpy as np
import torch

from . import _capi
from ._capi import PARAMS, Vec3In, Vec3Out, check, lib
from .records import DirectionSample3f, Ray3f, ScalarBoundingBox3f

_FLOAT_KEYS = ("turbidity", "sky_scale", "sun_scale", "sun_aperture", "latitude", "longitude",
               "timezone", "hour", "minute", "second")
_INT_KEYS = ("year", "month", "day")
_VARIANTS = {"rgb": _capi.VARIANT_RGB, "spectral": _capi.VARIANT_SPECTRAL}
_SEMANTICS = {"jit": _capi.SEMANTICS_JIT, "scalar": _capi.SEMANTICS_SCALAR}
_PRECISION = {"fast": _capi.PRECISION_FAST, "reference": _capi.PRECISION_REFERENCE}


def _alpha_uv(alpha):
    """roughconductor's alpha: a float (isotropic) or (alpha_u, alpha_v) -> two floats."""
    if np.ndim(alpha) == 0:
        return float(alpha), float(alpha)
    a = [float(x) for x in alpha]
    if len(a) != 2:
        raise ValueError("alpha must be a float or (alpha_u, alpha_v)")
    return a[0], a[1]


def _fa(values):
    arr = (C.c_float * len(values))(*[float(v) for v in values])
    return arr


def _build_props(d):
    L = lib()
    h = C.c_void_p()
    check(L.sunsky_props_create(C.byref(h)))
    try:
        for key, val in d.items():
            if key in ("type", "id"):
                continue
            k = key.encode()
            if key == "sun_direction":
                v = [float(x) for x in np.asarray(val, dtype=np.float64).reshape(-1)]
                if len(v) != 3:
                    raise ValueError("sun_direction needs 3 components")
                check(L.sunsky_props_set_vector3(h, k, *v))
            elif key == "to_world":
                m = np.asarray(val, dtype=np.float32).reshape(-1)
                if m.size != 16:
                    raise ValueError("to_world needs a 4x4 matrix")
                check(L.sunsky_props_set_transform(h, k, _fa(m)))
            elif key == "albedo" and isinstance(val, dict):
                t = val.get("type")
                if t == "irregular":
                    wl = [float(x) for x in str(val["wavelengths"]).split(",")]
                    vs = [float(x) for x in str(val["values"]).split(",")]
                    if len(wl) != len(vs):
                        raise ValueError("irregular spectrum: wavelengths/values length mismatch")
                    check(L.sunsky_props_set_irregular_spectrum(h, k, _fa(wl), _fa(vs), len(wl)))
                elif t in ("rgb", "spectrum", "regular") and "value" in val:
                    vs = np.atleast_1d(np.asarray(val["value"], dtype=np.float32)).tolist()
                    check(L.sunsky_props_set_spectrum(h, k, _fa(vs), len(vs)))
                elif t == "uniform":
                    check(L.sunsky_props_set_float(h, k, float(val["value"])))
                else:
                    raise ValueError(f"unsupported albedo texture {val!r}")
            elif key == "albedo" and np.ndim(val) > 0:
                vs = np.asarray(val, dtype=np.float32).reshape(-1).tolist()
                check(L.sunsky_props_set_spectrum(h, k, _fa(vs), len(vs)))
            elif isinstance(val, (bool, np.bool_)):
                raise ValueError(f"property '{key}' cannot be a boolean")
            elif isinstance(val, (int, np.integer)) and key not in _FLOAT_KEYS:
                check(L.sunsky_props_set_int(h, k, int(val)))
            elif isinstance(val, (int, float, np.integer, np.floating)):
                if key in _INT_KEYS and float(val) == int(val):
                    check(L.sunsky_props_set_int(h, k, int(val)))
                else:
                    check(L.sunsky_props_set_float(h, k, float(val)))
            else:
                raise ValueError(f"unsupported value for property '{key}': {val!r}")
    except Exception:
        L.sunsky_props_destroy(h)
        raise
    return h


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p()


class Parameters(dict):
    """mi.traverse() result: assign, then update() -> parameters_changed()."""

    def __init__(self, emitter, values):
        super().__init__(values)
        self._emitter = emitter
        self._dirty = set()

    def __setitem__(self, key, value):
        if key not in self:
            raise KeyError(f"unknown parameter '{key}'")
        super().__setitem__(key, value)
        self._dirty.add(key)

    def update(self, *args, **kw):
        if args or kw:
            for k, v in dict(*args, **kw).items():
                self[k] = v
        em = self._emitter
        try:
            for key in sorted(self._dirty):
                v = np.atleast_1d(np.asarray(self[key], dtype=np.float32)).reshape(-1)
                check(lib().sunsky_emitter_set_param(em._h, key.encode(), _fa(v.tolist()), v.size))
            if em.device is None:
                check(lib().sunsky_emitter_parameters_changed(em._h))
            else:
                # stream-ordered on the current torch stream: evals queued after this see the
                # new state; nothing waits for the device (sunsky_emitter_parameters_changed_async)
                with torch.cuda.device(em.device):
                    check(lib().sunsky_emitter_parameters_changed_async(em._h, em._stream()))
        except Exception:
            # a rejected update leaves the emitter at its last committed values: show them
            for key in self._dirty:
                super().__setitem__(key, em.get_param(key))
            raise
        finally:
            self._dirty.clear()
            em._info = None   # read back lazily (info(), sky_sampling_w, ...)


class SunskyEmitter:
    """The `sunsky` emitter (sunsky.cpp:152-1037) on one MI355X.

    variant   -- "rgb" | "spectral" (Mitsuba *_rgb / *_spectral variants)
    semantics -- "jit" (llvm_/cuda_ variants: quadrature sampling weight) |
                 "scalar" (scalar_ variants: weight 0.5, uniform wavelengths)
    precision -- "fast" (host-folded transcendental constants) | "reference"
    device    -- torch device for the tables, or "host" (staging only)
    """

    def __init__(self, props, variant="rgb", semantics="jit", dataset_path=None, precision="fast", device=None):
        if props.get("type", "sunsky") != "sunsky":
            raise ValueError(f"unsupported plugin type {props.get('type')!r}")
        self.variant, self.semantics = variant, semantics
        self.is_spectral = variant == "spectral"
        self._props = dict(props)
        self._h = None
        self._info = None
        host = device == "host"
        self.device = None if host else torch.device(device if device is not None else "cuda")
        if not host and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        ph = _build_props(props)
        h = C.c_void_p()
        try:
            ds = dataset_path.encode() if dataset_path else None
            if host:
                check(lib().sunsky_emitter_create_host(ph, _VARIANTS[variant], _SEMANTICS[semantics], ds, C.byref(h)))
            else:
                with torch.cuda.device(self.device):
                    check(lib().sunsky_emitter_create(ph, _VARIANTS[variant], _SEMANTICS[semantics], ds, C.byref(h)))
        finally:
            lib().sunsky_props_destroy(ph)
        self._h = h
        if precision != "fast":
            self.set_precision(precision)
        self._refresh_info()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            try:
                lib().sunsky_emitter_destroy(h)
            except Exception:   # interpreter shutdown: the library may already be gone
                pass

    # ------------------------------------------------------------ state
    def _refresh_info(self):
        inf = _capi.Info()
        check(lib().sunsky_emitter_get_info(self._h, C.byref(inf)))
        self._info = inf

    @property
    def _inf(self):
        """The emitter's info, read back (once per state) after a stream-ordered update."""
        if self._info is None:
            self._refresh_info()
        return self._info

    def get_param(self, name):
        """Current value of a traverse() parameter (sunsky_emitter_get_param)."""
        buf = (C.c_float * 16)()
        cnt = C.c_int()
        check(lib().sunsky_emitter_get_param(self._h, name.encode(), buf, 16, C.byref(cnt)))
        vals = np.frombuffer(buf, dtype=np.float32, count=cnt.value).copy()
        if name == "to_world":
            return vals.reshape(4, 4)
        if name in ("year", "month", "day"):
            return int(vals[0])
        return float(vals[0]) if cnt.value == 1 and name != "albedo" else vals

    def set_precision(self, precision):
        check(lib().sunsky_emitter_set_precision(self._h, _PRECISION[precision]))
        self._refresh_info()

    def info(self):
        i = self._inf
        return {
            "variant": i.variant, "semantics": i.semantics, "nb_channels": i.nb_channels,
            "active_record": bool(i.active_record), "turbidity": i.turbidity, "sky_scale": i.sky_scale,
            "sun_scale": i.sun_scale, "sun_half_aperture": i.sun_half_aperture, "cos_cutoff": i.cos_cutoff,
            "area_ratio": i.area_ratio, "sun_dir_world": np.array(i.sun_dir_world),
            "sun_dir_local": np.array(i.sun_dir_local), "sun_angles": np.array(i.sun_angles),
            "w_sky": i.sky_sampling_w, "bsphere_center": np.array(i.bsphere_center),
            "bsphere_radius": i.bsphere_radius, "flags": i.flags, "device": i.device,
            "precision": "fast" if i.precision == _capi.PRECISION_FAST else "reference",
        }

    def table(self, name):
        cnt = C.c_size_t()
        tid = _capi.TABLES[name]
        check(lib().sunsky_emitter_get_table(self._h, tid, None, 0, C.byref(cnt)))
        buf = (C.c_float * max(cnt.value, 1))()
        check(lib().sunsky_emitter_get_table(self._h, tid, buf, cnt.value, C.byref(cnt)))
        return np.frombuffer(buf, dtype=np.float32, count=cnt.value).copy()

    @property
    def flags(self):
        return self._inf.flags

    @property
    def sky_sampling_w(self):
        return self._inf.sky_sampling_w

    def bbox(self):
        mn, mx = (C.c_float * 3)(), (C.c_float * 3)()
        check(lib().sunsky_emitter_bbox(self._h, mn, mx))
        return ScalarBoundingBox3f(tuple(mn), tuple(mx))

    def set_scene(self, bbox_min=None, bbox_max=None):
        """set_scene(scene) with the scene's bounding box (sunsky.cpp:287-301)."""
        if bbox_min is None or bbox_max is None or any(a > b for a, b in zip(bbox_min, bbox_max)):
            check(lib().sunsky_emitter_set_scene(self._h, 0, None, 0.0))
        else:
            mn, mx = np.asarray(bbox_min, np.float64), np.asarray(bbox_max, np.float64)
            c = (mn + mx) / 2
            r = float(np.linalg.norm(mx - c))   # BoundingBox::bounding_sphere
            check(lib().sunsky_emitter_set_scene(self._h, 1, _fa(c.tolist()), r))
        self._refresh_info()

    def traverse(self):
        """Parameters exposed by traverse() (sunsky.cpp:220-240), read back from the emitter."""
        keys = ["turbidity", "sky_scale", "sun_scale", "albedo"]
        if self.info()["active_record"]:
            keys += ["latitude", "longitude", "timezone", "year", "day", "month", "hour", "minute", "second"]
        else:
            keys += ["sun_direction"]
        keys += ["to_world"]
        return Parameters(self, {k: self.get_param(k) for k in keys})

    def __repr__(self):
        buf = C.create_string_buffer(4096)
        check(lib().sunsky_emitter_to_string(self._h, buf, 4096))
        return buf.value.decode()

    # ------------------------------------------------------------ helpers
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _f32(self, t, rows=None):
        if t is None:
            return None
        t = torch.as_tensor(t, dtype=torch.float32, device=self.device)
        if rows is not None and t.dim() == 1 and rows == 1:
            t = t.unsqueeze(0)
        return t.contiguous()

    def _plane(self, t, n, name):
        """One fp32 plane of n values on the emitter's device (a 0-d value is broadcast)."""
        t = self._f32(t)
        if t.dim() == 0:
            t = t.expand(n).contiguous()
        if t.dim() != 1 or t.shape[0] != n:
            raise ValueError(f"{name} must have {n} values (one per lane), got shape {tuple(t.shape)}")
        return t

    def _planes(self, t, rows, n, name):
        """A (rows, n) SoA fp32 tensor on the emitter's device."""
        t = self._f32(t)
        if t.dim() != 2 or t.shape[0] != rows or t.shape[1] != n:
            raise ValueError(f"{name} must be a ({rows}, {n}) tensor, got shape {tuple(t.shape)}")
        return t

    def _out(self, out, shape, row_stride_ok=False):
        """Caller-provided output: float32 on the emitter's device, the given shape, planes
        contiguous (rows may be strided when row_stride_ok)."""
        if out is None:
            return torch.empty(shape, dtype=torch.float32, device=self.device)
        if (not isinstance(out, torch.Tensor) or out.dtype != torch.float32 or out.device != self.device
                or tuple(out.shape) != tuple(shape)):
            raise ValueError(f"out must be a float32 tensor of shape {tuple(shape)} on {self.device}")
        if not (out.is_contiguous() or (row_stride_ok and out.stride(-1) == 1 and out.stride(0) >= shape[-1])):
            raise ValueError("out planes must be contiguous")
        return out

    def _mask(self, active, n):
        if active is None or active is True:
            return None
        a = torch.as_tensor(active, device=self.device)
        if a.dim() == 0:
            a = a.expand(n)
        if a.dim() != 1 or a.shape[0] != n:
            raise ValueError(f"active mask must have {n} entries, got shape {tuple(a.shape)}")
        return a.to(torch.uint8).contiguous()

    def _vec_in(self, v, n=None, name="vectors"):
        v = self._f32(v)
        if v.dim() != 2 or v.shape[0] != 3:
            raise ValueError(f"{name} are SoA tensors of shape (3, n)")
        if n is not None and v.shape[1] != n:
            raise ValueError(f"{name} must have {n} lanes, got {v.shape[1]}")
        return v, Vec3In(v[0].data_ptr(), v[1].data_ptr(), v[2].data_ptr())

    def _wavelengths(self, wl, n):
        """Per-lane wavelengths as a (k, n) plane set, 1 <= k <= 16 (Spectrum<Float, k>); a scalar
        or a single value is broadcast to every lane."""
        if wl is None:
            raise ValueError("spectral variants need wavelengths")
        wl = torch.as_tensor(wl, dtype=torch.float32, device=self.device)
        if wl.dim() == 0 or (wl.dim() == 1 and wl.numel() == 1):
            wl = wl.reshape(1, 1).expand(1, n)
        elif wl.dim() == 1:
            if wl.shape[0] != n:
                raise ValueError(f"wavelengths: {wl.shape[0]} values for {n} lanes")
            wl = wl.view(1, n)
        elif wl.dim() != 2 or wl.shape[1] != n:
            raise ValueError(f"wavelengths must be (k, {n}), got shape {tuple(wl.shape)}")
        if not 1 <= wl.shape[0] <= _capi.MAX_LAMBDA_PER_RAY:
            raise ValueError(f"1..{_capi.MAX_LAMBDA_PER_RAY} wavelengths per lane, got {wl.shape[0]}")
        return wl.contiguous()

    # ------------------------------------------------------------ hot path
    def eval(self, si, active=None):
        """eval(si, active) -- sunsky.cpp:303-352.  RGB -> (3, n); spectral -> (k, n)."""
        return self._eval(si.wi, si.wavelengths, active, lib().sunsky_eval)

    def eval_direction(self, it, ds, active=None):
        """eval_direction(it, ds, active) -- sunsky.cpp:453-461 (wi = -ds.d)."""
        wl = getattr(it, "wavelengths", None)
        return self._eval(ds.d, wl, active, lib().sunsky_eval_direction)

    def _eval(self, wi, wavelengths, active, fn):
        wi, vin = self._vec_in(wi)
        n = wi.shape[1]
        m = self._mask(active, n)
        if self.is_spectral:
            if wavelengths is None:
                raise ValueError("spectral eval needs si.wavelengths")
            wl = self._wavelengths(wavelengths, n)
            k = wl.shape[0]
            out = torch.empty((k, n), dtype=torch.float32, device=self.device)
            check(fn(self._h, vin, _ptr(wl), k, n, _ptr(m), n, _ptr(out), n, self._stream()))
        else:
            out = torch.empty((3, n), dtype=torch.float32, device=self.device)
            check(fn(self._h, vin, None, 0, 0, _ptr(m), n, _ptr(out), n, self._stream()))
        return out

    def eval_jvp(self, si, param, tangent, active=None):
        """Forward-mode derivative of eval(si) along `tangent` of a differentiable
        parameter ("turbidity", "albedo", "sun_direction"; sunsky.cpp:220-240) -- the
        reference's dr.forward_from(param) / dr.grad(eval(si)).  -> (value, d_value)."""
        wi, vin = self._vec_in(si.wi)
        n = wi.shape[1]
        m = self._mask(active, n)
        tan = [float(x) for x in np.atleast_1d(np.asarray(tangent, dtype=np.float32))]
        if param not in PARAMS:
            raise ValueError(f"'{param}' is not a differentiable parameter ({', '.join(PARAMS)})")
        wl, k = None, 3
        if self.is_spectral:
            wl = self._wavelengths(getattr(si, "wavelengths", None), n)
            k = wl.shape[0]
        out = torch.empty((k, n), dtype=torch.float32, device=self.device)
        dout = torch.empty((k, n), dtype=torch.float32, device=self.device)
        check(lib().sunsky_eval_jvp(self._h, PARAMS[param], _fa(tan), len(tan), vin, _ptr(wl),
                                    k if self.is_spectral else 0, n, _ptr(m), n, _ptr(out), _ptr(dout), n,
                                    self._stream()))
        return out, dout

    def tangent_tables(self, param, tangent, on_device=True):
        """The tangent of the staged tables along `tangent` of `param` (sunsky.h:158-231,
        404-419): {"dsky": (nch, 10) d{A..I, rad}, "dsun_local": (3,), "dsun": sun table},
        staged by the device kernel eval_jvp uses, or on the host."""
        tan = [float(x) for x in np.atleast_1d(np.asarray(tangent, dtype=np.float32))]
        if param not in PARAMS:
            raise ValueError(f"'{param}' is not a differentiable parameter ({', '.join(PARAMS)})")
        buf = (C.c_float * (128 + 3240))()
        cnt = C.c_size_t()
        check(lib().sunsky_emitter_tangent_tables(self._h, PARAMS[param], _fa(tan), len(tan), int(on_device), buf,
                                                  len(buf), C.byref(cnt)))
        v = np.frombuffer(buf, dtype=np.float32, count=cnt.value).copy()
        nch = self.info()["nb_channels"]
        block = 3240 if nch == 3 else 1980
        return {"dsky": v[: nch * 10].reshape(nch, 10), "dsun_local": v[110:113], "dsun": v[128:128 + block]}

    def eval_vjp(self, si, d_out, active=None, grad=None):
        """Reverse mode: accumulate sum(d_out * d eval(si) / d param) into `grad` (a (16,)
        device tensor; zeros if None) and return it together with a dict view
        {"turbidity", "albedo" (per channel), "sun_direction" (world, 3)}."""
        wi, vin = self._vec_in(si.wi)
        n = wi.shape[1]
        m = self._mask(active, n)
        wl, k = None, 3
        if self.is_spectral:
            wl = self._wavelengths(getattr(si, "wavelengths", None), n)
            k = wl.shape[0]
        d_out = self._f32(d_out)
        if tuple(d_out.shape) != (k, n):
            raise ValueError(f"d_out must have shape ({k}, {n})")
        if grad is None:
            grad = torch.zeros(_capi.GRAD_COUNT, dtype=torch.float32, device=self.device)
        elif (not isinstance(grad, torch.Tensor) or grad.dtype != torch.float32 or grad.device != self.device
              or not grad.is_contiguous() or grad.numel() < _capi.GRAD_COUNT):
            raise ValueError(f"grad must be a contiguous float32 tensor of >= {_capi.GRAD_COUNT} values on "
                             f"{self.device}")
        check(lib().sunsky_eval_vjp(self._h, vin, _ptr(wl), k if self.is_spectral else 0, n, _ptr(m), n,
                                    _ptr(d_out), n, _ptr(grad), self._stream()))
        nch = 11 if self.is_spectral else 3
        view = {"turbidity": grad[_capi.GRAD_TURBIDITY],
                "albedo": grad[_capi.GRAD_ALBEDO:_capi.GRAD_ALBEDO + nch],
                "sun_direction": grad[_capi.GRAD_SUN_DIRECTION:_capi.GRAD_SUN_DIRECTION + 3]}
        return grad, view

    def bake_latlong(self, width, height, theta=(0.0, math.pi), phi=(0.0, 2 * math.pi), wavelengths=None,
                     out=None):
        """Lat-long environment map of the emitter (sunsky_bake_latlong): (C, height, width),
        pixel (x, y) = eval(wi = -sphdir(linspace(*theta, height)[y], linspace(*phi, width)[x]))
        -- sunsky-testing/sky_data_test.py:58-79 with helpers.py get_spherical_rays."""
        if self.is_spectral:
            if wavelengths is None:
                raise ValueError("a spectral bake needs a wavelength list")
            lam = [float(x) for x in np.atleast_1d(np.asarray(wavelengths, dtype=np.float32))]
            k, lam_p, m = len(lam), _fa(lam), len(lam)
        else:
            k, lam_p, m = 3, None, 0
        out = self._out(out, (k, height, width))
        check(lib().sunsky_bake_latlong(self._h, width, height, float(theta[0]), float(theta[1]), float(phi[0]),
                                        float(phi[1]), lam_p, m, _ptr(out), height * width, self._stream()))
        return out

    def direct_diffuse(self, normals, seed=0, spp=1, wavelengths=None, reflectance=None, out=None,
                       visibility=None):
        """Sun-and-sky light at smooth-diffuse points (sunsky_direct_diffuse): the path
        integrator's emitter sampling + BSDF sampling with MIS at one vertex
        (path.cpp:176-250, diffuse.cpp:100-180), spp PCG32 samples per point.
        normals (3, n); wavelengths (k <= 4, n) for spectral -> (C, n).
        visibility: None (unoccluded) or a (spp, n) uint8 tensor of the caller's tracer
        verdicts on the rays of direct_diffuse_rays (bit 0 shadow ray unoccluded, bit 1
        BSDF ray escaped)."""
        normals, nin = self._vec_in(normals)
        n = normals.shape[1]
        vis = None
        if visibility is not None:
            vis = torch.as_tensor(visibility, device=self.device)
            if vis.dim() != 2 or tuple(vis.shape) != (int(spp), n):
                raise ValueError(f"visibility must be a ({int(spp)}, {n}) tensor, got shape {tuple(vis.shape)}")
            vis = vis.to(torch.uint8).contiguous()
        if self.is_spectral:
            if wavelengths is None:
                raise ValueError("spectral direct lighting needs per-point wavelengths")
            wl = self._wavelengths(wavelengths, n)
            if wl.shape[0] > 4:
                raise ValueError("direct_diffuse takes up to 4 wavelengths per point")
            k, lam_p, lstride = wl.shape[0], _ptr(wl), wl.stride(0)
        else:
            wl, k, lam_p, lstride = None, 3, None, 0
        rho = None
        if reflectance is not None:   # gray albedo per point (include/sunsky_amd.h)
            rho = self._plane(reflectance, n, "reflectance")
        out = self._out(out, (k, n))
        check(lib().sunsky_direct_diffuse(self._h, nin, _ptr(rho), lam_p, k if self.is_spectral else 0, lstride,
                                          int(seed) & 0xFFFFFFFF, int(spp), _ptr(vis), n, n, _ptr(out),
                                          out.stride(0), self._stream()))
        return out

    def direct_diffuse_rays(self, normals, seed=0, spp=1):
        """The shadow rays (emitter samples) and BSDF rays of direct_diffuse's samples for the
        same (normals, seed, spp) (sunsky_direct_diffuse_rays) -> (emitter_dir, bsdf_dir), each
        (3, spp, n) world directions, (0, 0, 0) where no ray is needed."""
        normals, nin = self._vec_in(normals)
        n = normals.shape[1]
        if int(spp) < 1:
            raise ValueError("spp must be >= 1")
        em = torch.empty((3, int(spp), n), dtype=torch.float32, device=self.device)
        bs = torch.empty((3, int(spp), n), dtype=torch.float32, device=self.device)
        check(lib().sunsky_direct_diffuse_rays(
            self._h, nin, int(seed) & 0xFFFFFFFF, int(spp), n,
            Vec3Out(em[0].data_ptr(), em[1].data_ptr(), em[2].data_ptr()),
            Vec3Out(bs[0].data_ptr(), bs[1].data_ptr(), bs[2].data_ptr()), n, self._stream()))
        return em, bs

    def direct_conductor(self, normals, wi, alpha=0.1, distribution="beckmann", eta=0.0, k=1.0, seed=0, spp=1,
                         wavelengths=None, out=None, visibility=None):
        """Sun-and-sky light a rough conductor reflects towards wi (sunsky_direct_conductor): one
        path vertex (path.cpp:176-250) with roughconductor.cpp (Beckmann / GGX, visible normals;
        the reference's defaults: Beckmann, alpha 0.1, eta 0, k 1).  alpha: a float, or
        (alpha_u, alpha_v) for an anisotropic distribution (sunsky_direct_conductor_aniso; alpha_u
        along the first tangent of coordinate_system(normal)).  normals, wi (3, n) world unit
        vectors; eta / k: 1 or 3 per-channel values (spectral: the first, for every
        wavelength) -> (C, n)."""
        normals, nin = self._vec_in(normals)
        wi, win = self._vec_in(wi)
        n = normals.shape[1]
        if wi.shape[1] != n:
            raise ValueError("normals and wi must have the same number of points")
        dist = {"beckmann": 0, "ggx": 1}.get(str(distribution).lower())
        if dist is None:
            raise ValueError(f"invalid distribution '{distribution}', must be 'beckmann' or 'ggx'")
        vis = None
        if visibility is not None:
            vis = torch.as_tensor(visibility, device=self.device)
            if vis.dim() != 2 or tuple(vis.shape) != (int(spp), n):
                raise ValueError(f"visibility must be a ({int(spp)}, {n}) tensor, got shape {tuple(vis.shape)}")
            vis = vis.to(torch.uint8).contiguous()
        if self.is_spectral:
            if wavelengths is None:
                raise ValueError("spectral direct lighting needs per-point wavelengths")
            wl = self._wavelengths(wavelengths, n)
            if wl.shape[0] > 4:
                raise ValueError("direct_conductor takes up to 4 wavelengths per point")
            kk, lam_p, lstride = wl.shape[0], _ptr(wl), wl.stride(0)
        else:
            wl, kk, lam_p, lstride = None, 3, None, 0
        e3 = [float(x) for x in np.broadcast_to(np.asarray(eta, np.float32), (3,))]
        k3 = [float(x) for x in np.broadcast_to(np.asarray(k, np.float32), (3,))]
        out = self._out(out, (kk, n))
        tail = (_fa(e3), _fa(k3), lam_p, kk if self.is_spectral else 0, lstride, int(seed) & 0xFFFFFFFF, int(spp),
                _ptr(vis), n, n, _ptr(out), out.stride(0), self._stream())
        au, av = _alpha_uv(alpha)
        if au == av:
            check(lib().sunsky_direct_conductor(self._h, nin, win, dist, au, *tail))
        else:
            check(lib().sunsky_direct_conductor_aniso(self._h, nin, win, dist, au, av, *tail))
        return out

    def direct_conductor_rays(self, normals, wi, alpha=0.1, distribution="beckmann", seed=0, spp=1, eta=None,
                              k=None):
        """The shadow and BSDF rays of direct_conductor's samples -> (emitter_dir, bsdf_dir), each
        (3, spp, n) world directions, (0, 0, 0) where no ray is needed; alpha as direct_conductor.  With eta and k also the
        BSDF samples' weights F G1 (the throughput of a path continuing along bsdf_dir) ->
        (emitter_dir, bsdf_dir, bsdf_weight), bsdf_weight (3 | 1, spp, n)."""
        normals, nin = self._vec_in(normals)
        wi, win = self._vec_in(wi)
        n = normals.shape[1]
        dist = {"beckmann": 0, "ggx": 1}.get(str(distribution).lower())
        if dist is None:
            raise ValueError(f"invalid distribution '{distribution}', must be 'beckmann' or 'ggx'")
        if int(spp) < 1:
            raise ValueError("spp must be >= 1")
        if (eta is None) != (k is None):
            raise ValueError("the BSDF weights need both eta and k")
        em = torch.empty((3, int(spp), n), dtype=torch.float32, device=self.device)
        bs = torch.empty((3, int(spp), n), dtype=torch.float32, device=self.device)
        bw, e3, k3 = None, None, None
        if eta is not None:
            e3 = _fa([float(x) for x in np.broadcast_to(np.asarray(eta, np.float32), (3,))])
            k3 = _fa([float(x) for x in np.broadcast_to(np.asarray(k, np.float32), (3,))])
            bw = torch.empty((1 if self.is_spectral else 3, int(spp), n), dtype=torch.float32, device=self.device)
        tail = (e3, k3, int(seed) & 0xFFFFFFFF, int(spp), n, Vec3Out(em[0].data_ptr(), em[1].data_ptr(), em[2].data_ptr()),
                Vec3Out(bs[0].data_ptr(), bs[1].data_ptr(), bs[2].data_ptr()), _ptr(bw), n, self._stream())
        au, av = _alpha_uv(alpha)
        if au == av:
            check(lib().sunsky_direct_conductor_rays(self._h, nin, win, dist, au, *tail))
        else:
            check(lib().sunsky_direct_conductor_rays_aniso(self._h, nin, win, dist, au, av, *tail))
        return (em, bs) if bw is None else (em, bs, bw)

    def eval_spectral_broadcast(self, wi, wavelengths, active=None, out=None):
        """Spectral eval of one wavelength list for every direction -> (m, n)."""
        wi, vin = self._vec_in(wi)
        n = wi.shape[1]
        lam = [float(x) for x in np.atleast_1d(np.asarray(wavelengths, dtype=np.float32))]
        out = self._out(out, (len(lam), n), row_stride_ok=True)
        m = self._mask(active, n)
        check(lib().sunsky_eval_spectral_broadcast(self._h, vin, _fa(lam), len(lam), _ptr(m), n,
                                                   _ptr(out), out.stride(0), self._stream()))
        return out

    def sample_direction(self, it, sample, active=None, positions=True):
        """sample_direction(it, sample, active) -- sunsky.cpp:399-441 -> (ds, weight).

        positions=False leaves ds.p and ds.dist unset (None): with no mask and no it.p
        the C ABI then runs the LEAN kernel (d, pdf and weight bitwise the same)."""
        sample = self._f32(sample)
        if sample.dim() != 2 or sample.shape[0] != 2:
            raise ValueError("sample is a (2, n) tensor")
        n = sample.shape[1]
        m = self._mask(active, n)
        p = getattr(it, "p", None) if it is not None else None
        if p is not None:
            p, pin = self._vec_in(p, n, "it.p")
        else:
            pin = Vec3In(None, None, None)
        d = torch.empty((3, n), dtype=torch.float32, device=self.device)
        pdf = torch.empty(n, dtype=torch.float32, device=self.device)
        if positions:
            pos = torch.empty((3, n), dtype=torch.float32, device=self.device)
            dist = torch.empty(n, dtype=torch.float32, device=self.device)
            pout = Vec3Out(pos[0].data_ptr(), pos[1].data_ptr(), pos[2].data_ptr())
        else:
            pos = dist = None
            pout = Vec3Out(None, None, None)
        wl = None
        k = 3
        if self.is_spectral:
            wl = self._wavelengths(getattr(it, "wavelengths", None), n)
            k = wl.shape[0]
        w = torch.empty((k, n), dtype=torch.float32, device=self.device)
        check(lib().sunsky_sample_direction(
            self._h, _ptr(sample[0]), _ptr(sample[1]), pin, _ptr(wl), k if self.is_spectral else 0, n,
            _ptr(m), n, Vec3Out(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr()), _ptr(pdf), _ptr(dist),
            pout, _ptr(w), n, self._stream()))
        ds = DirectionSample3f(p=pos, n=-d, uv=sample, time=getattr(it, "time", None), pdf=pdf, delta=False,
                               d=d, dist=dist, emitter=self)
        return ds, w

    def pdf_direction(self, it, ds, active=None):
        """pdf_direction(it, ds, active) -- sunsky.cpp:443-451 -> (n,)."""
        d, vin = self._vec_in(ds.d)
        n = d.shape[1]
        m = self._mask(active, n)
        out = torch.empty(n, dtype=torch.float32, device=self.device)
        check(lib().sunsky_pdf_direction(self._h, vin, _ptr(m), n, _ptr(out), self._stream()))
        return out

    def sample_ray(self, time, wavelength_sample, sample2, sample3, active=None):
        """sample_ray(time, wavelength_sample, sample2, sample3, active) -- sunsky.cpp:354-397."""
        s2 = self._f32(sample2)
        if s2.dim() != 2 or s2.shape[0] != 2:
            raise ValueError("sample2 is a (2, n) tensor")
        n = s2.shape[1]
        s3 = self._planes(sample3, 2, n, "sample3")
        ws = None
        if self.is_spectral or wavelength_sample is not None:
            if wavelength_sample is None:
                raise ValueError("spectral sample_ray needs a wavelength sample")
            ws = self._plane(wavelength_sample, n, "wavelength_sample")
        m = self._mask(active, n)
        o = torch.empty((3, n), dtype=torch.float32, device=self.device)
        d = torch.empty((3, n), dtype=torch.float32, device=self.device)
        lam = torch.empty((4, n), dtype=torch.float32, device=self.device)
        w = torch.empty((4 if self.is_spectral else 3, n), dtype=torch.float32, device=self.device)
        check(lib().sunsky_sample_ray(
            self._h, _ptr(ws), _ptr(s2[0]), _ptr(s2[1]), _ptr(s3[0]), _ptr(s3[1]), _ptr(m), n,
            Vec3Out(o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr()),
            Vec3Out(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr()), _ptr(lam), n, _ptr(w), n, self._stream()))
        return Ray3f(o=o, d=d, time=time, wavelengths=lam), w

    def sample_wavelengths(self, si, sample, active=None):
        """sample_wavelengths(si, sample, active) -- sunsky.cpp:463-480."""
        wi, vin = self._vec_in(si.wi)
        n = wi.shape[1]
        s = self._plane(sample, n, "sample") if (sample is not None or self.is_spectral) else None
        m = self._mask(active, n)
        lam = torch.empty((4, n), dtype=torch.float32, device=self.device)
        w = torch.empty((4 if self.is_spectral else 3, n), dtype=torch.float32, device=self.device)
        check(lib().sunsky_sample_wavelengths(self._h, vin, _ptr(s), _ptr(m), n, _ptr(lam), n, _ptr(w), n,
                                              self._stream()))
        return lam, w

    def sample_position(self, time=None, sample=None, active=None):
        """sample_position -- NotImplementedError like the scalar reference (sunsky.cpp:483-495)."""
        check(lib().sunsky_sample_position(self._h))


def load_dict(d, variant="rgb", semantics="jit", **kw):
    """mi.load_dict({'type': 'sunsky', ...}) counterpart."""
    if d.get("type") != "sunsky":
        raise ValueError(f"unsupported plugin type {d.get('type')!r} (only 'sunsky')")
    return SunskyEmitter(d, variant=variant, semantics=semantics, **kw)


def array_from_file(path, file_dtype=0):
    """array_from_file_d/_f (sunsky_v.cpp:16-17) -> (float64 ndarray with the file's shape)."""
    cnt = C.c_size_t()
    shape = (C.c_uint64 * 16)()
    nd = C.c_int()
    check(lib().sunsky_array_from_file(str(path).encode(), file_dtype, None, 0, C.byref(cnt), shape, C.byref(nd)))
    buf = (C.c_double * max(cnt.value, 1))()
    check(lib().sunsky_array_from_file(str(path).encode(), file_dtype, buf, cnt.value, C.byref(cnt), shape, C.byref(nd)))
    return np.frombuffer(buf, dtype=np.float64, count=cnt.value).reshape([shape[i] for i in range(nd.value)]).copy()


def array_to_file(path, data, shape=None):
    """array_to_file (sunsky_v.cpp:18)."""
    arr = np.ascontiguousarray(np.asarray(data, dtype=np.float32).reshape(-1))
    sh = list(shape) if shape else [arr.size]
    shp = (C.c_uint64 * len(sh))(*sh)
    check(lib().sunsky_array_to_file(str(path).encode(), arr.ctypes.data_as(C.POINTER(C.c_float)), arr.size, shp,
                                     len(sh)))


def hosek_sun_rad(turbidity, wavelength, elevation, gamma, dataset_path=None):
    """mi.hosek_sun_rad (sunsky_v.cpp:19): Hosek-Wilkie solar radiance, fp64 (ArHosekSkyModel.c:686-784)."""
    out = C.c_double()
    check(lib().sunsky_hosek_sun_rad(dataset_path.encode() if dataset_path else None, float(turbidity),
                                     float(wavelength), float(elevation), float(gamma), C.byref(out)))
    return out.value


def default_dataset_path():
    buf = C.create_string_buffer(4096)
    check(lib().sunsky_default_dataset_path(buf, 4096))
    return buf.value.decode()
