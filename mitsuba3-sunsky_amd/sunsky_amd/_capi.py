"""ctypes declarations of the C ABI (include/sunsky_amd.h).

The library is the in-tree build (mitsuba3-sunsky_amd/build/libsunsky_amd.so).
There is no fallback: if it (or its gfx950 code object) is missing, every
entry point raises.
"""
import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD_DIR = os.path.join(PKG_ROOT, "build")
LIB_PATH = os.path.join(BUILD_DIR, "libsunsky_amd.so")
CODE_OBJECT = os.path.join(BUILD_DIR, "sunsky_kernels.hsaco")
CODE_OBJECT_IDENT = os.path.join(BUILD_DIR, "sunsky_kernels_ident.hsaco")   # identity to_world
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "sunsky_amd.h")

OK = 0
ERRORS = {1: ValueError, 2: FileNotFoundError, 3: ValueError, 4: RuntimeError, 5: NotImplementedError, 6: RuntimeError,
          7: RuntimeError}

VARIANT_RGB, VARIANT_SPECTRAL = 0, 1
SEMANTICS_JIT, SEMANTICS_SCALAR = 0, 1
PRECISION_FAST, PRECISION_REFERENCE = 0, 1
TABLES = {"sky_params": 0, "sky_radiance": 1, "sun_radiance": 2, "sun_ld": 3, "gaussians": 4,
          "gaussian_cdf": 5, "spectral_pdf": 6, "spectral_cdf": 7, "albedo": 8, "sun_sky_fit": 9,
          "sun_segments": 10}
FLAG_INFINITE, FLAG_SPATIALLY_VARYING = 0x04, 0x10
PARAMS = {"turbidity": 0, "albedo": 1, "sun_direction": 2}   # sunsky_param (differentiable, sunsky.cpp:220-240)
MAX_LAMBDA_PER_RAY = 16   # kMaxLambdaPerRay (csrc/sunsky_types.h)
GRAD_COUNT, GRAD_TURBIDITY, GRAD_ALBEDO, GRAD_SUN_DIRECTION = 16, 0, 1, 12   # eval_vjp gradient layout

c_float_p = C.POINTER(C.c_float)
vp = C.c_void_p


class Vec3In(C.Structure):
    _fields_ = [("x", vp), ("y", vp), ("z", vp)]


class Vec3Out(C.Structure):
    _fields_ = [("x", vp), ("y", vp), ("z", vp)]


class Info(C.Structure):
    _fields_ = [
        ("variant", C.c_int), ("semantics", C.c_int), ("nb_channels", C.c_int), ("active_record", C.c_int),
        ("turbidity", C.c_float), ("sky_scale", C.c_float), ("sun_scale", C.c_float),
        ("sun_half_aperture", C.c_float), ("cos_cutoff", C.c_float), ("area_ratio", C.c_float),
        ("sun_dir_world", C.c_float * 3), ("sun_dir_local", C.c_float * 3), ("sun_angles", C.c_float * 2),
        ("sky_sampling_w", C.c_float), ("bsphere_center", C.c_float * 3), ("bsphere_radius", C.c_float),
        ("flags", C.c_uint), ("device", C.c_int), ("precision", C.c_int),
    ]


_SIGS = {
    "sunsky_abi_version": (C.c_int, []),
    "sunsky_last_error": (C.c_char_p, []),
    "sunsky_props_create": (C.c_int, [C.POINTER(vp)]),
    "sunsky_props_destroy": (None, [vp]),
    "sunsky_props_set_float": (C.c_int, [vp, C.c_char_p, C.c_double]),
    "sunsky_props_set_int": (C.c_int, [vp, C.c_char_p, C.c_int64]),
    "sunsky_props_set_vector3": (C.c_int, [vp, C.c_char_p, C.c_float, C.c_float, C.c_float]),
    "sunsky_props_set_transform": (C.c_int, [vp, C.c_char_p, c_float_p]),
    "sunsky_props_set_spectrum": (C.c_int, [vp, C.c_char_p, c_float_p, C.c_int]),
    "sunsky_props_set_irregular_spectrum": (C.c_int, [vp, C.c_char_p, c_float_p, c_float_p, C.c_int]),
    "sunsky_emitter_create": (C.c_int, [vp, C.c_int, C.c_int, C.c_char_p, C.POINTER(vp)]),
    "sunsky_emitter_create_host": (C.c_int, [vp, C.c_int, C.c_int, C.c_char_p, C.POINTER(vp)]),
    "sunsky_emitter_destroy": (None, [vp]),
    "sunsky_emitter_set_param": (C.c_int, [vp, C.c_char_p, c_float_p, C.c_int]),
    "sunsky_emitter_parameters_changed": (C.c_int, [vp]),
    "sunsky_emitter_parameters_changed_async": (C.c_int, [vp, vp]),
    "sunsky_emitter_inject_staging_fault": (C.c_int, [vp, C.c_int]),
    "sunsky_emitter_sun_segments": (C.c_int, [vp, vp, C.c_size_t, vp, vp]),
    "sunsky_emitter_get_param": (C.c_int, [vp, C.c_char_p, c_float_p, C.c_int, C.POINTER(C.c_int)]),
    "sunsky_emitter_set_scene": (C.c_int, [vp, C.c_int, c_float_p, C.c_float]),
    "sunsky_emitter_set_precision": (C.c_int, [vp, C.c_int]),
    "sunsky_emitter_get_info": (C.c_int, [vp, C.POINTER(Info)]),
    "sunsky_emitter_get_table": (C.c_int, [vp, C.c_int, c_float_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "sunsky_emitter_to_string": (C.c_int, [vp, C.c_char_p, C.c_size_t]),
    "sunsky_emitter_bbox": (C.c_int, [vp, c_float_p, c_float_p]),
    "sunsky_eval": (C.c_int, [vp, Vec3In, vp, C.c_int, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp]),
    "sunsky_eval_direction": (C.c_int, [vp, Vec3In, vp, C.c_int, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp]),
    "sunsky_eval_spectral_broadcast": (C.c_int, [vp, Vec3In, c_float_p, C.c_int, vp, C.c_size_t, vp, C.c_size_t, vp]),
    "sunsky_sample_direction": (C.c_int, [vp, vp, vp, Vec3In, vp, C.c_int, C.c_size_t, vp, C.c_size_t, Vec3Out,
                                          vp, vp, Vec3Out, vp, C.c_size_t, vp]),
    "sunsky_pdf_direction": (C.c_int, [vp, Vec3In, vp, C.c_size_t, vp, vp]),
    "sunsky_sample_ray": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, C.c_size_t, Vec3Out, Vec3Out, vp, C.c_size_t,
                                    vp, C.c_size_t, vp]),
    "sunsky_sample_wavelengths": (C.c_int, [vp, Vec3In, vp, vp, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp]),
    "sunsky_sample_position": (C.c_int, [vp]),
    "sunsky_eval_jvp": (C.c_int, [vp, C.c_int, c_float_p, C.c_int, Vec3In, vp, C.c_int, C.c_size_t, vp, C.c_size_t,
                                  vp, vp, C.c_size_t, vp]),
    "sunsky_bake_latlong": (C.c_int, [vp, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, c_float_p,
                                      C.c_int, vp, C.c_size_t, vp]),
    "sunsky_direct_diffuse": (C.c_int, [vp, Vec3In, vp, vp, C.c_int, C.c_size_t, C.c_uint32, C.c_uint32,
                                        vp, C.c_size_t, C.c_size_t, vp, C.c_size_t, vp]),
    "sunsky_direct_diffuse_rays": (C.c_int, [vp, Vec3In, C.c_uint32, C.c_uint32, C.c_size_t, Vec3Out, Vec3Out,
                                             C.c_size_t, vp]),
    "sunsky_direct_conductor": (C.c_int, [vp, Vec3In, Vec3In, C.c_int, C.c_float, c_float_p, c_float_p, vp, C.c_int,
                                          C.c_size_t, C.c_uint32, C.c_uint32, vp, C.c_size_t, C.c_size_t, vp,
                                          C.c_size_t, vp]),
    "sunsky_direct_conductor_rays": (C.c_int, [vp, Vec3In, Vec3In, C.c_int, C.c_float, c_float_p, c_float_p,
                                               C.c_uint32, C.c_uint32, C.c_size_t, Vec3Out, Vec3Out, vp,
                                               C.c_size_t, vp]),
    "sunsky_direct_conductor_aniso": (C.c_int, [vp, Vec3In, Vec3In, C.c_int, C.c_float, C.c_float, c_float_p,
                                                c_float_p, vp, C.c_int, C.c_size_t, C.c_uint32, C.c_uint32, vp,
                                                C.c_size_t, C.c_size_t, vp, C.c_size_t, vp]),
    "sunsky_direct_conductor_rays_aniso": (C.c_int, [vp, Vec3In, Vec3In, C.c_int, C.c_float, C.c_float, c_float_p,
                                                     c_float_p, C.c_uint32, C.c_uint32, C.c_size_t, Vec3Out, Vec3Out,
                                                     vp, C.c_size_t, vp]),
    "sunsky_hosek_sun_rad": (C.c_int, [C.c_char_p, C.c_double, C.c_double, C.c_double, C.c_double,
                                       C.POINTER(C.c_double)]),
    "plugin_name": (C.c_char_p, []),
    "plugin_descr": (C.c_char_p, []),
    "sunsky_eval_vjp": (C.c_int, [vp, Vec3In, vp, C.c_int, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, vp, vp]),
    "sunsky_emitter_tangent_tables": (C.c_int, [vp, C.c_int, c_float_p, C.c_int, C.c_int, c_float_p, C.c_size_t,
                                                C.POINTER(C.c_size_t)]),
    "sunsky_array_from_file": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_double), C.c_size_t,
                                         C.POINTER(C.c_size_t), C.POINTER(C.c_uint64), C.POINTER(C.c_int)]),
    "sunsky_array_to_file": (C.c_int, [C.c_char_p, c_float_p, C.c_size_t, C.POINTER(C.c_uint64), C.c_int]),
    "sunsky_default_dataset_path": (C.c_int, [C.c_char_p, C.c_size_t]),
    "sunsky_comm_get_unique_id": (C.c_int, [C.c_char_p]),
    "sunsky_comm_create": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(vp)]),
    "sunsky_comm_destroy": (None, [vp]),
    "sunsky_comm_info": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "sunsky_gather_radiance": (C.c_int, [vp, C.c_int, vp, C.c_size_t, C.c_int, C.POINTER(C.c_size_t), vp,
                                         C.c_size_t, vp]),
}

_lib = None


def lib():
    """Load the in-tree C-ABI library (torch first, so the process shares one
    HIP runtime: libamdhip64.so.7 is resolved by soname)."""
    global _lib
    if _lib is None:
        try:
            import torch  # noqa: F401  (HIP runtime owner)
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"sunsky_amd native library not built: {LIB_PATH} "
                              "(run __graft_entry__.build() or make -C mitsuba3-sunsky_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != OK:
        msg = lib().sunsky_last_error().decode(errors="replace")
        raise ERRORS.get(rc, RuntimeError)(msg)
    return rc


def declared_functions():
    """Every function prototype declared in include/sunsky_amd.h."""
    import re
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sunsky_[a-z0-9_]+)\s*\(", src)))
