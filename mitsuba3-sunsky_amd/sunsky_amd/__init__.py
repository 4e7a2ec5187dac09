"""sunsky_amd -- MI355X-native sun/sky emitter (drop-in for the `sunsky`
plugin of matttsss/mitsuba3-sunsky).  See DESIGN.md / INTEGRATION.md."""
from ._capi import lib, declared_functions, LIB_PATH, CODE_OBJECT, CODE_OBJECT_IDENT  # noqa: F401
from .emitter import (SunskyEmitter, Parameters, load_dict, array_from_file, array_to_file,  # noqa: F401
                      default_dataset_path, hosek_sun_rad)
from .records import (SurfaceInteraction3f, Interaction3f, DirectionSample3f, Ray3f,  # noqa: F401
                      ScalarBoundingBox3f)

__all__ = ["SunskyEmitter", "Parameters", "load_dict", "array_from_file", "array_to_file",
           "default_dataset_path", "hosek_sun_rad", "SurfaceInteraction3f", "Interaction3f", "DirectionSample3f", "Ray3f",
           "ScalarBoundingBox3f", "lib", "declared_functions"]
