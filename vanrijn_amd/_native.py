"""ctypes binding of the C ABI in include/vanrijn_amd.h (libvanrijn_amd.so, built for gfx950).

There is no CPU fallback: if the in-tree library is missing or fails to load, every entry point
raises.  Structures mirror the header field for field.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# VR_LIBRARY: an alternative build for A/B timing (tools/ab.sh); the default is the in-tree library
LIB_PATH = os.environ.get("VR_LIBRARY") or os.path.join(HERE, "lib", "libvanrijn_amd.so")

VR_OK = 0
STATUS = {
    0: "VR_OK", -1: "VR_ERROR_INVALID_ARGUMENT", -2: "VR_ERROR_OUT_OF_MEMORY", -3: "VR_ERROR_DEVICE",
    -4: "VR_ERROR_NO_DEVICE", -5: "VR_ERROR_SINGULAR_BASIS", -6: "VR_ERROR_IO", -7: "VR_ERROR_UNSUPPORTED",
    -8: "VR_ERROR_HOST_ONLY",
}
MATERIAL_LAMBERTIAN, MATERIAL_REFLECTIVE, MATERIAL_PHONG, MATERIAL_DIELECTRIC = 0, 1, 2, 3
PRIMITIVE_PLANE, PRIMITIVE_SPHERE = 0, 1
OBJECT_PRIMITIVE_LIST, OBJECT_BVH = 0, 1
SCENE_HOST_ONLY = 1
SCENE_DEVICE_BVH = 2
SCENE_REFERENCE_BVH = 4
SCENE_DEVICE_SAH = 8
SCENE_GREEDY_COLLAPSE = 16
SCENE_WIDE_OFFSETS = 32
LAUNCH_TIMED, LAUNCH_COUNTERS, LAUNCH_DEFER_TIMES, LAUNCH_NO_CULL = 1, 2, 4, 8
LAUNCH_NO_DIST_CULL, LAUNCH_NO_COOP, LAUNCH_NO_LONE_WALK, LAUNCH_STACK32 = 16, 32, 64, 128
VARIANT_COOP, VARIANT_WIDE_OFFSETS, VARIANT_STACK16 = 1, 2, 4
SCENE_INFO_NAN_FREE = 1


class VrError(RuntimeError):
    def __init__(self, code, message):
        super().__init__(f"{STATUS.get(code, code)}: {message}")
        self.code = code


class Vec3(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]


class Spectrum(C.Structure):
    _fields_ = [("shortest_wavelength", C.c_double), ("longest_wavelength", C.c_double),
                ("sample_count", C.c_uint32), ("samples", C.POINTER(C.c_double))]


class MaterialDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_uint32), ("colour", Spectrum),
                ("diffuse_strength", C.c_double), ("reflection_strength", C.c_double), ("smoothness", C.c_double)]


class PrimitiveDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_uint32), ("vector", Vec3), ("scalar", C.c_double)]


class MeshDesc(C.Structure):
    _fields_ = [("triangle_count", C.c_uint64), ("vertices", C.POINTER(C.c_double)),
                ("normals", C.POINTER(C.c_double)), ("material", C.c_uint32), ("reserved", C.c_uint32)]


class ObjectDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("first", C.c_uint32), ("count", C.c_uint32), ("reserved", C.c_uint32)]


class DirectionalLightC(C.Structure):
    _fields_ = [("direction", Vec3), ("spectrum", Spectrum)]


class IntegratorDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("light_count", C.c_uint32), ("ambient_light", Spectrum),
                ("lights", C.POINTER(DirectionalLightC))]


INTEGRATOR_SIMPLE_RANDOM, INTEGRATOR_WHITTED = 0, 1


class SceneDesc(C.Structure):
    _fields_ = [("camera_location", Vec3), ("material_count", C.c_uint32), ("primitive_count", C.c_uint32),
                ("mesh_count", C.c_uint32), ("object_count", C.c_uint32),
                ("materials", C.POINTER(MaterialDesc)), ("primitives", C.POINTER(PrimitiveDesc)),
                ("meshes", C.POINTER(MeshDesc)), ("objects", C.POINTER(ObjectDesc)),
                ("integrator", C.POINTER(IntegratorDesc))]


class SceneInfo(C.Structure):
    _fields_ = [("triangle_count", C.c_uint64), ("node_count", C.c_uint64), ("max_bvh_depth", C.c_uint32),
                ("object_count", C.c_uint32), ("extent", C.c_double), ("device_bytes", C.c_uint64),
                ("wide_node_count", C.c_uint64), ("traversal_stack", C.c_uint32), ("flags", C.c_uint32)]


class TileC(C.Structure):
    _fields_ = [("start_column", C.c_uint64), ("end_column", C.c_uint64), ("start_row", C.c_uint64),
                ("end_row", C.c_uint64)]


class AccumulationBufferC(C.Structure):
    _fields_ = [("width", C.c_uint64), ("height", C.c_uint64), ("colour", C.c_void_p),
                ("colour_sum", C.c_void_p), ("colour_bias", C.c_void_p), ("weight", C.c_void_p),
                ("weight_bias", C.c_void_p)]


class RenderParams(C.Structure):
    _fields_ = [("tile", TileC), ("height", C.c_uint64), ("width", C.c_uint64), ("spp", C.c_uint32),
                ("accumulate", C.c_uint32), ("seed", C.c_uint64), ("first_sample", C.c_uint64)]


class LaunchStats(C.Structure):
    _fields_ = [("kernel_ms", C.c_float), ("timed", C.c_uint32), ("box_tests", C.c_uint64),
                ("node_visits", C.c_uint64), ("triangle_tests", C.c_uint64), ("rays", C.c_uint64),
                ("shaded_triangle_hits", C.c_uint64), ("samples", C.c_uint64), ("traversal_slots", C.c_uint64),
                ("path_loop_slots", C.c_uint64), ("exact_box_tests", C.c_uint64), ("reduce_ms", C.c_float),
                ("passes", C.c_uint32), ("variant", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "reserved"}


class LaunchTimes(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("reduce_ms", C.c_double), ("launches", C.c_uint32),
                ("passes", C.c_uint32), ("max_passes", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_ if n != "reserved"}


class SampleRecord(C.Structure):
    _fields_ = [("wavelength", C.c_double), ("intensity", C.c_double), ("xyz", C.c_double * 3),
                ("bounces", C.c_int32), ("flags", C.c_int32)]


class HitRecord(C.Structure):
    _fields_ = [("valid", C.c_int32), ("object", C.c_int32), ("primitive", C.c_int64), ("distance", C.c_double),
                ("location", C.c_double * 3), ("normal", C.c_double * 3), ("tangent", C.c_double * 3),
                ("cotangent", C.c_double * 3), ("retro", C.c_double * 3)]


# every function declared in include/vanrijn_amd.h: name -> (restype, argtypes)
_p, _u32, _u64, _i32, _d = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32, C.c_double
SIGNATURES = {
    "vr_scene_create": (C.c_int, [C.POINTER(SceneDesc), _i32, _u32, C.POINTER(C.c_void_p)]),
    "vr_scene_destroy": (None, [_p]),
    "vr_scene_get_info": (C.c_int, [_p, C.POINTER(SceneInfo)]),
    "vr_scene_bvh_leaf_order": (C.c_int, [_p, _u32, _p]),
    "vr_scene_bvh_nodes": (C.c_int, [_p, _p]),
    "vr_partial_render_scene": (C.c_int, [_p, TileC, _u64, _u64, C.POINTER(AccumulationBufferC)]),
    "vr_render_tile": (C.c_int, [_p, C.POINTER(RenderParams), C.POINTER(AccumulationBufferC)]),
    "vr_render_tile_device": (C.c_int, [_p, C.POINTER(RenderParams), _p, _p, _u32, C.POINTER(LaunchStats)]),
    "vr_stream_check_error": (C.c_int, [_p, _p]),
    "vr_collect_launch_times": (C.c_int, [_p, _p, C.POINTER(LaunchTimes)]),
    "vr_resolve_state": (C.c_int, [_p, _u64, _p]),
    "vr_merge_tile": (C.c_int, [C.POINTER(AccumulationBufferC), TileC, C.POINTER(AccumulationBufferC)]),
    "vr_render_samples": (C.c_int, [_p, C.POINTER(RenderParams), _p]),
    "vr_trace_rays": (C.c_int, [_p, _u64, _p, _p, _p]),
    "vr_spectrum_reflection_from_linear_rgb": (C.c_int, [_d, _d, _d, _p]),
    "vr_spectrum_intensity_at_wavelength": (_d, [C.POINTER(Spectrum), _d]),
    "vr_colour_xyz_for_wavelength": (None, [_d, _p]),
    "vr_load_obj": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint64), C.POINTER(C.POINTER(C.c_double)),
                              C.POINTER(C.POINTER(C.c_double))]),
    "vr_mesh_free": (None, [C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "vr_tone_map_device": (C.c_int, [_p, _u64, _p, _i32, _p]),
    "vr_tone_map": (C.c_int, [_p, _u64, _p, _i32]),
    "vr_write_png": (C.c_int, [C.c_char_p, _p, _u32, _u32]),
    "vr_scene_set_staging_limit": (C.c_int, [_p, _u64]),
    "vr_debug_set_fault_object": (C.c_int, [_p, _i32]),
    "vr_debug_set_launch_flags": (C.c_int, [_p, _u32]),
    "vr_scene_needs_wide_offsets": (C.c_int, [_u64, _u64]),
    "vr_device_count": (C.c_int, []),
    "vr_last_error": (C.c_char_p, []),
    "vr_abi_version": (C.c_uint32, []),
}

_lib = None


def lib():
    """Load the in-tree HIP library; raise loudly if it is not there (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -m vanrijn_amd.build` (hipcc, gfx950) first")
        # torch's HIP runtime first: the library's libamdhip64 dependency then resolves to the one
        # already loaded (same soname), so the library and torch share one runtime.  Loaded the
        # other way round, torch would find the system runtime in place of its own and see no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                # an older build under A/B (tools/ab.sh, VR_LIBRARY) may predate a symbol; the
                # in-tree library must export every one (tests/test_abi.py)
                if os.environ.get("VR_LIBRARY"):
                    continue
                raise
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != VR_OK:
        raise VrError(rc, lib().vr_last_error().decode(errors="replace"))
    return rc
