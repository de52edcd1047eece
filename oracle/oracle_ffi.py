"""ctypes wrapper of the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The oracle is the CPU restatement of the reference hot path (oracle/vr_oracle.c); it is the
checker for the MI355X product path, never part of it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

MODE_REFERENCE = 0
MODE_PRUNED = 1
MATERIAL_LAMBERTIAN = 0
MATERIAL_REFLECTIVE = 1
MATERIAL_PHONG = 2
MATERIAL_DIELECTRIC = 3
PRIM_PLANE = 0
PRIM_SPHERE = 1


class Hit(C.Structure):
    _fields_ = [
        ("valid", C.c_int32), ("object", C.c_int32), ("primitive", C.c_int64), ("material", C.c_int32),
        ("pad", C.c_int32), ("distance", C.c_double), ("location", C.c_double * 3), ("normal", C.c_double * 3),
        ("tangent", C.c_double * 3), ("cotangent", C.c_double * 3), ("retro", C.c_double * 3),
    ]


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("box_tests", "triangle_tests", "rays", "samples", "closest_hits", "errors")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


SAMPLE_RECORD_DTYPE = np.dtype([("wavelength", "<f8"), ("intensity", "<f8"), ("xyz", "<f8", (3,)),
                                ("bounces", "<i4"), ("flags", "<i4")])

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        d, p, u64, i64, i32, u32 = C.c_double, C.c_void_p, C.c_uint64, C.c_int64, C.c_int32, C.c_uint32
        sig = {
            "orc_mix64": (u64, [u64]),
            "orc_hash32": (C.c_uint32, [C.c_uint32]),
            "orc_stream_base": (u64, [u64, u64, u64]),
            "orc_stream_draw": (u64, [u64, u64]),
            "orc_u64_to_standard": (d, [u64]),
            "orc_u64_to_open01": (d, [u64]),
            "orc_normalize": (None, [p, p]),
            "orc_bbox_intersect": (C.c_int, [p, p, p, p]),
            "orc_triangle_intersect": (None, [p, p, p, p, p]),
            "orc_sphere_intersect": (None, [p, d, p, p, p]),
            "orc_plane_new": (None, [p, p, p, p]),
            "orc_plane_intersect": (None, [p, p, p, d, p, p, p]),
            "orc_mat3_inverse": (C.c_int, [p, p]),
            "orc_mat3_determinant": (d, [p]),
            "orc_mat3_first_minor": (d, [p, i32, i32]),
            "orc_mat3_cofactor_matrix": (None, [p, p]),
            "orc_mat3_transpose": (None, [p, p]),
            "orc_mat3_mul": (None, [p, p, p]),
            "orc_mat3_mul_vec": (None, [p, p, p]),
            "orc_change_of_basis": (None, [p, p, p, p]),
            "orc_interval_new": (None, [d, d, p]),
            "orc_interval_union": (None, [p, p, p]),
            "orc_interval_intersection": (None, [p, p, p]),
            "orc_interval_expand": (None, [p, d, p]),
            "orc_interval_is_empty": (C.c_int, [p]),
            "orc_interval_is_degenerate": (C.c_int, [p]),
            "orc_interval_contains": (C.c_int, [p, d]),
            "orc_bbox_from_corners": (None, [p, p, p]),
            "orc_bbox_from_points": (None, [i64, p, p]),
            "orc_bbox_union": (None, [p, p, p]),
            "orc_bbox_contains_point": (C.c_int, [p, p]),
            "orc_bbox_largest_dimension": (C.c_int, [p]),
            "orc_ray_new": (None, [p, p, p, p]),
            "orc_ray_point_at": (None, [p, p, d, p]),
            "orc_spectrum_intensity": (d, [d, d, i32, p, d]),
            "orc_reflection_from_linear_rgb": (None, [d, d, d, p]),
            "orc_colour_xyz_for_wavelength": (None, [d, p]),
            "orc_colour_xyz_to_linear_rgb": (None, [p, p]),
            "orc_colour_xyz_from_linear_rgb": (None, [p, p]),
            "orc_sky_intensity": (d, [p, d]),
            "orc_tone_map": (None, [p, u64, p]),
            "orc_scene_set_whitted": (C.c_int, [p, d, d, i32, p, i32, p, p, p, p, p]),
            "orc_ray_for_pixel": (None, [p, u64, u64, u64, u64, d, d, p, p]),
            "orc_update_pixel": (None, [p, p, p, p, p, d, d, d]),
            "orc_merge_tile": (None, [u64, p, p, u64, u64, u64, u64, p, p]),
            "orc_scene_new": (p, [p]),
            "orc_scene_free": (None, [p]),
            "orc_scene_add_material": (C.c_int, [p, i32, d, d, i32, p, d, d, d]),
            "orc_scene_add_primitive_list": (C.c_int, [p, i32, p, p, p, p]),
            "orc_scene_add_mesh": (C.c_int, [p, i64, p, p, i32]),
            "orc_scene_mesh_leaf_order": (C.c_int, [p, i32, p]),
            "orc_scene_mesh_depth": (C.c_int, [p, i32]),
            "orc_trace": (C.c_int, [p, i64, p, p, i32, p, p]),
            "orc_render_tile": (C.c_int, [p, u64, u64, u64, u64, u64, u64, u32, u64, u64, i32, i32, i32,
                                          p, p, p, p, p, p]),
            "orc_render_samples": (C.c_int, [p, u64, u64, u64, u64, u64, u64, u32, u64, u64, i32, i32, p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def f64(x, n=None):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if n is not None:
        assert a.size == n, (a.shape, n)
    return a


# ---------------------------------------------------------------- low level
def hit_to_dict(h):
    if not h.valid:
        return None
    return {"distance": h.distance, "location": np.array(h.location[:]), "normal": np.array(h.normal[:]),
            "tangent": np.array(h.tangent[:]), "cotangent": np.array(h.cotangent[:]), "retro": np.array(h.retro[:]),
            "object": h.object, "primitive": h.primitive, "material": h.material}


def normalize(v):
    out = np.zeros(3)
    lib().orc_normalize(_ptr(f64(v, 3)), _ptr(out))
    return out


def bbox_intersect(corner1, corner2, origin, direction):
    return bool(lib().orc_bbox_intersect(_ptr(f64(corner1, 3)), _ptr(f64(corner2, 3)), _ptr(f64(origin, 3)),
                                         _ptr(f64(direction, 3))))


def triangle_intersect(vertices, normals, origin, direction):
    h = Hit()
    lib().orc_triangle_intersect(_ptr(f64(vertices, 9)), _ptr(f64(normals, 9)), _ptr(f64(origin, 3)),
                                 _ptr(f64(direction, 3)), C.byref(h))
    return hit_to_dict(h)


def sphere_intersect(centre, radius, origin, direction):
    h = Hit()
    lib().orc_sphere_intersect(_ptr(f64(centre, 3)), radius, _ptr(f64(origin, 3)), _ptr(f64(direction, 3)),
                               C.byref(h))
    return hit_to_dict(h)


def plane_new(normal):
    n, t, c = np.zeros(3), np.zeros(3), np.zeros(3)
    lib().orc_plane_new(_ptr(f64(normal, 3)), _ptr(n), _ptr(t), _ptr(c))
    return n, t, c


def plane_intersect(normal, distance, origin, direction):
    n, t, c = plane_new(normal)
    h = Hit()
    lib().orc_plane_intersect(_ptr(n), _ptr(t), _ptr(c), distance, _ptr(f64(origin, 3)), _ptr(f64(direction, 3)),
                              C.byref(h))
    return hit_to_dict(h)


def mat3_inverse(m):
    out = np.zeros(9)
    ok = lib().orc_mat3_inverse(_ptr(f64(m, 9)), _ptr(out))
    return out.reshape(3, 3) if ok else None


def mat3_determinant(m):
    return lib().orc_mat3_determinant(_ptr(f64(m, 9)))


def mat3_first_minor(m, row, column):
    return lib().orc_mat3_first_minor(_ptr(f64(m, 9)), row, column)


def _mat_out(fn, *args):
    out = np.zeros(9)
    fn(*[_ptr(a) for a in args], _ptr(out))
    return out.reshape(3, 3)


def mat3_cofactor_matrix(m):
    return _mat_out(lib().orc_mat3_cofactor_matrix, f64(m, 9))


def mat3_transpose(m):
    return _mat_out(lib().orc_mat3_transpose, f64(m, 9))


def mat3_mul(a, b):
    return _mat_out(lib().orc_mat3_mul, f64(a, 9), f64(b, 9))


def mat3_mul_vec(m, v):
    out = np.zeros(3)
    lib().orc_mat3_mul_vec(_ptr(f64(m, 9)), _ptr(f64(v, 3)), _ptr(out))
    return out


def change_of_basis(x, y, z):
    return _mat_out(lib().orc_change_of_basis, f64(x, 3), f64(y, 3), f64(z, 3))


# Interval {min, max} (util/interval.rs) and util BoundingBox {min x, max x, ..., max z}
def interval_new(a, b):
    out = np.zeros(2)
    lib().orc_interval_new(a, b, _ptr(out))
    return out


def interval_union(a, b):
    out = np.zeros(2)
    lib().orc_interval_union(_ptr(f64(a, 2)), _ptr(f64(b, 2)), _ptr(out))
    return out


def interval_intersection(a, b):
    out = np.zeros(2)
    lib().orc_interval_intersection(_ptr(f64(a, 2)), _ptr(f64(b, 2)), _ptr(out))
    return out


def interval_expand(a, v):
    out = np.zeros(2)
    lib().orc_interval_expand(_ptr(f64(a, 2)), v, _ptr(out))
    return out


def interval_is_empty(a):
    return bool(lib().orc_interval_is_empty(_ptr(f64(a, 2))))


def interval_is_degenerate(a):
    return bool(lib().orc_interval_is_degenerate(_ptr(f64(a, 2))))


def interval_contains(a, v):
    return bool(lib().orc_interval_contains(_ptr(f64(a, 2)), v))


def bbox_from_corners(a, b):
    out = np.zeros(6)
    lib().orc_bbox_from_corners(_ptr(f64(a, 3)), _ptr(f64(b, 3)), _ptr(out))
    return out


def bbox_from_points(points):
    p = f64(points).reshape(-1, 3)
    out = np.zeros(6)
    lib().orc_bbox_from_points(len(p), _ptr(p), _ptr(out))
    return out


def bbox_union(a, b):
    out = np.zeros(6)
    lib().orc_bbox_union(_ptr(f64(a, 6)), _ptr(f64(b, 6)), _ptr(out))
    return out


def bbox_contains_point(b, p):
    return bool(lib().orc_bbox_contains_point(_ptr(f64(b, 6)), _ptr(f64(p, 3))))


def bbox_largest_dimension(b):
    return lib().orc_bbox_largest_dimension(_ptr(f64(b, 6)))


def ray_new(origin, direction):
    o, d = np.zeros(3), np.zeros(3)
    lib().orc_ray_new(_ptr(f64(origin, 3)), _ptr(f64(direction, 3)), _ptr(o), _ptr(d))
    return o, d


def ray_point_at(origin, direction, t):
    out = np.zeros(3)
    lib().orc_ray_point_at(_ptr(f64(origin, 3)), _ptr(f64(direction, 3)), t, _ptr(out))
    return out


def spectrum_intensity(shortest, longest, samples, wavelength):
    s = f64(samples)
    return lib().orc_spectrum_intensity(shortest, longest, s.size, _ptr(s), wavelength)


def reflection_from_linear_rgb(r, g, b):
    out = np.zeros(32)
    lib().orc_reflection_from_linear_rgb(r, g, b, _ptr(out))
    return out


def xyz_for_wavelength(wl):
    out = np.zeros(3)
    lib().orc_colour_xyz_for_wavelength(wl, _ptr(out))
    return out


def xyz_to_linear_rgb(xyz):
    out = np.zeros(3)
    lib().orc_colour_xyz_to_linear_rgb(_ptr(f64(xyz, 3)), _ptr(out))
    return out


def tone_map(colour):
    """ClampingToneMapper over a colour buffer [..., 3] (XYZ) -> uint8 [..., 3]."""
    c = np.ascontiguousarray(colour, dtype=np.float64)
    out = np.zeros(c.shape, dtype=np.uint8)
    lib().orc_tone_map(_ptr(c), c.size // 3, _ptr(out))
    return out


def xyz_from_linear_rgb(rgb):
    out = np.zeros(3)
    lib().orc_colour_xyz_from_linear_rgb(_ptr(f64(rgb, 3)), _ptr(out))
    return out


def sky_intensity(w, wl):
    return lib().orc_sky_intensity(_ptr(f64(w, 3)), wl)


def ray_for_pixel(camera, width, height, row, column, ux, uy):
    o, d = np.zeros(3), np.zeros(3)
    lib().orc_ray_for_pixel(_ptr(f64(camera, 3)), width, height, row, column, ux, uy, _ptr(o), _ptr(d))
    return o, d


# ---------------------------------------------------------------- scene
class OracleScene:
    """Mirror of reference `Scene` built from a vanrijn_amd.scenes.SceneSpec (plain data)."""

    def __init__(self, spec):
        L = lib()
        self.spec = spec
        self.handle = C.c_void_p(L.orc_scene_new(_ptr(f64(spec.camera_location, 3))))
        for m in spec.materials:
            s = f64(m.colour.samples)
            r = L.orc_scene_add_material(self.handle, m.kind, m.colour.shortest_wavelength,
                                         m.colour.longest_wavelength, s.size, _ptr(s), m.diffuse_strength,
                                         m.reflection_strength, getattr(m, "smoothness", 0.0))
            assert r >= 0
        ig = getattr(spec, "integrator", None)
        if ig is not None:  # WhittedIntegrator
            amb = f64(ig.ambient_light.samples)
            n = len(ig.lights)
            dirs = f64([li.direction for li in ig.lights] or [[0.0, 0.0, 0.0]]).reshape(-1)
            sh = f64([li.spectrum.shortest_wavelength for li in ig.lights] or [0.0])
            lo = f64([li.spectrum.longest_wavelength for li in ig.lights] or [0.0])
            cnt = np.array([len(li.spectrum.samples) for li in ig.lights] or [1], dtype=np.int32)
            samp = np.zeros((max(n, 1), 64))
            for j, li in enumerate(ig.lights):
                samp[j, :len(li.spectrum.samples)] = li.spectrum.samples
            assert L.orc_scene_set_whitted(self.handle, ig.ambient_light.shortest_wavelength,
                                           ig.ambient_light.longest_wavelength, amb.size, _ptr(amb), n, _ptr(dirs),
                                           _ptr(sh), _ptr(lo), cnt.ctypes.data_as(C.c_void_p), _ptr(samp)) == 0
        for obj in spec.objects:
            if obj.kind == "primitives":
                kinds = np.array([p.kind for p in obj.primitives], dtype=np.int32)
                mats = np.array([p.material for p in obj.primitives], dtype=np.int32)
                vecs = f64([p.vector for p in obj.primitives]).reshape(-1)
                sc = f64([p.scalar for p in obj.primitives])
                L.orc_scene_add_primitive_list(self.handle, len(kinds), _ptr(kinds), _ptr(mats), _ptr(vecs), _ptr(sc))
            else:
                mesh = spec.meshes[obj.mesh]
                v = f64(mesh.vertices).reshape(-1)
                n = f64(mesh.normals).reshape(-1)
                L.orc_scene_add_mesh(self.handle, v.size // 9, _ptr(v), _ptr(n), mesh.material)

    def __del__(self):
        if getattr(self, "handle", None):
            lib().orc_scene_free(self.handle)
            self.handle = None

    def leaf_order(self, object_index):
        mesh = self.spec.meshes[self.spec.objects[object_index].mesh]
        out = np.zeros(len(mesh.vertices), dtype=np.int64)
        assert lib().orc_scene_mesh_leaf_order(self.handle, object_index, _ptr(out)) == 0
        return out

    def depth(self, object_index):
        return lib().orc_scene_mesh_depth(self.handle, object_index)

    def trace(self, origins, directions, mode=MODE_REFERENCE):
        o = f64(origins).reshape(-1, 3)
        d = f64(directions).reshape(-1, 3)
        hits = (Hit * len(o))()
        cnt = Counters()
        lib().orc_trace(self.handle, len(o), _ptr(o), _ptr(d), mode, hits, C.byref(cnt))
        return list(hits), cnt.as_dict()

    def render_tile(self, tile, height, width, spp, seed, first_sample=0, mode=MODE_REFERENCE, nthreads=1,
                    accumulate=None):
        """Returns dict of tile arrays (colour/colour_sum/colour_bias [h,w,3], weight/weight_bias [h,w])."""
        th, tw = tile.end_row - tile.start_row, tile.end_column - tile.start_column
        if accumulate is None:
            buf = {"colour": np.zeros((th, tw, 3)), "colour_sum": np.zeros((th, tw, 3)),
                   "colour_bias": np.zeros((th, tw, 3)), "weight": np.zeros((th, tw)),
                   "weight_bias": np.zeros((th, tw))}
            acc = 0
        else:
            buf, acc = accumulate, 1
        cnt = Counters()
        rc = lib().orc_render_tile(self.handle, tile.start_column, tile.end_column, tile.start_row, tile.end_row,
                                   height, width, spp, seed, first_sample, mode, nthreads, acc,
                                   _ptr(buf["colour"]), _ptr(buf["colour_sum"]), _ptr(buf["colour_bias"]),
                                   _ptr(buf["weight"]), _ptr(buf["weight_bias"]), C.byref(cnt))
        if rc < 0:
            raise ValueError("oracle render_tile rejected its arguments")
        buf["counters"] = cnt.as_dict()
        return buf

    def render_samples(self, tile, height, width, spp, seed, first_sample=0, mode=MODE_REFERENCE, nthreads=1):
        th, tw = tile.end_row - tile.start_row, tile.end_column - tile.start_column
        out = np.zeros(th * tw * spp, dtype=SAMPLE_RECORD_DTYPE)
        rc = lib().orc_render_samples(self.handle, tile.start_column, tile.end_column, tile.start_row, tile.end_row,
                                      height, width, spp, seed, first_sample, mode, nthreads, _ptr(out))
        if rc < 0:
            raise ValueError("oracle render_samples rejected its arguments")
        return out.reshape(th, tw, spp)
