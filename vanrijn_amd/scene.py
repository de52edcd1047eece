"""Host-side mirror of the reference's scene API (names and argument meaning as in vanrijn).

    colour::ColourRgbF / NamedColour      src/colour/colour_rgb.rs:5-105
    colour::Spectrum                      src/colour/spectrum.rs:5-175
    materials::LambertianMaterial         src/materials/lambertian_material.rs:12-25
    materials::ReflectiveMaterial         src/materials/reflective_material.rs:8-13
    raycasting::{Plane, Sphere}           src/raycasting/plane.rs:18-31, sphere.rs:15-23
    raycasting::BoundingVolumeHierarchy   src/raycasting/bounding_volume_hierarchy.rs:49-51
    mesh::load_obj                        src/mesh.rs:74-88
    scene::Scene                          src/scene.rs:5-8

A `Scene` lowers to a plain-data `SceneSpec` (numbers only) which the C ABI consumes
(`vr_scene_create`) -- and which the test oracle consumes too, so both see identical inputs.
"""
from dataclasses import dataclass, field
import atexit
import ctypes as C
from enum import Enum
from typing import List
import weakref

import numpy as np

from . import _native as N

# every DeviceScene not yet released: destroyed at interpreter exit while the library and the HIP
# runtime are still loaded (module teardown order would otherwise decide)
_LIVE = weakref.WeakSet()


@atexit.register
def _release_live_scenes():
    for s in list(_LIVE):
        s.release()

SHORTEST_VISIBLE_WAVELENGTH = 380.0  # src/colour/mod.rs:13
LONGEST_VISIBLE_WAVELENGTH = 740.0   # src/colour/mod.rs:14


# ------------------------------------------------------------------------------ colours / spectra
class NamedColour(Enum):
    Black = (0.0, 0.0, 0.0)
    White = (1.0, 1.0, 1.0)
    Red = (1.0, 0.0, 0.0)
    Lime = (0.0, 1.0, 0.0)
    Blue = (0.0, 0.0, 1.0)
    Yellow = (1.0, 1.0, 0.0)
    Cyan = (0.0, 1.0, 1.0)
    Magenta = (1.0, 0.0, 1.0)
    Gray = (0.5, 0.5, 0.5)
    Maroon = (0.5, 0.0, 0.0)
    Olive = (0.5, 0.5, 0.0)
    Green = (0.0, 0.5, 0.0)
    Purple = (0.5, 0.0, 0.5)
    Teal = (0.0, 0.5, 0.5)
    Navy = (0.0, 0.0, 0.5)


@dataclass(frozen=True)
class ColourRgbF:
    red: float
    green: float
    blue: float

    @staticmethod
    def new(r, g, b):
        return ColourRgbF(float(r), float(g), float(b))

    @staticmethod
    def from_named(name: NamedColour):
        return ColourRgbF(*name.value)


@dataclass
class Spectrum:
    shortest_wavelength: float
    longest_wavelength: float
    samples: np.ndarray

    @staticmethod
    def black():
        return Spectrum(SHORTEST_VISIBLE_WAVELENGTH, LONGEST_VISIBLE_WAVELENGTH, np.zeros(2))

    @staticmethod
    def grey(brightness):
        return Spectrum(SHORTEST_VISIBLE_WAVELENGTH, LONGEST_VISIBLE_WAVELENGTH, np.full(2, float(brightness)))

    @staticmethod
    def reflection_from_linear_rgb(colour: ColourRgbF):
        out = np.zeros(32)
        N.check(N.lib().vr_spectrum_reflection_from_linear_rgb(colour.red, colour.green, colour.blue,
                                                                out.ctypes.data_as(C.c_void_p)))
        return Spectrum(380.0, 720.0, out)

    def intensity_at_wavelength(self, wavelength):
        s = np.ascontiguousarray(self.samples, dtype=np.float64)
        sp = N.Spectrum(self.shortest_wavelength, self.longest_wavelength, s.size,
                        s.ctypes.data_as(C.POINTER(C.c_double)))
        return N.lib().vr_spectrum_intensity_at_wavelength(C.byref(sp), float(wavelength))


# ------------------------------------------------------------------------------ materials
@dataclass
class LambertianMaterial:
    colour: Spectrum
    diffuse_strength: float

    @staticmethod
    def new_dummy():  # lambertian_material.rs:19-24
        return LambertianMaterial(Spectrum.black(), 1.0)


@dataclass
class ReflectiveMaterial:
    colour: Spectrum
    diffuse_strength: float
    reflection_strength: float


@dataclass
class PhongMaterial:
    """materials/phong_material.rs:8-37; sampled by CosineWeightedHemisphere (materials/mod.rs:28-33)."""
    colour: Spectrum
    diffuse_strength: float
    specular_strength: float
    smoothness: float


@dataclass
class SmoothTransparentDialectric:
    """materials/smooth_transparent_dialectric.rs:64-115 (the reference's spelling): refractive index
    eta(lambda) as a Spectrum."""
    eta: Spectrum

    @staticmethod
    def new(eta):
        return SmoothTransparentDialectric(eta)


# ------------------------------------------------------------------------------ integrators
@dataclass
class DirectionalLight:
    """integrators/whitted_integrator.rs:10-13."""
    direction: tuple
    spectrum: Spectrum


@dataclass
class WhittedIntegrator:
    """integrators/whitted_integrator.rs:15-87.  The reference's partial_render_scene always uses
    SimpleRandomIntegrator (camera.rs:103); here a Scene may carry this one instead."""
    ambient_light: Spectrum
    lights: list


# ------------------------------------------------------------------------------ geometry
@dataclass
class Plane:
    normal: tuple
    distance_from_origin: float
    material: object


@dataclass
class Sphere:
    centre: tuple
    radius: float
    material: object


@dataclass
class Mesh:
    """A triangle mesh: vertices/normals float64 [n][3][3] (Vec<Triangle>, triangle.rs:8-13)."""
    vertices: np.ndarray
    normals: np.ndarray
    material: object

    def __len__(self):
        return len(self.vertices)


class BoundingVolumeHierarchy:
    """BoundingVolumeHierarchy::build over a mesh.  The tree is built (with the reference's median
    split) by the native library when the scene is created."""

    def __init__(self, mesh: Mesh):
        self.mesh = mesh

    @staticmethod
    def build(mesh: Mesh):
        return BoundingVolumeHierarchy(mesh)


def load_obj(path, material):
    """mesh::load_obj: OBJ positions/normals as f32 widened to f64, fan-triangulated polygons."""
    L = N.lib()
    n = C.c_uint64()
    v = C.POINTER(C.c_double)()
    nn = C.POINTER(C.c_double)()
    N.check(L.vr_load_obj(str(path).encode(), C.byref(n), C.byref(v), C.byref(nn)))
    try:
        cnt = int(n.value) * 9
        verts = np.ctypeslib.as_array(v, shape=(max(cnt, 1),))[:cnt].copy().reshape(-1, 3, 3)
        norms = np.ctypeslib.as_array(nn, shape=(max(cnt, 1),))[:cnt].copy().reshape(-1, 3, 3)
    finally:
        L.vr_mesh_free(v, nn)
    return Mesh(verts, norms, material)


# ------------------------------------------------------------------------------ plain-data spec
@dataclass
class MaterialSpec:
    kind: int
    colour: Spectrum
    diffuse_strength: float
    reflection_strength: float = 0.0  # reflective; Phong's specular strength
    smoothness: float = 0.0           # Phong


@dataclass
class PrimitiveSpec:
    kind: int
    material: int
    vector: tuple
    scalar: float


@dataclass
class MeshSpec:
    vertices: np.ndarray
    normals: np.ndarray
    material: int


@dataclass
class ObjectSpec:
    kind: str  # "primitives" | "bvh"
    primitives: List[PrimitiveSpec] = field(default_factory=list)
    mesh: int = -1


@dataclass
class SceneSpec:
    camera_location: tuple
    materials: List[MaterialSpec]
    meshes: List[MeshSpec]
    objects: List[ObjectSpec]
    integrator: object = None  # None (SimpleRandomIntegrator) or WhittedIntegrator


class Scene:
    """scene::Scene { camera_location, objects } (src/scene.rs:5-8).

    objects: list whose items are either a list of Plane/Sphere (a Vec<Box<dyn Primitive>>
    aggregate) or a BoundingVolumeHierarchy."""

    def __init__(self, camera_location, objects, integrator=None):
        self.camera_location = tuple(float(c) for c in camera_location)
        self.objects = list(objects)
        self.integrator = integrator
        self._spec = None
        self._device_scenes = {}

    def spec(self) -> SceneSpec:
        if self._spec is None:
            mats, mat_ids = [], {}

            def mid(m):
                if id(m) not in mat_ids:
                    mat_ids[id(m)] = len(mats)
                    if isinstance(m, ReflectiveMaterial):
                        mats.append(MaterialSpec(N.MATERIAL_REFLECTIVE, m.colour, m.diffuse_strength,
                                                 m.reflection_strength))
                    elif isinstance(m, LambertianMaterial):
                        mats.append(MaterialSpec(N.MATERIAL_LAMBERTIAN, m.colour, m.diffuse_strength, 0.0))
                    elif isinstance(m, PhongMaterial):
                        mats.append(MaterialSpec(N.MATERIAL_PHONG, m.colour, m.diffuse_strength, m.specular_strength,
                                                 m.smoothness))
                    elif isinstance(m, SmoothTransparentDialectric):
                        mats.append(MaterialSpec(N.MATERIAL_DIELECTRIC, m.eta, 0.0, 0.0))
                    else:
                        raise TypeError(f"unsupported material {type(m).__name__}")
                return mat_ids[id(m)]

            meshes, objs = [], []
            for o in self.objects:
                if isinstance(o, BoundingVolumeHierarchy):
                    meshes.append(MeshSpec(np.ascontiguousarray(o.mesh.vertices, dtype=np.float64),
                                           np.ascontiguousarray(o.mesh.normals, dtype=np.float64),
                                           mid(o.mesh.material)))
                    objs.append(ObjectSpec("bvh", mesh=len(meshes) - 1))
                else:
                    prims = []
                    for p in o:
                        if isinstance(p, Plane):
                            prims.append(PrimitiveSpec(N.PRIMITIVE_PLANE, mid(p.material), tuple(p.normal),
                                                       float(p.distance_from_origin)))
                        elif isinstance(p, Sphere):
                            prims.append(PrimitiveSpec(N.PRIMITIVE_SPHERE, mid(p.material), tuple(p.centre),
                                                       float(p.radius)))
                        else:
                            raise TypeError(f"unsupported primitive {type(p).__name__}")
                    objs.append(ObjectSpec("primitives", prims))
            self._spec = SceneSpec(self.camera_location, mats, meshes, objs, self.integrator)
        return self._spec

    def device_scene(self, device=0, host_only=False, device_bvh=False, reference_bvh=False, device_sah=False,
                     wide_offsets=False):
        key = (device, host_only, device_bvh, reference_bvh, device_sah, wide_offsets)
        if key not in self._device_scenes:
            self._device_scenes[key] = DeviceScene(self.spec(), device, host_only, device_bvh, reference_bvh,
                                                   device_sah, wide_offsets=wide_offsets)
        return self._device_scenes[key]


class DeviceScene:
    """Owner of a `vr_scene*` (flattened BVH resident in one GPU's HBM)."""

    def __init__(self, spec: SceneSpec, device=0, host_only=False, device_bvh=False, reference_bvh=False,
                 device_sah=False, greedy_collapse=False, wide_offsets=False):
        """device_bvh: build the BVHs on the GPU (VR_SCENE_DEVICE_BVH: the reference's tree);
        reference_bvh: traverse the reference's median-split tree instead of the SAH tree;
        device_sah: build the SAH traversal tree on the GPU too (VR_SCENE_DEVICE_SAH);
        greedy_collapse: the greedy 4-wide collapse instead of the SAH-optimal one (inspection);
        wide_offsets: render with the 64-bit-offset kernels that scenes past 53.7 M triangles or 2^25
        wide nodes take automatically (VR_SCENE_WIDE_OFFSETS; identical renders)."""
        L = N.lib()
        self.spec = spec
        keep = []  # keep ctypes buffers alive during vr_scene_create
        mats = (N.MaterialDesc * max(len(spec.materials), 1))()
        for i, m in enumerate(spec.materials):
            s = np.ascontiguousarray(m.colour.samples, dtype=np.float64)
            keep.append(s)
            mats[i] = N.MaterialDesc(m.kind, 0, N.Spectrum(m.colour.shortest_wavelength, m.colour.longest_wavelength,
                                                           s.size, s.ctypes.data_as(C.POINTER(C.c_double))),
                                     m.diffuse_strength, m.reflection_strength, m.smoothness)
        prims, objs, meshes = [], [], []
        for o in spec.objects:
            if o.kind == "primitives":
                objs.append(N.ObjectDesc(N.OBJECT_PRIMITIVE_LIST, len(prims), len(o.primitives), 0))
                for p in o.primitives:
                    prims.append(N.PrimitiveDesc(p.kind, p.material, N.Vec3(*p.vector), p.scalar))
            else:
                objs.append(N.ObjectDesc(N.OBJECT_BVH, o.mesh, 1, 0))
        for m in spec.meshes:
            v = np.ascontiguousarray(m.vertices, dtype=np.float64).reshape(-1)
            nn = np.ascontiguousarray(m.normals, dtype=np.float64).reshape(-1)
            assert v.size == nn.size and v.size % 9 == 0
            keep += [v, nn]
            meshes.append(N.MeshDesc(v.size // 9, v.ctypes.data_as(C.POINTER(C.c_double)),
                                     nn.ctypes.data_as(C.POINTER(C.c_double)), m.material, 0))
        prim_arr = (N.PrimitiveDesc * max(len(prims), 1))(*prims)
        obj_arr = (N.ObjectDesc * max(len(objs), 1))(*objs)
        mesh_arr = (N.MeshDesc * max(len(meshes), 1))(*meshes)
        ig = None
        if spec.integrator is not None:
            def cspec(sp):
                a = np.ascontiguousarray(sp.samples, dtype=np.float64)
                keep.append(a)
                return N.Spectrum(sp.shortest_wavelength, sp.longest_wavelength, a.size,
                                  a.ctypes.data_as(C.POINTER(C.c_double)))
            lights = (N.DirectionalLightC * max(len(spec.integrator.lights), 1))()
            for j, li in enumerate(spec.integrator.lights):
                lights[j] = N.DirectionalLightC(N.Vec3(*li.direction), cspec(li.spectrum))
            keep.append(lights)
            ig = N.IntegratorDesc(N.INTEGRATOR_WHITTED, len(spec.integrator.lights),
                                  cspec(spec.integrator.ambient_light), lights)
        desc = N.SceneDesc(N.Vec3(*spec.camera_location), len(spec.materials), len(prims), len(meshes), len(objs),
                           mats, prim_arr, mesh_arr, obj_arr, C.pointer(ig) if ig is not None else None)
        h = C.c_void_p()
        flags = ((N.SCENE_HOST_ONLY if host_only else 0) | (N.SCENE_DEVICE_BVH if device_bvh else 0) |
                 (N.SCENE_REFERENCE_BVH if reference_bvh else 0) | (N.SCENE_DEVICE_SAH if device_sah else 0) |
                 (N.SCENE_GREEDY_COLLAPSE if greedy_collapse else 0) | (N.SCENE_WIDE_OFFSETS if wide_offsets else 0))
        N.check(L.vr_scene_create(C.byref(desc), device, flags, C.byref(h)))
        self.handle = h
        self.device = device
        self.host_only = host_only
        # bound now: at interpreter exit module globals (N, N.lib) may already be torn down when
        # __del__ runs; scenes still alive then are released by _release_live_scenes (atexit)
        self._destroy = L.vr_scene_destroy
        _LIVE.add(self)

    def release(self):
        """vr_scene_destroy now (waits for the scene's queued work); idempotent."""
        h = getattr(self, "handle", None)
        if h:
            self.handle = None
            self._destroy(h)

    def __del__(self):
        self.release()

    def set_staging_limit(self, nbytes):
        """vr_scene_set_staging_limit: cap one call's staging memory (0: half the free HBM); larger
        frames run in several launches with bit-identical records."""
        N.check(N.lib().vr_scene_set_staging_limit(self.handle, int(nbytes)))

    def info(self):
        i = N.SceneInfo()
        N.check(N.lib().vr_scene_get_info(self.handle, C.byref(i)))
        d = {n: getattr(i, n) for n, _ in i._fields_}
        d["nan_free"] = bool(d["flags"] & N.SCENE_INFO_NAN_FREE)
        return d

    def set_fault_object(self, obj):
        """Test hook (vr_debug_set_fault_object): hits on scene object `obj` report the singular
        shading basis (VR_ERROR_SINGULAR_BASIS); -1 turns it off."""
        N.check(N.lib().vr_debug_set_fault_object(self.handle, obj))

    def set_launch_flags(self, no_cull=False, no_dist_cull=False, no_coop=False, no_lone_walk=False, stack32=False):
        """Test hook (vr_debug_set_launch_flags): every later render of this scene -- per-sample
        records and host buffers included -- skips the frustum culling, the BVH distance culling or
        the cooperative tail or its whole-walk form, or keeps 32-bit traversal-stack entries (each
        leaves the records bit-identical)."""
        flags = ((N.LAUNCH_NO_CULL if no_cull else 0) | (N.LAUNCH_NO_DIST_CULL if no_dist_cull else 0) |
                 (N.LAUNCH_NO_COOP if no_coop else 0) | (N.LAUNCH_NO_LONE_WALK if no_lone_walk else 0) |
                 (N.LAUNCH_STACK32 if stack32 else 0))
        N.check(N.lib().vr_debug_set_launch_flags(self.handle, flags))

    NODE_DTYPE = np.dtype([("box", "<f8", (2, 6)), ("child", "<i4", (2,)), ("pad", "<i4", (6,))])

    def bvh_nodes(self):
        """The flattened interior nodes (vr_scene_bvh_nodes), a structured array."""
        out = np.zeros(self.info()["node_count"], dtype=self.NODE_DTYPE)
        if out.size:
            N.check(N.lib().vr_scene_bvh_nodes(self.handle, out.ctypes.data_as(C.c_void_p)))
        return out

    def leaf_order(self, mesh):
        out = np.zeros(len(self.spec.meshes[mesh].vertices), dtype=np.uint64)
        N.check(N.lib().vr_scene_bvh_leaf_order(self.handle, mesh, out.ctypes.data_as(C.c_void_p)))
        return out
