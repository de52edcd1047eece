"""Scenes of the reference's harnesses, and the procedural meshes that stand in for the bunny.

* `main_scene(mesh)`  -- src/main.rs:120-189: plane y=-2 and three spheres in one primitive list,
  then the mesh's BVH; Lambertian materials; camera (-2, 1, -5).
* `bench_scene(mesh)` -- benches/simple_scene.rs:19-38: the mesh BVH only, ReflectiveMaterial
  {yellow, diffuse 0.05, reflection 0.9} (the bench passes a ColourRgbF where a Spectrum is needed,
  so it does not compile; the intended Spectrum::reflection_from_linear_rgb(yellow)
  is used here).

`test_data/stanford_bunny.obj` is a Git-LFS pointer in the reference, so the default
mesh is a deterministic procedural stand-in, `procedural_bunny()`: a cube-sphere (6 faces x 76^2
quads x 2 = 69,312 triangles, close to the real bunny's 69,451) radially displaced by a head, two
ears, a tail and 48 hashed bumps, with smooth area-weighted vertex normals.  It is built only from
IEEE-exact operations (+ - * / sqrt max and integer hashing), so every machine produces the same
bits.  A real OBJ can be used instead with `load_bunny(path)`, which checks the reference file's
size and sha256 first.
"""
import hashlib
import os

import numpy as np

from .scene import (BoundingVolumeHierarchy, ColourRgbF, LambertianMaterial, Mesh, NamedColour, PhongMaterial, Plane,
                    ReflectiveMaterial, Scene, SmoothTransparentDialectric, Spectrum, Sphere, load_obj,
                    DirectionalLight, WhittedIntegrator)

CAMERA_LOCATION = (-2.0, 1.0, -5.0)  # main.rs:139, simple_scene.rs:25
BUNNY_SHA256 = "7ee71a949c270c53226056a0ad120e8a8dcdba54d36c2420f987dd1cdd4e302f"
BUNNY_SIZE = 4858404

_M64 = (1 << 64) - 1


def _mix64(z):
    z &= _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _unit(seed, k):
    """k-th uniform double in [0, 1) of a hashed stream (exact integer -> float conversion)."""
    return (_mix64(seed + (k + 1) * 0x9E3779B97F4A7C15) >> 11) * 2.0 ** -53


def _normalize_rows(v):
    n = np.sqrt(v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1] + v[..., 2] * v[..., 2])
    return v * (1.0 / n)[..., None]


def cube_sphere(n):
    """Unique lattice vertices of a cube surface ([-n, n]^3 integer points with a coordinate at
    +-n) and outward-wound triangles (6 * n^2 * 2)."""
    index = {}
    verts = []

    def vid(p):
        if p not in index:
            index[p] = len(verts)
            verts.append(p)
        return index[p]

    tris = []
    # (axis, sign): face at coordinate sign*n along axis, parameterised by the other two axes
    for axis in range(3):
        for sign in (1, -1):
            a1, a2 = (axis + 1) % 3, (axis + 2) % 3
            for i in range(n):
                for j in range(n):
                    q = []
                    for di, dj in ((0, 0), (1, 0), (1, 1), (0, 1)):
                        p = [0, 0, 0]
                        p[axis] = sign * n
                        p[a1] = -n + 2 * (i + di)
                        p[a2] = -n + 2 * (j + dj)
                        q.append(vid(tuple(p)))
                    if sign > 0:
                        tris.append((q[0], q[1], q[2]))
                        tris.append((q[0], q[2], q[3]))
                    else:
                        tris.append((q[0], q[2], q[1]))
                        tris.append((q[0], q[3], q[2]))
    lattice = np.array(verts, dtype=np.float64) * (1.0 / n)
    return lattice, np.array(tris, dtype=np.int64)


def _bump(dirs, centre, radius, amplitude):
    c = np.array(centre, dtype=np.float64)
    c = c * (1.0 / np.sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]))
    d = dirs - c
    d2 = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]
    w = np.maximum(0.0, 1.0 - d2 * (1.0 / (radius * radius)))
    return amplitude * (w * w)


def displaced_mesh(n, bumps, noise_seed, noise_count, noise_amp, scale, centre):
    lattice, tris = cube_sphere(n)
    dirs = _normalize_rows(lattice)
    r = np.ones(len(dirs))
    for b in bumps:
        r = r + _bump(dirs, *b)
    for k in range(noise_count):
        c = (2.0 * _unit(noise_seed, 4 * k) - 1.0, 2.0 * _unit(noise_seed, 4 * k + 1) - 1.0,
             2.0 * _unit(noise_seed, 4 * k + 2) - 1.0)
        amp = noise_amp * (2.0 * _unit(noise_seed, 4 * k + 3) - 1.0)
        r = r + _bump(dirs, c, 0.35, amp)
    pos = dirs * r[:, None] * np.array(scale, dtype=np.float64) + np.array(centre, dtype=np.float64)
    # smooth vertex normals: area-weighted sum of face normals, accumulated in a fixed order
    v0, v1, v2 = pos[tris[:, 0]], pos[tris[:, 1]], pos[tris[:, 2]]
    e1, e2 = v1 - v0, v2 - v0
    fn = np.stack([e1[:, 1] * e2[:, 2] - e1[:, 2] * e2[:, 1], e1[:, 2] * e2[:, 0] - e1[:, 0] * e2[:, 2],
                   e1[:, 0] * e2[:, 1] - e1[:, 1] * e2[:, 0]], axis=1)
    vn = np.zeros_like(pos)
    for c in range(3):
        np.add.at(vn, tris[:, c], fn)
    vn = _normalize_rows(vn)
    vertices = np.ascontiguousarray(pos[tris])
    normals = np.ascontiguousarray(vn[tris])
    return vertices, normals


# head, ears, tail: (direction, angular radius, amplitude) in the unit-sphere frame
_BUNNY_BUMPS = [
    ((0.35, 0.55, -0.75), 0.75, 0.30),   # head
    ((0.15, 1.0, -0.45), 0.30, 0.95),    # left ear
    ((0.50, 1.0, -0.30), 0.30, 0.90),    # right ear
    ((-0.85, 0.15, 0.5), 0.45, 0.18),    # tail
    ((0.0, -1.0, 0.0), 0.9, -0.25),      # flattened base
]


def procedural_bunny(n=76):
    """The stand-in mesh: 69,312 triangles, bounds about x [-3.2, -0.45], y [-1.7, 1.05],
    z [-1.4, 1.25]: in front of the camera, above the plane y = -2."""
    return displaced_mesh(n, _BUNNY_BUMPS, noise_seed=0xB0BB1E, noise_count=48, noise_amp=0.04,
                          scale=(1.25, 1.05, 1.15), centre=(-1.7, -0.8, 0.0))


def synthetic_sphere_mesh(n=296):
    """C5's deep-BVH stress mesh: 12 * 296^2 = 1,051,392 triangles, radius ~1.5 around the
    stand-in bunny's position, displacement noise seed 0x1DEA."""
    return displaced_mesh(n, [], noise_seed=0x1DEA, noise_count=96, noise_amp=0.06, scale=(1.5, 1.5, 1.5),
                          centre=(-1.7, -0.4, 0.2))


def load_bunny(path):
    """The real reference mesh (test_data/stanford_bunny.obj), verified before use."""
    if os.path.getsize(path) != BUNNY_SIZE:
        raise ValueError(f"{path}: size differs from the reference bunny ({BUNNY_SIZE} B)")
    h = hashlib.sha256(open(path, "rb").read()).hexdigest()
    if h != BUNNY_SHA256:
        raise ValueError(f"{path}: sha256 {h} differs from the reference bunny")
    return path


def _mesh_arrays(mesh):
    if mesh is None:
        return procedural_bunny()
    if isinstance(mesh, str):
        m = load_obj(load_bunny(mesh), None)
        return m.vertices, m.normals
    return mesh


def main_scene(mesh=None):
    """src/main.rs:120-189."""
    v, nrm = _mesh_arrays(mesh)
    bunny = Mesh(v, nrm, LambertianMaterial(Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(
        NamedColour.Yellow)), 0.05))
    return Scene(CAMERA_LOCATION, [
        [
            Plane((0.0, 1.0, 0.0), -2.0, LambertianMaterial(
                Spectrum.reflection_from_linear_rgb(ColourRgbF.new(0.55, 0.27, 0.04)), 0.1)),
            Sphere((-6.25, -0.5, 1.0), 1.0, LambertianMaterial(
                Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(NamedColour.Green)), 0.1)),
            Sphere((-4.25, -0.5, 2.0), 1.0, LambertianMaterial(
                Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(NamedColour.Blue)), 0.1)),
            Sphere((-5.0, 1.5, 1.0), 1.0, LambertianMaterial(
                Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(NamedColour.Red)), 0.05)),
        ],
        BoundingVolumeHierarchy.build(bunny),
    ])


def bench_scene(mesh=None):
    """benches/simple_scene.rs:19-38 (mesh BVH only, reflective yellow)."""
    v, nrm = _mesh_arrays(mesh)
    mat = ReflectiveMaterial(Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(NamedColour.Yellow)), 0.05,
                             0.9)
    return Scene(CAMERA_LOCATION, [BoundingVolumeHierarchy.build(Mesh(v, nrm, mat))])


def materials_scene(mesh=None):
    """main.rs's layout with every material kind: a Phong sphere, a glass sphere
    (SmoothTransparentDialectric, eta 1.5), a reflective sphere, Lambertian plane and bunny.
    The reference instantiates Phong and the dielectric nowhere; this scene exercises them."""
    v, nrm = _mesh_arrays(mesh)
    bunny = Mesh(v, nrm, LambertianMaterial(Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(
        NamedColour.Yellow)), 0.05))
    return Scene(CAMERA_LOCATION, [
        [
            Plane((0.0, 1.0, 0.0), -2.0, LambertianMaterial(
                Spectrum.reflection_from_linear_rgb(ColourRgbF.new(0.55, 0.27, 0.04)), 0.1)),
            Sphere((-6.25, -0.5, 1.0), 1.0, PhongMaterial(
                Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(NamedColour.Green)), 0.1, 0.3, 40.0)),
            Sphere((-4.25, -0.5, 2.0), 1.0, SmoothTransparentDialectric(Spectrum.grey(1.5))),
            Sphere((-5.0, 1.5, 1.0), 1.0, ReflectiveMaterial(
                Spectrum.reflection_from_linear_rgb(ColourRgbF.from_named(NamedColour.Red)), 0.05, 0.9)),
        ],
        BoundingVolumeHierarchy.build(bunny),
    ])


def whitted_scene(mesh=None):
    """materials_scene rendered with the WhittedIntegrator: two directional lights and an
    ambient term (the reference ships no Whitted scene; this one exercises every material)."""
    s = materials_scene(mesh)
    warm = Spectrum.reflection_from_linear_rgb(ColourRgbF.new(1.0, 0.9, 0.7))
    cool = Spectrum.reflection_from_linear_rgb(ColourRgbF.new(0.3, 0.4, 0.8))
    s.integrator = WhittedIntegrator(Spectrum.grey(0.05), [DirectionalLight((0.4, 1.0, -0.3), warm),
                                                           DirectionalLight((-0.6, 0.8, 0.2), cool)])
    return s


def synthetic_scene():
    """C5: main.rs's plane and spheres + the 1M-triangle synthetic mesh (Lambertian yellow)."""
    s = main_scene(synthetic_sphere_mesh())
    return s
