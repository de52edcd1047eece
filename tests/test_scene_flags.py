"""VR_SCENE_INFO_NAN_FREE (vr_host.cpp shading_finite), host-only scenes (CPU).

The early stop of zero-throughput paths is allowed only where every continuation is provably
finite ("NaN fidelity"): each traced triangle's vertex normals strictly on
one side of its plane, no Phong / dielectric material.  Otherwise the reference's 0 * NaN must
reach the pixel (simple_random_integrator.rs:39-53, mesh.rs:37, triangle.rs:73-78)."""
import numpy as np

from vanrijn_amd import scenes
from vanrijn_amd.scene import (BoundingVolumeHierarchy, LambertianMaterial, Mesh, PhongMaterial, Scene, Spectrum)


def _flag(scene):
    return scene.device_scene(0, host_only=True).info()["nan_free"]


def _tri_scene(normals):
    v = np.array([[[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]]])
    mat = LambertianMaterial(Spectrum.grey(0.5), 0.5)
    return Scene((0.0, 0.0, -5.0), [BoundingVolumeHierarchy.build(Mesh(v, np.asarray(normals, float)[None], mat))])


def test_reference_scenes_are_nan_free():
    small = scenes.displaced_mesh(10, scenes._BUNNY_BUMPS, 0xB0BB1E, 8, 0.04, (1.25, 1.05, 1.15), (-1.7, -0.8, 0.0))
    assert _flag(scenes.main_scene(small)) and _flag(scenes.bench_scene(small))


def test_normals_decide():
    up = [0.0, 0.0, 1.0]
    assert _flag(_tri_scene([up, up, up]))
    assert _flag(_tri_scene([[0.0, 0.0, -1.0]] * 3))          # all on the other side: fine too
    assert _flag(_tri_scene([[0.3, 0.0, 1.0], [0.0, -0.5, 1.0], up]))
    assert not _flag(_tri_scene([[0.0, 0.0, 0.0]] * 3))       # an OBJ without normals (mesh.rs:37)
    assert not _flag(_tri_scene([up, up, [0.0, 0.0, -1.0]]))  # the interpolated normal can vanish
    assert not _flag(_tri_scene([up, up, [1.0, 0.0, 0.0]]))   # in the plane: cotangent can vanish
    assert not _flag(_tri_scene([up, up, [np.nan, 0.0, 1.0]]))


def test_degenerate_triangle_and_phong():
    mat = LambertianMaterial(Spectrum.grey(0.5), 0.5)
    v = np.array([[[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [2.0, 0.0, 0.0]]])  # zero area
    n = np.tile([0.0, 0.0, 1.0], (1, 3, 1))
    assert not _flag(Scene((0.0, 0.0, -5.0), [BoundingVolumeHierarchy.build(Mesh(v, n, mat))]))
    up = np.tile([0.0, 0.0, 1.0], (1, 3, 1))
    good = np.array([[[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]]])
    phong = PhongMaterial(Spectrum.grey(0.5), 0.5, 0.3, 10.0)
    assert not _flag(Scene((0.0, 0.0, -5.0), [BoundingVolumeHierarchy.build(Mesh(good, up, phong))]))
