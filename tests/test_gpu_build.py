"""BoundingVolumeHierarchy::build_from_slice (bounding_volume_hierarchy.rs:38-74) on the device
(VR_SCENE_DEVICE_BVH, vanrijn_amd/csrc/vr_build.hip) against the host build (vr_host.cpp), which
the oracle pins (tests/test_oracle_scene.py: leaf orders equal to the oracle's build).

Bar: identical interior nodes (child boxes compared with ==, child links), identical leaf order
and depth, and bitwise-identical renders.  Meshes cover the shapes the median split meets: n = 1,
2, 3 and odd sizes, equal box centres (ties broken by input index), flat axes (largest_dimension's
-1 rule), -0.0 coordinates, and the bunny stand-in.
"""
import time

import numpy as np
import pytest

from vanrijn_amd import scenes
from vanrijn_amd.render import Tile, render_tile_device
from vanrijn_amd.scene import LambertianMaterial, Mesh, Scene, Spectrum, BoundingVolumeHierarchy

pytestmark = pytest.mark.gpu


def _mesh_scene(v):
    v = np.asarray(v, dtype=np.float64).reshape(-1, 3, 3)
    n = np.zeros_like(v)
    n[..., 2] = 1.0
    mat = LambertianMaterial(Spectrum.grey(0.5), 0.5)
    return Scene((0.0, 0.0, -5.0), [BoundingVolumeHierarchy.build(Mesh(v, n, mat))])


def _random_mesh(rng, n, ties=False, flat=False):
    v = rng.normal(size=(n, 3, 3))
    if ties:  # many equal box centres
        v = np.round(v * 2) / 2
    if flat:  # one axis without extent
        v[..., 2] = 0.0
        v[: n // 3, :, 2] = -0.0
    return v


def _compare(scene):
    host = scene.device_scene(0, host_only=True, reference_bvh=True)
    dev = scene.device_scene(0, device_bvh=True)
    hi, di = host.info(), dev.info()
    assert (hi["node_count"], hi["triangle_count"], hi["max_bvh_depth"]) == \
           (di["node_count"], di["triangle_count"], di["max_bvh_depth"])
    hn, dn = host.bvh_nodes(), dev.bvh_nodes()
    assert np.array_equal(hn["child"], dn["child"])
    assert np.array_equal(hn["box"], dn["box"])  # == : a zero's sign may differ, never a value
    for m in range(len(scene.spec().meshes)):
        assert np.array_equal(host.leaf_order(m), dev.leaf_order(m))
    # the render kernel's 4-wide trees differ (host: surface-area collapse of the SAH tree;
    # device: parity collapse of the median-split tree) -- the images may not
    _render_equal(scene.device_scene(0), dev)
    assert 0 < di["wide_node_count"] <= max(1, di["node_count"]) or di["node_count"] == 0
    return dev


def _render_equal(a, b, W=48, H=40):
    import torch
    out = []
    for ds in (a, b):
        st = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
        render_tile_device(ds, Tile(0, W, 0, H), H, W, 3, 0x5EED0001, 0, st.data_ptr())
        out.append(st.cpu().numpy())
    # bitwise where finite; degenerate shading bases (an edge parallel to the normal) give NaN
    # photons in the reference too (oracle: the same samples), and NaN != NaN
    assert np.array_equal(out[0], out[1], equal_nan=True)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 1000, 4097])
def test_device_build_matches_host_random(n):
    rng = np.random.default_rng(n)
    _compare(_mesh_scene(_random_mesh(rng, n)))


@pytest.mark.parametrize("kind", ["ties", "flat"])
def test_device_build_matches_host_degenerate(kind):
    rng = np.random.default_rng(11)
    _compare(_mesh_scene(_random_mesh(rng, 3000, ties=kind == "ties", flat=kind == "flat")))


def test_device_build_bunny_renders_identically():
    import torch
    s = scenes.main_scene(scenes.procedural_bunny())
    dev = _compare(s)
    host = s.device_scene(0, reference_bvh=True)
    sah = s.device_scene(0)  # the default SAH traversal tree: the same image, bit for bit
    W, H = 192, 128
    out = []
    for ds in (host, dev, sah):
        st = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
        render_tile_device(ds, Tile(0, W, 0, H), H, W, 4, 0x5EED0001, 0, st.data_ptr())
        out.append(st.cpu())
    assert torch.equal(out[0], out[1])
    assert torch.equal(out[0], out[2])


def test_device_build_c5_mesh():
    """the 1,051,392-triangle synthetic mesh -- equal leaf order, and the time."""
    v, n = scenes.synthetic_sphere_mesh()
    s = Scene(scenes.CAMERA_LOCATION, [BoundingVolumeHierarchy.build(Mesh(v, n, LambertianMaterial(
        Spectrum.grey(0.5), 0.5)))])
    t0 = time.perf_counter()
    dev = s.device_scene(0, device_bvh=True)
    t_dev = time.perf_counter() - t0
    t0 = time.perf_counter()
    host = s.device_scene(0, host_only=True, reference_bvh=True)
    t_host = time.perf_counter() - t0
    assert np.array_equal(host.leaf_order(0), dev.leaf_order(0))
    hn, dn = host.bvh_nodes(), dev.bvh_nodes()
    assert np.array_equal(hn["child"], dn["child"]) and np.array_equal(hn["box"], dn["box"])
    print(f"C5 build: device {t_dev:.3f} s, host {t_host:.3f} s; wide nodes {dev.info()['wide_node_count']}, "
          f"stack {dev.info()['traversal_stack']}")
    _render_equal(s.device_scene(0), dev)


# ---------------------------------------------------------------- the SAH traversal tree on the device
def _sah_tree_is_valid(ds, n):
    """The device SAH tree: n - 1 interior nodes, every triangle in exactly one leaf, every child
    box containing its subtree's triangle boxes (the union rule the conservative walk relies on)."""
    nodes = ds.bvh_nodes()
    assert len(nodes) == n - 1
    leaves = np.sort(~nodes["child"][nodes["child"] < 0])
    assert np.array_equal(leaves, np.arange(n))
    inner = nodes["child"][nodes["child"] >= 0]
    assert len(np.unique(inner)) == len(inner) == n - 2  # every non-root interior node once
    for i in range(len(nodes)):
        for c in range(2):
            ch = nodes["child"][i, c]
            if ch >= 0:  # a child node's own boxes lie inside the box the parent keeps for it
                pb = nodes["box"][i, c]
                for cc in range(2):
                    b = nodes["box"][ch, cc]
                    assert (b[0::2] >= pb[0::2]).all() and (b[1::2] <= pb[1::2]).all()


@pytest.mark.parametrize("n", [2, 3, 17, 1000, 4097])
def test_device_sah_tree_renders_like_the_host_tree(n):
    rng = np.random.default_rng(100 + n)
    s = _mesh_scene(_random_mesh(rng, n, ties=n == 1000))
    dev = s.device_scene(0, device_sah=True)
    host = s.device_scene(0)
    assert np.array_equal(dev.leaf_order(0), host.leaf_order(0))  # the reference ranks
    _sah_tree_is_valid(dev, n)
    _render_equal(host, dev)


def test_device_sah_bunny_and_c5():
    """The default traversal tree built on the device: the main.rs scene renders bit-identically
    to the host-built scene, and the C5 mesh builds in well under a second."""
    import torch
    s = scenes.main_scene(scenes.procedural_bunny())
    dev, host = s.device_scene(0, device_sah=True), s.device_scene(0)
    assert dev.info()["traversal_stack"] <= 47 and dev.info()["nan_free"]
    _render_equal(host, dev, W=160, H=120)
    v, n = scenes.synthetic_sphere_mesh()
    c5 = Scene(scenes.CAMERA_LOCATION, [BoundingVolumeHierarchy.build(Mesh(v, n, LambertianMaterial(
        Spectrum.grey(0.5), 0.5)))])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d5 = c5.device_scene(0, device_sah=True)
    t_dev = time.perf_counter() - t0
    t0 = time.perf_counter()
    h5 = c5.device_scene(0)
    t_host = time.perf_counter() - t0
    i5 = d5.info()
    print(f"C5 SAH build: device {t_dev:.3f} s, host {t_host:.3f} s; wide nodes {i5['wide_node_count']} "
          f"(host {h5.info()['wide_node_count']}), stack {i5['traversal_stack']}, depth {i5['max_bvh_depth']}")
    assert t_dev < 1.0
    assert np.array_equal(d5.leaf_order(0), h5.leaf_order(0))
    _render_equal(h5, d5, W=64, H=48)
