"""The 4-wide traversal tree's collapse (CPU: host-only scenes, no GPU).

The SAH-optimal DP collapse (vr_host.cpp WideBuilder; VR_SCENE_GREEDY_COLLAPSE builds the greedy one) may take a node's DP expansion
only where its subtree's stack bound keeps the greedy tree's LDS stack class (24 / 32 / 48 entries of
the render kernel's traversal stack): the stack bound never moves to a larger class, and the DP tree
never has more wide nodes than the greedy one (fuller nodes).  Which tree is walked does not change
a record (the GPU tests render both); this checks the builder's invariants.
"""
import pytest

from vanrijn_amd import scenes
from vanrijn_amd.scene import DeviceScene


def stack_class(stack):
    d = stack + 1  # the kernel's depth: the bound + 1 spare entry for branchless pushes
    return 0 if d <= 24 else (1 if d <= 32 else 2)


def info(spec, dp):
    return DeviceScene(spec, 0, host_only=True, greedy_collapse=not dp).info()


@pytest.mark.parametrize("mesh", [
    scenes.displaced_mesh(16, scenes._BUNNY_BUMPS, 0xB0BB1E, 24, 0.04, (1.25, 1.05, 1.15), (-1.7, -0.8, 0.0)),
    scenes.displaced_mesh(40, scenes._BUNNY_BUMPS, 0x5EED, 40, 0.08, (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)),
])
def test_dp_collapse_keeps_stack_class_and_fills_nodes(mesh):
    spec = scenes.main_scene(mesh).spec()
    g = info(spec, False)
    d = info(spec, True)
    assert g["triangle_count"] == d["triangle_count"] > 1000
    assert stack_class(d["traversal_stack"]) <= stack_class(g["traversal_stack"])
    assert d["wide_node_count"] <= g["wide_node_count"]
    # every wide node holds at least two children: n triangles need at least (n - 1) / 3 nodes
    assert d["wide_node_count"] >= (d["triangle_count"] - 1) // 3
