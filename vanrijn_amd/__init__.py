"""vanrijn_amd -- MI355X (gfx950) native core for vanrijn's per-pixel path-tracing hot path.

The product is the C-ABI library vanrijn_amd/lib/libvanrijn_amd.so (HIP kernels + C++ host,
include/vanrijn_amd.h).  This package is the host-side mirror of the reference's API over that
library; every pixel is computed on the GPU.
"""
from .render import (AccumulationBuffer, ImageRgbU8, Tile, TileIterator, partial_render_scene, render_samples,
                     render_tile, render_tile_device, resolve_state, tone_map_device, trace_rays)
from .scene import (BoundingVolumeHierarchy, ColourRgbF, DeviceScene, DirectionalLight, LambertianMaterial, Mesh,
                    NamedColour, PhongMaterial, Plane, WhittedIntegrator, ReflectiveMaterial, Scene, SceneSpec, SmoothTransparentDialectric, Sphere,
                    Spectrum, load_obj)
from . import _native

__all__ = [
    "AccumulationBuffer", "ImageRgbU8", "Tile", "TileIterator", "partial_render_scene", "render_samples", "render_tile",
    "render_tile_device", "resolve_state", "tone_map_device", "trace_rays", "BoundingVolumeHierarchy", "ColourRgbF", "DeviceScene",
    "LambertianMaterial", "Mesh", "NamedColour", "PhongMaterial", "Plane", "ReflectiveMaterial", "Scene", "SceneSpec",
    "SmoothTransparentDialectric", "Sphere", "Spectrum", "load_obj", "DirectionalLight", "WhittedIntegrator",
]


def device_count():
    return _native.lib().vr_device_count()
