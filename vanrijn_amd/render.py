"""Render API mirroring the reference (camera.rs, accumulation_buffer.rs, util/tile_iterator.rs).

    partial_render_scene(scene, tile, height, width) -> AccumulationBuffer   camera.rs:95-130
    AccumulationBuffer::{new, update_pixel, merge_tile}                     accumulation_buffer.rs:14-85
    Tile / TileIterator                                                     util/tile_iterator.rs:1-67
    AccumulationBuffer::to_image_rgb_u8(&ClampingToneMapper)               accumulation_buffer.rs:38-42
    ImageRgbU8 (get_colour, get_pixel_data, write_png)                      image.rs:8-66

Every render call goes through the C ABI into the gfx950 kernels; nothing here computes a pixel.
"""
import ctypes as C
import sys
import threading
from dataclasses import dataclass

import numpy as np

from . import _native as N
from . import records as R

RECURSION_LIMIT = 128  # camera.rs:69
SAMPLE_RECORD_DTYPE = np.dtype([("wavelength", "<f8"), ("intensity", "<f8"), ("xyz", "<f8", (3,)),
                                ("bounces", "<i4"), ("flags", "<i4")])
HIT_RECORD_DTYPE = np.dtype([("valid", "<i4"), ("object", "<i4"), ("primitive", "<i8"), ("distance", "<f8"),
                             ("location", "<f8", (3,)), ("normal", "<f8", (3,)), ("tangent", "<f8", (3,)),
                             ("cotangent", "<f8", (3,)), ("retro", "<f8", (3,))])
assert SAMPLE_RECORD_DTYPE.itemsize == C.sizeof(N.SampleRecord)
assert HIT_RECORD_DTYPE.itemsize == C.sizeof(N.HitRecord)


@dataclass(frozen=True)
class Tile:
    start_column: int
    end_column: int
    start_row: int
    end_row: int

    def width(self):
        return self.end_column - self.start_column

    def height(self):
        return self.end_row - self.start_row

    def _c(self):
        return N.TileC(self.start_column, self.end_column, self.start_row, self.end_row)


class TileIterator:
    """Row-major tiles of at most tile_size x tile_size covering the image exactly once."""

    def __init__(self, total_width, total_height, tile_size):
        assert tile_size > 0
        self.w, self.h, self.s = total_width, total_height, tile_size

    def __iter__(self):
        row = 0
        while row < self.h:
            col = 0
            while col < self.w:
                yield Tile(col, min(self.w, col + self.s), row, min(self.h, row + self.s))
                col += self.s
            row += self.s


class _OutputPool:
    """Backing stores for output AccumulationBuffers (11 f64 per pixel).  A store is handed out
    again only when nothing but the pool refers to it: every numpy view derived from a store --
    the five arrays of a buffer, and any slice or reshape a caller makes of them -- holds the store
    itself as its `.base`, so the store's reference count says whether any such view is alive."""

    def __init__(self, keep=32):
        self.keep = keep
        self.lock = threading.Lock()
        self.stores = []  # backing arrays
        # the reference count of a store nothing but the pool refers to, measured on this
        # interpreter (how many temporaries getrefcount itself sees differs between versions)
        probe = [np.empty(1)]
        self._free_refs = sys.getrefcount(probe[0])

    @staticmethod
    def _split(store, width, height):
        n = width * height
        return (store[0:3 * n].reshape(height, width, 3), store[3 * n:6 * n].reshape(height, width, 3),
                store[6 * n:9 * n].reshape(height, width, 3), store[9 * n:10 * n].reshape(height, width),
                store[10 * n:11 * n].reshape(height, width))

    def _free(self, i):
        # references: the pool's list (and getrefcount's own); any live view adds its .base
        return sys.getrefcount(self.stores[i]) <= self._free_refs

    def views(self, width, height):
        size = 11 * width * height
        with self.lock:
            for i in range(len(self.stores)):
                if self.stores[i].size == size and self._free(i):
                    return self._split(self.stores[i], width, height)
            store = np.empty(size)
            self.stores.append(store)
            if len(self.stores) > self.keep:  # forget a free store (or the oldest: its views keep it alive)
                for i in range(len(self.stores)):
                    if self._free(i):
                        del self.stores[i]
                        break
                else:
                    del self.stores[0]
            return self._split(store, width, height)


_OUTPUT_POOL = _OutputPool()


class AccumulationBuffer:
    """Per-pixel Kahan-compensated XYZ sums and weights; `colour` is the running mean.

    Arrays are [height][width][3] (XYZ) and [height][width] (weights), row-major like Array2D.
    The reference's `new(a, b)` names its parameters (height, width) but yields width = a,
    height = b (accumulation_buffer.rs:15-28 via array2d.rs:13-19); `new(width, height)` here.
    """

    def __init__(self, width, height):
        self.colour_buffer = np.zeros((height, width, 3))
        self.colour_sum_buffer = np.zeros((height, width, 3))
        self.colour_bias_buffer = np.zeros((height, width, 3))
        self.weight_buffer = np.zeros((height, width))
        self.weight_bias_buffer = np.zeros((height, width))

    @staticmethod
    def new(width, height):
        return AccumulationBuffer(width, height)

    @classmethod
    def _for_output(cls, width, height):
        """A buffer the library overwrites completely (all five arrays): no zeroing pass, and its
        memory recycled from buffers nobody references any more (_OutputPool) -- fresh pages cost
        a page fault per 4 KB on first write, as much host time as a 1-spp render itself."""
        b = cls.__new__(cls)
        (b.colour_buffer, b.colour_sum_buffer, b.colour_bias_buffer, b.weight_buffer,
         b.weight_bias_buffer) = _OUTPUT_POOL.views(width, height)
        return b

    def width(self):
        return self.colour_buffer.shape[1]

    def height(self):
        return self.colour_buffer.shape[0]

    def _c(self):
        for a in (self.colour_buffer, self.colour_sum_buffer, self.colour_bias_buffer, self.weight_buffer,
                  self.weight_bias_buffer):
            assert a.flags.c_contiguous and a.dtype == np.float64
        return N.AccumulationBufferC(self.width(), self.height(), self.colour_buffer.ctypes.data,
                                     self.colour_sum_buffer.ctypes.data, self.colour_bias_buffer.ctypes.data,
                                     self.weight_buffer.ctypes.data, self.weight_bias_buffer.ctypes.data)

    def merge_tile(self, tile: Tile, src: "AccumulationBuffer"):
        """accumulation_buffer.rs:62-85: weighted blend of the means; weights add (vr_merge_tile,
        host code in the library; the size asserts become VrError)."""
        dc, sc = self._c(), src._c()
        N.check(N.lib().vr_merge_tile(C.byref(dc), tile._c(), C.byref(sc)))

    def to_image_rgb_u8(self, device=0) -> "ImageRgbU8":
        """ClampingToneMapper over the XYZ colour buffer (image.rs:166-187), on the GPU."""
        c = np.ascontiguousarray(self.colour_buffer)
        out = np.zeros(c.shape, dtype=np.uint8)
        N.check(N.lib().vr_tone_map(c.ctypes.data_as(C.c_void_p), c.size // 3, out.ctypes.data_as(C.c_void_p),
                                    device))
        return ImageRgbU8(out)

    @staticmethod
    def from_state(state, width=None, height=None):
        """Build from a tile's state records (vanrijn_amd/records.py layout, ABI 7: a flat array of
        8 f64 per pixel, the sums half then the compensations half).  `width` / `height` may be left
        out for a [height][width][8] array, whose shape gives them; such an array must hold the flat
        layout reshaped, not the interleaved per-pixel records of ABI <= 6 -- a shape that does not
        fit raises ValueError instead of misreading the data."""
        a = np.asarray(state.cpu() if hasattr(state, "cpu") else state, dtype=np.float64)
        if width is None or height is None:
            if a.ndim != 3 or a.shape[2] != 8:
                raise ValueError("from_state: pass width and height, or a [height][width][8] array")
            height, width = a.shape[0], a.shape[1]
        if a.size != 8 * width * height:
            raise ValueError(f"from_state: {a.size} values for a {width}x{height} tile (8 f64 per pixel expected)")
        f = R.fields(a.reshape(-1), (height, width))
        b = AccumulationBuffer(width, height)
        b.colour_sum_buffer[...] = f["colour_sum"]
        b.colour_bias_buffer[...] = f["colour_bias"]
        b.weight_buffer[...] = f["weight"]
        b.weight_bias_buffer[...] = f["weight_bias"]
        wgt = f["weight"][..., None]
        with np.errstate(divide="ignore", invalid="ignore"):
            b.colour_buffer[...] = np.where(wgt != 0.0, f["colour_sum"] * (1.0 / wgt), 0.0)
        return b


def _scene_handle(scene, device):
    from .scene import DeviceScene, Scene
    if isinstance(scene, DeviceScene):
        return scene
    if isinstance(scene, Scene):
        return scene.device_scene(device)
    raise TypeError("expected Scene or DeviceScene")


def _params(tile, height, width, spp, seed, first_sample, accumulate):
    return N.RenderParams(tile._c(), height, width, spp, 1 if accumulate else 0, seed, first_sample)


def partial_render_scene(scene, tile: Tile, height: int, width: int, device=0) -> AccumulationBuffer:
    """camera.rs:95-130: one sample per pixel of `tile` into a fresh tile AccumulationBuffer."""
    ds = _scene_handle(scene, device)
    out = AccumulationBuffer._for_output(tile.width(), tile.height())
    oc = out._c()
    N.check(N.lib().vr_partial_render_scene(ds.handle, tile._c(), height, width, C.byref(oc)))
    return out


def render_tile(scene, tile: Tile, height, width, spp, seed, first_sample=0, accumulate: AccumulationBuffer = None,
                device=0) -> AccumulationBuffer:
    """spp samples per pixel with explicit seed / sample range (update_pixel semantics)."""
    ds = _scene_handle(scene, device)
    buf = accumulate if accumulate is not None else AccumulationBuffer._for_output(tile.width(), tile.height())
    bc = buf._c()
    p = _params(tile, height, width, spp, seed, first_sample, accumulate is not None)
    N.check(N.lib().vr_render_tile(ds.handle, C.byref(p), C.byref(bc)))
    return buf


def render_samples(scene, tile: Tile, height, width, spp, seed, first_sample=0, device=0):
    """Per-(pixel, sample) records [tile_h][tile_w][spp] (decision-identity checks)."""
    ds = _scene_handle(scene, device)
    out = np.zeros(tile.width() * tile.height() * spp, dtype=SAMPLE_RECORD_DTYPE)
    p = _params(tile, height, width, spp, seed, first_sample, False)
    N.check(N.lib().vr_render_samples(ds.handle, C.byref(p), out.ctypes.data_as(C.c_void_p)))
    return out.reshape(tile.height(), tile.width(), spp)


def trace_rays(scene, origins, directions, device=0):
    """Sampler::sample for a batch of rays (directions used as given)."""
    ds = _scene_handle(scene, device)
    o = np.ascontiguousarray(origins, dtype=np.float64).reshape(-1, 3)
    d = np.ascontiguousarray(directions, dtype=np.float64).reshape(-1, 3)
    out = np.zeros(len(o), dtype=HIT_RECORD_DTYPE)
    N.check(N.lib().vr_trace_rays(ds.handle, len(o), o.ctypes.data_as(C.c_void_p), d.ctypes.data_as(C.c_void_p),
                                  out.ctypes.data_as(C.c_void_p)))
    return out


def render_tile_device(scene, tile: Tile, height, width, spp, seed, first_sample, state_ptr, stream_ptr=None,
                       accumulate=False, timed=False, counters=False, device=0, defer_times=False, cull=True,
                       dist_cull=True, coop=True, lone_walk=True, stack16=True):
    """Enqueue a render into device state records (8 f64 per pixel, vanrijn_amd/records.py) at
    `state_ptr` (a device pointer, e.g. torch.Tensor.data_ptr()).  Returns launch stats (kernel
    time when timed; `variant`: the VR_VARIANT_* bits of the kernel that ran; `defer_times`: the
    events are recorded without waiting, read by collect_launch_times; `cull=False`: every sample
    traced, VR_LAUNCH_NO_CULL; `dist_cull=False`: no BVH distance culling, VR_LAUNCH_NO_DIST_CULL;
    `coop=False`: no cooperative tail, VR_LAUNCH_NO_COOP; `lone_walk=False`: the tail's walks in
    coop_step's per-step form only, VR_LAUNCH_NO_LONE_WALK; `stack16=False`: 32-bit traversal-stack
    entries where 16-bit ones would do, VR_LAUNCH_STACK32 -- all five leave the records bit-identical)."""
    ds = _scene_handle(scene, device)
    p = _params(tile, height, width, spp, seed, first_sample, accumulate)
    st = N.LaunchStats()
    flags = (N.LAUNCH_TIMED if timed or defer_times else 0) | (N.LAUNCH_COUNTERS if counters else 0) | \
        (N.LAUNCH_DEFER_TIMES if defer_times else 0) | (0 if cull else N.LAUNCH_NO_CULL) | \
        (0 if dist_cull else N.LAUNCH_NO_DIST_CULL) | (0 if coop else N.LAUNCH_NO_COOP) | \
        (0 if lone_walk else N.LAUNCH_NO_LONE_WALK) | (0 if stack16 else N.LAUNCH_STACK32)
    N.check(N.lib().vr_render_tile_device(ds.handle, C.byref(p), C.c_void_p(state_ptr),
                                          C.c_void_p(stream_ptr or 0), flags, C.byref(st)))
    return st.as_dict()


def collect_launch_times(scene, stream_ptr=None, device=0):
    """Waits for the defer_times launches of `scene` on the stream since the last collection:
    {kernel_ms, reduce_ms (sums), launches, passes, max_passes} (vr_collect_launch_times); raises
    their device errors like stream_check_error."""
    ds = _scene_handle(scene, device)
    t = N.LaunchTimes()
    N.check(N.lib().vr_collect_launch_times(ds.handle, C.c_void_p(stream_ptr or 0), C.byref(t)))
    return t.as_dict()


def stream_check_error(scene, stream_ptr=None, device=0):
    """Errors of earlier asynchronous launches of `scene` on a stream (vr_stream_check_error):
    raises VrError(VR_ERROR_SINGULAR_BASIS) once, then the stream is clean again."""
    ds = _scene_handle(scene, device)
    N.check(N.lib().vr_stream_check_error(ds.handle, C.c_void_p(stream_ptr or 0)))


def resolve_state(state):
    """Mean XYZ [pixels, 3] of flat state records (accumulation_buffer.rs:59)."""
    s = np.ascontiguousarray(np.asarray(state, dtype=np.float64).reshape(-1))
    n = R.pixels(s)
    out = np.zeros((n, 3))
    N.check(N.lib().vr_resolve_state(s.ctypes.data_as(C.c_void_p), n, out.ctypes.data_as(C.c_void_p)))
    return out


class ImageRgbU8:
    """image.rs:8-66: 8-bit RGB pixels, row-major [height][width][3]."""

    def __init__(self, data):
        self.data = np.ascontiguousarray(data, dtype=np.uint8)
        assert self.data.ndim == 3 and self.data.shape[2] == 3

    @staticmethod
    def new(width, height):
        return ImageRgbU8(np.zeros((height, width, 3), dtype=np.uint8))

    def get_width(self):
        return self.data.shape[1]

    def get_height(self):
        return self.data.shape[0]

    def get_colour(self, row, column):
        return tuple(int(v) for v in self.data[row, column])

    def get_pixel_data(self):
        return self.data.tobytes()

    def write_png(self, path):
        N.check(N.lib().vr_write_png(str(path).encode(), self.data.ctypes.data_as(C.c_void_p), self.get_width(),
                                     self.get_height()))


def tone_map_device(state_ptr, pixel_count, rgb_ptr, stream_ptr=None, device=0):
    """Device records (vanrijn_amd/records.py) -> device RGB bytes (3 per pixel), on a stream."""
    N.check(N.lib().vr_tone_map_device(C.c_void_p(state_ptr), pixel_count, C.c_void_p(rgb_ptr), device,
                                       C.c_void_p(stream_ptr or 0)))
