"""Display end of the path: ClampingToneMapper over ColourXyz::to_srgb and ImageRgbU8::write_png.

Reference: src/image.rs:52-66 (write_png), :110-128 (NormalizedAsByte), :141-187 (ClampingToneMapper),
src/colour/colour_xyz.rs:49-84 (to_linear_rgb, to_srgb, srgb_gamma with 12.98 / 1.005),
src/accumulation_buffer.rs:38-42 (to_image_rgb_u8).

CPU tests: the oracle's tone map against the reference's own tone-mapper and byte-conversion tests
(restated through XYZ inputs), against an independent numpy restatement, and the PNG writer
(host-only code in the library) round-tripped through zlib.  GPU tests: the device tone map (from
device records and from a host colour buffer) against the oracle, byte for byte.  pow() is glibc's
on the oracle side and ocml's on the GPU; they may differ by 1 ulp, which changes a byte only for a
value within ~1e-16 of a k/255 boundary (never observed).
"""
import struct
import zlib

import numpy as np
import pytest

from vanrijn_amd import scenes
from vanrijn_amd.render import AccumulationBuffer, ImageRgbU8, Tile, render_tile, resolve_state

XYZ_TO_RGB = [(3.24096994, -1.53738318, -0.49861076), (-0.96924364, 1.87596750, 0.04155506),
              (0.05563008, -0.20397696, 1.05697151)]


def numpy_tone_map(xyz):
    """Independent restatement (numpy float64, same operation order, libm pow)."""
    xyz = np.asarray(xyz, dtype=np.float64)
    out = np.zeros(xyz.shape, dtype=np.uint8)
    for k, (a, b, c) in enumerate(XYZ_TO_RGB):
        lin = ((-0.0 + a * xyz[..., 0]) + b * xyz[..., 1]) + c * xyz[..., 2]
        with np.errstate(invalid="ignore"):
            g = np.where(lin <= 0.0031308, 12.98 * lin, 1.005 * np.power(np.maximum(lin, 0.0), 1.0 / 2.4) - 0.055)
        g = np.where(np.isnan(lin), np.nan, g)
        c01 = np.clip(g, 0.0, 1.0)
        out[..., k] = np.where(np.isnan(c01), 0, np.floor(np.nan_to_num(c01) * 255.0)).astype(np.uint8)
    return out


def test_tone_map_reference_byte_tests(oracle):
    # image.rs:229-277 (normalized_to_byte) and :279-352 (clamping tone mapper), through XYZ:
    # black stays black; super-saturated channels clamp to 255; linear 1.0 maps through the
    # reference's srgb_gamma (1.005 - 0.055 = 0.95 -> 242), not to 255 as the sRGB standard would
    def via_rgb(rgb):
        return oracle.tone_map(np.array([oracle.xyz_from_linear_rgb(rgb)]))[0].tolist()

    assert via_rgb([0.0, 0.0, 0.0]) == [0, 0, 0]
    assert via_rgb([2.0, 2.0, 2.0]) == [255, 255, 255]
    assert via_rgb([0.0, 2.0, 0.0]) == [0, 255, 0]
    assert via_rgb([1.0, 1.0, 1.0]) == [242, 242, 242]
    assert via_rgb([0.5, 0.0, 0.0])[0] == int(np.floor((1.005 * 0.5 ** (1 / 2.4) - 0.055) * 255.0))
    # NaN (0/0 colour) -> 0, negative -> 0
    assert oracle.tone_map(np.array([[np.nan, 0.0, 0.0]]))[0].tolist() == [0, 0, 0]
    assert oracle.tone_map(np.array([[-1.0, -1.0, -1.0]]))[0].tolist() == [0, 0, 0]


def test_tone_map_oracle_matches_numpy_restatement(oracle):
    rng = np.random.default_rng(7)
    xyz = np.concatenate([rng.uniform(-0.2, 1.5, (20000, 3)), rng.exponential(0.05, (20000, 3)),
                          np.array([[0.0, 0.0, 0.0], [1e300, 1e300, 1e300], [0.0031308 / 3.24, 0.0, 0.0]])])
    assert np.array_equal(oracle.tone_map(xyz), numpy_tone_map(xyz))


def _decode_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, []
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        (crc,) = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert zlib.crc32(typ + body) == crc
        chunks.append((typ, body))
        pos += 12 + n
    assert chunks[0][0] == b"IHDR" and chunks[-1][0] == b"IEND"
    w, h, depth, ctype, comp, filt, interlace = struct.unpack(">IIBBBBB", chunks[0][1])
    assert (depth, ctype, comp, filt, interlace) == (8, 2, 0, 0, 0)
    raw = zlib.decompress(b"".join(b for t, b in chunks if t == b"IDAT"))
    rows = np.frombuffer(raw, dtype=np.uint8).reshape(h, 1 + 3 * w)
    assert np.all(rows[:, 0] == 0)
    return rows[:, 1:].reshape(h, w, 3)


def test_write_png_roundtrip(tmp_path):
    rng = np.random.default_rng(3)
    img = ImageRgbU8(rng.integers(0, 256, (37, 53, 3), dtype=np.uint8))
    path = tmp_path / "out.png"
    img.write_png(path)
    assert np.array_equal(_decode_png(path), img.data)
    # image.rs:197-218: pixel data is row-major RGB
    assert img.get_pixel_data()[3 * (2 * 53 + 5):3 * (2 * 53 + 5) + 3] == bytes(img.data[2, 5])


def test_write_png_rejects_empty_image(tmp_path):
    from vanrijn_amd._native import VrError
    with pytest.raises(VrError):
        ImageRgbU8.new(0, 4).write_png(tmp_path / "x.png")


@pytest.mark.gpu
def test_device_tone_map_matches_oracle(oracle, tmp_path):
    import torch
    from vanrijn_amd.render import render_tile_device, tone_map_device
    s = scenes.main_scene(scenes.procedural_bunny())
    W, H = 160, 120
    state = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    render_tile_device(s, Tile(0, W, 0, H), H, W, 4, 0x5EED0001, 0, state.data_ptr())
    rgb = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
    tone_map_device(state.data_ptr(), H * W, rgb.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    colour = resolve_state(state.cpu().numpy()).reshape(H, W, 3)
    want = oracle.tone_map(colour)
    got = rgb.cpu().numpy().reshape(H, W, 3)
    assert np.array_equal(got, want)
    assert got.max() > 0  # the frame is not black
    # host path (AccumulationBuffer.to_image_rgb_u8) and the PNG of it
    buf = render_tile(s, Tile(0, W, 0, H), H, W, 4, 0x5EED0001)
    img = buf.to_image_rgb_u8()
    assert np.array_equal(img.data, oracle.tone_map(buf.colour_buffer))
    img.write_png(tmp_path / "frame.png")
    assert np.array_equal(_decode_png(tmp_path / "frame.png"), img.data)


@pytest.mark.gpu
def test_tone_map_empty_and_unsampled_pixels():
    buf = AccumulationBuffer(3, 2)  # no update_pixel yet: colour 0 -> black
    assert buf.to_image_rgb_u8().data.tolist() == [[[0, 0, 0]] * 3] * 2
