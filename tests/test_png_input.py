"""PNG input: gz_png_decode against the reference
CLI's own reader.  The fixtures (tests/golden/png/, made by
tests/golden/make_png_fixtures.py) cover every colour type and bit depth,
Adam7 interlacing, tRNS colour keys and palette alphas, several IDAT chunks,
stored deflate blocks, 1-pixel images and damaged files; their expected RGB
is what the reference's ReadPNG (guetzli.cc:51-156, libpng; oracle/_ref/
png_driver) returned for them."""
import hashlib
import json
import os

import pytest

from oracle_lib import GOLDEN

MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
PNG = MANIFEST["png"]


@pytest.mark.parametrize("name", sorted(PNG))
def test_png_decode_matches_reference_reader(gz, name):
    e = PNG[name]
    data = open(os.path.join(GOLDEN, e["file"]), "rb").read()
    if e.get("fail"):
        with pytest.raises(gz.GuetzliError):
            gz.png_decode(data)
        return
    w, h, rgb = gz.png_decode(data)
    assert (w, h) == (e["w"], e["h"])
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == e["rgb_sha256"]


def test_png_decode_rejects_non_png(gz):
    with pytest.raises(gz.GuetzliError):
        gz.png_decode(b"\xff\xd8\xff\xe0not a png at all")


def test_bees_png_is_the_golden_rgb(gz):
    """bees.png (the reference's test image) decodes to tests/golden/bees.rgb,
    the RGB every bees known answer starts from."""
    w, h, rgb = gz.png_decode(open(os.path.join(GOLDEN, "png", "bees.png"), "rb").read())
    ref = open(os.path.join(GOLDEN, "bees.rgb"), "rb").read()
    assert (w, h) == (444, 258) and rgb.tobytes() == ref


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["bees_q95", "bees_q84"])
def test_png_file_encode_reproduces_reference(gz, name):
    """The CLI path `guetzli --c --quality Q bees.png out.jpg` (guetzli.cc:
    322-343): PNG file in, the reference's JPEG bytes out."""
    e = MANIFEST["e2e"][name]
    data = open(os.path.join(GOLDEN, "png", "bees.png"), "rb").read()
    out, st = gz.process_file(data, gz.Params.for_quality(e["quality"]), return_stats=True)
    assert st.iterations == e["iters"]
    assert hashlib.sha256(out).hexdigest() == e["sha256"]


def _png_chunk(kind, data):
    import struct
    import zlib
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


@pytest.mark.parametrize("w,h,depth,ctype", [(1000000, 1000000, 16, 6), (60000, 60000, 8, 2)])
def test_png_decode_rejects_huge_header_with_tiny_data(gz, w, h, depth, ctype):
    """A header promising far more pixels than its compressed data can hold
    (deflate expands at most 1032:1) fails before anything of that size is
    allocated -- the 'not enough image data' outcome libpng gives the
    reference's ReadPNG -- instead of an allocation of ~8e12 bytes or an
    exception crossing the C ABI."""
    import struct
    import zlib
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0)
    data = (b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", ihdr) +
            _png_chunk(b"IDAT", zlib.compress(b"\x00" * 64)) + _png_chunk(b"IEND", b""))
    with pytest.raises(gz.GuetzliError):
        gz.png_decode(data)
