"""JPEG input: guetzli::Process on a JPEG file (processor.cc:1029-1066).

The reader (ReadJpeg, jpeg_data_reader.cc) and the 4:4:4 decode
(DecodeJpegToRGB, jpeg_data_decoder.cc:45-55) are host code, checked on the
CPU against the reference's own answers on the committed inputs
(tests/golden/jpeg/, made by tests/golden/make_jpeg_fixtures.py: baseline,
optimized-Huffman with restart markers, progressive, 4:2:0, a guetzli
output): sha256 of the quantized coefficients and of the decoded RGB.  The
encode itself runs on the GPU and must reproduce the reference's bytes.
"""
import hashlib
import json
import os

import pytest

import guetzli_amd as gz

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = json.load(open(os.path.join(GOLDEN, "manifest.json")))["jpeg"]


def _data(name):
    return open(os.path.join(GOLDEN, CASES[name]["input"]), "rb").read()


def _sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("name", sorted(CASES))
def test_read_and_decode_match_reference(name):
    e = CASES[name]
    data = _data(name)
    assert _sha(data) == e["input_sha256"]
    w, h, nc, coeffs, rgb = gz.jpeg_decode(data)
    assert (w, h, nc) == (e["w"], e["h"], e.get("ncomp", 3))
    assert _sha(coeffs.tobytes()) == e["coeffs_sha256"]
    # (4:2:0 via the fancy upsampler; a one-component file decodes to no RGB,
    # as DecodeJpegToRGB returns an empty vector)
    assert _sha(b"" if rgb is None else rgb.tobytes()) == e["rgb_sha256"]


def test_progressive_input_decodes_ac_coefficients():
    # the progressive file's AC bands come from first + refinement scans
    w, h, _, co, rgb = gz.jpeg_decode(_data("synth_pil_q85_444_prog"))
    assert rgb.shape == (h, w, 3)
    assert (co.reshape(3, -1, 64)[:, :, 1:] != 0).any()


@pytest.mark.parametrize("bad", [b"", b"\xff\xd8", b"not a jpeg at all",
                                 "truncated", "no_eoi_scan"])
def test_reader_rejects_invalid_input(bad):
    if bad == "truncated":
        bad = _data("bees_pil_q90_444")[:600]
    elif bad == "no_eoi_scan":
        d = _data("tiny_pil_q85_444")
        bad = d[:d.index(b"\xff\xda")]  # headers only
    with pytest.raises(gz.GuetzliError) as ei:
        gz.jpeg_decode(bad)
    assert ei.value.status == 1  # GZ_ERR_INVALID_ARG


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(n for n in CASES if CASES[n]["reference_ok"]))
def test_process_jpeg_matches_reference(name):
    e = CASES[name]
    assert e["reference_ok"]
    params = gz.Params.for_quality(e["quality"], clear_metadata=e.get("clear_metadata", True))
    out, st = gz.process_jpeg(_data(name), params, return_stats=True)
    assert st.iterations == e["iters"]
    assert len(out) == e["bytes"]
    assert _sha(out) == e["sha256"]


@pytest.mark.gpu
def test_process_jpeg_one_component_rejected_as_reference():
    """A one-component (grayscale) JPEG: the reference's Process returns
    false (ProcessJpegData accepts only 3-component YCbCr input), and so does
    this build -- with an error, not an encode."""
    assert not CASES["gray1_pil_q85"]["reference_ok"]
    with pytest.raises(gz.GuetzliError):
        gz.process_jpeg(_data("gray1_pil_q85"), gz.Params.for_quality(95))


@pytest.mark.gpu
def test_process_jpeg_rejects_garbage():
    with pytest.raises(gz.GuetzliError) as ei:
        gz.process_jpeg(b"\xff\xd8\xff\xe0garbage", gz.Params.for_quality(95))
    assert ei.value.status == 1


def test_oversized_sof_rejected_before_allocation():
    """A ~20-byte file whose SOF declares 65535 x 65535 (67 M blocks per
    component) is JPEG_IMAGE_TOO_LARGE in the reference (more than 2^21
    blocks, jpeg_data_reader.cc:151-158): refused with INVALID_ARG before
    any coefficient memory is allocated."""
    import resource
    sof = bytes([0xFF, 0xC0, 0x00, 0x11, 0x08, 0xFF, 0xFF, 0xFF, 0xFF, 0x03,
                 0x01, 0x11, 0x00, 0x02, 0x11, 0x00, 0x03, 0x11, 0x00])
    data = b"\xff\xd8" + sof + b"\xff\xd9"
    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    with pytest.raises(gz.GuetzliError) as e:
        gz.jpeg_decode(data)
    assert e.value.status == gz.GZ_ERR_INVALID_ARG
    assert "too large" in str(e.value)
    # no multi-GB allocation happened on the way (max RSS grew < 64 MB)
    assert resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - rss0 < 64 * 1024
