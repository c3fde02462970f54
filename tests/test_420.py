"""The 4:2:0 pass (Params::try_420 / force_420 / use_silver_screen and 4:2:0
JPEG input; guetzli/processor.cc:986-1016, output_image.cc:124-205,
494-640, preprocess_downsample.cc).

CPU: the host model of the downsampled image -- Downsample, the factor-2
pixel state through CopyFromJpegData / ApplyGlobalQuantization / arbitrary
SetCoeffBlock sequences, SaveToJpegData + WriteJpeg -- against the
reference's own OutputImage, stage by stage (oracle/_ref/image420_check,
built from /root/reference by oracle/Makefile; skipped where it is absent).

GPU: whole encodes against the reference's bytes (tests/golden/manifest.json
"e2e_420", made by tests/golden/make_fixtures.py e2e-420 with
oracle/_ref/guetzli_ref): the Y search with the chroma planes as they are,
the wavefront chroma search (k_block_zeroing420), the back end's
factor-2 bookkeeping, the downsampling quantization generator.
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
CHECK = os.path.join(ROOT, "oracle", "_ref", "image420_check")
E2E = MANIFEST.get("e2e_420", {})


def _crop(tmp_path, w, h, x0, y0):
    bees = np.fromfile(os.path.join(GOLDEN, "bees.rgb"), np.uint8).reshape(258, 444, 3)
    p = tmp_path / ("crop_%dx%d.rgb" % (w, h))
    np.ascontiguousarray(bees[y0:y0 + h, x0:x0 + w]).tofile(p)
    return str(p)


@pytest.mark.skipif(not os.path.exists(CHECK), reason="oracle/_ref/image420_check not built")
@pytest.mark.parametrize("silver", [0, 1])
@pytest.mark.parametrize("size", [(444, 258, 0, 0), (100, 77, 200, 100), (41, 33, 10, 20), (17, 15, 300, 200),
                                  (250, 129, 50, 60)])
def test_host_model_matches_reference_output_image(tmp_path, size, silver):
    w, h, x0, y0 = size
    rgb = os.path.join(GOLDEN, "bees.rgb") if (w, h) == (444, 258) else _crop(tmp_path, w, h, x0, y0)
    r = subprocess.run([CHECK, rgb, str(w), str(h), str(silver), str(w * 7 + h)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok")


def test_known_answers_present():
    # force / try / silver screen / odd sizes / params variants / full size
    assert len(E2E) >= 10
    assert "synth_1920x1080_s0_q95_force420" in E2E
    kinds = {k for e in E2E.values() for k in e["params"]}
    assert {"force_420", "try_420", "silver", "new_model", "lookahead"} <= kinds


def _params(gz, e):
    p = gz.Params.for_quality(e["quality"])
    pr = e["params"]
    p.force_420 = bool(pr.get("force_420", 0))
    p.try_420 = bool(pr.get("try_420", 0))
    p.use_silver_screen = bool(pr.get("silver", 0))
    p.zeroing_greedy_lookahead = pr.get("lookahead", 3)
    p.new_zeroing_model = bool(pr.get("new_model", 1))
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(E2E))
def test_process_420_known_answers(name):
    import guetzli_amd as gz
    e = E2E[name]
    if e["input"].startswith("synthetic:"):
        rgb = gz.synthetic_frame(int(e["input"].split(":")[1]), e["w"], e["h"])
    else:
        rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
    data, st = gz.process(rgb, e["w"], e["h"], _params(gz, e), return_stats=True)
    assert st.iterations == e["iters"]
    assert hashlib.sha256(data).hexdigest() == e["sha256"]

# (4:2:0 JPEG input: tests/test_jpeg_input.py, synth_pil_q85_420)
