#!/usr/bin/env python3
"""JPEG-input fixtures: input JPEG files and the reference's answers on them
(guetzli::Process(params, stats, jpeg, out), processor.cc:1029-1066, `--c`
mode, through oracle/_ref/guetzli_ref).  Build container only (needs PIL to
make the inputs and the reference build); writes tests/golden/jpeg/*.jpg and
tests/golden/manifest.json["jpeg"].

  python tests/golden/make_jpeg_fixtures.py

Per input: sha256 of the reference decoder's RGB (DecodeJpegToRGB) and of its
quantized coefficients (ReadJpeg), and the encode's bytes sha256 + iteration
count at the given quality (or "reference_ok": false if the reference
rejects it).
"""
import hashlib
import io
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
import guetzli_amd  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "guetzli_ref")
OUT_DIR = os.path.join(HERE, "jpeg")


def pil_jpeg(rgb, **kw):
    buf = io.BytesIO()
    Image.fromarray(rgb).save(buf, "JPEG", **kw)
    return buf.getvalue()


def inputs():
    bees = np.fromfile(os.path.join(HERE, "bees.rgb"), np.uint8).reshape(258, 444, 3)
    synth = guetzli_amd.synthetic_frame(5, 160, 120)
    tiny = guetzli_amd.synthetic_frame(6, 40, 36)
    out = {
        # baseline 4:4:4, standard Huffman tables
        "bees_pil_q90_444": (pil_jpeg(bees, quality=90, subsampling=0), 95),
        # optimized Huffman tables, restart markers every 4 MCUs
        "synth_pil_q80_444_rst": (pil_jpeg(synth, quality=80, subsampling=0, optimize=True,
                                           restart_marker_blocks=4), 90),
        # above the 32-pixel Butteraugli minimum only just
        "tiny_pil_q85_444": (pil_jpeg(tiny, quality=85, subsampling=0), 95),
        # 4:2:0 and progressive: the reference handles them, this build does not
        "synth_pil_q85_420": (pil_jpeg(synth, quality=85, subsampling=2), 95),
        "synth_pil_q85_444_prog": (pil_jpeg(synth, quality=85, subsampling=0, progressive=True), 95),
        # APP1 (Exif) + COM segments, encoded with clear_metadata = false
        # (the input's APPn / COM are carried to the output)
        "synth_pil_q85_444_meta": (pil_jpeg(synth, quality=85, subsampling=0,
                                            exif=b"Exif\x00\x00MM\x00*\x00\x00\x00\x08\x00\x00",
                                            comment=b"guetzli-mi355x fixture"), 95),
    }
    # gray content in three components (R = G = B): a 4:4:4 YCbCr input the
    # reference encodes (its chroma planes carry only rounding noise); and a
    # one-component grayscale file, which the reference's ProcessJpegData
    # rejects (processor.cc:946-949: only 3-component YCbCr input)
    gray = np.repeat(bees[:120, :160, 1:2], 3, axis=2)
    out["graycontent_pil_q85_444"] = (pil_jpeg(np.ascontiguousarray(gray), quality=85,
                                               subsampling=0), 95)
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(bees[:120, :160, 1])).save(buf, "JPEG", quality=85)
    out["gray1_pil_q85"] = (buf.getvalue(), 95)
    # 4:2:0 with all-zero chroma (YCbCr given directly: Cb = Cr = 128, no
    # colour conversion, so every chroma coefficient is 0): the reference
    # keeps one component and searches Y alone (processor.cc:990-1016)
    ycc = np.zeros((120, 160, 3), np.uint8)
    ycc[..., 0] = bees[:120, :160, 1]
    ycc[..., 1:] = 128
    buf = io.BytesIO()
    Image.fromarray(ycc, mode="YCbCr").save(buf, "JPEG", quality=85, subsampling=2)
    out["gray420_pil_q85"] = (buf.getvalue(), 95)
    # a guetzli output as input (SOF1, guetzli's own table layout)
    tmp = tempfile.mkdtemp()
    raw = os.path.join(tmp, "bees88.rgb")
    np.ascontiguousarray(bees[:64, :88]).tofile(raw)
    jp = os.path.join(tmp, "bees88.jpg")
    subprocess.run([REF, "encode", raw, "88", "64", "90", jp], check=True, capture_output=True)
    out["bees88_guetzli_q90"] = (open(jp, "rb").read(), 95)
    return out


def main():
    os.makedirs(OUT_DIR, exist_ok=True)
    man_path = os.path.join(HERE, "manifest.json")
    man = json.load(open(man_path))
    entries = {}
    tmp = tempfile.mkdtemp()
    for name, (data, quality) in sorted(inputs().items()):
        path = os.path.join(OUT_DIR, name + ".jpg")
        open(path, "wb").write(data)
        e = {"input": "jpeg/%s.jpg" % name, "quality": quality,
             "input_sha256": hashlib.sha256(data).hexdigest()}
        rgb_p, co_p = os.path.join(tmp, "d.rgb"), os.path.join(tmp, "d.co")
        r = subprocess.run([REF, "decode", path, rgb_p, co_p], capture_output=True, text=True)
        if r.returncode == 0:
            info = json.loads(r.stdout)
            e.update(w=info["w"], h=info["h"], ncomp=info["ncomp"],
                     rgb_sha256=hashlib.sha256(open(rgb_p, "rb").read()).hexdigest(),
                     coeffs_sha256=hashlib.sha256(open(co_p, "rb").read()).hexdigest())
        out_p = os.path.join(tmp, "o.jpg")
        keep = name.endswith("_meta")
        if keep:
            e["clear_metadata"] = False
        r = subprocess.run([REF, "encode_jpeg", path, str(quality), out_p] + (["keep"] if keep else []),
                           capture_output=True, text=True)
        e["reference_ok"] = r.returncode == 0
        if r.returncode == 0:
            info = json.loads(r.stdout)
            e.update(sha256=hashlib.sha256(open(out_p, "rb").read()).hexdigest(),
                     bytes=info["bytes"], iters=info["iters"])
        entries[name] = e
        print(name, json.dumps(e))
    man["jpeg"] = entries
    json.dump(man, open(man_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
