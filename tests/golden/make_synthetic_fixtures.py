#!/usr/bin/env python3
"""Known answers of the reference (`guetzli --c`, oracle/_ref) on synthetic
frames from the product's deterministic generator (gz_synthetic_frame).
Build container only; writes tests/golden/manifest.json["synthetic"].

  python tests/golden/make_synthetic_fixtures.py [name ...]
"""
import fcntl
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
import guetzli_amd  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "guetzli_ref")
CASES = {
    "synth_256x256_s0_q95": (0, 256, 256, 95),
    "synth_640x360_s3_q95": (3, 640, 360, 95),
    "synth_1920x1080_s0_q95": (0, 1920, 1080, 95),
    "synth_1920x1080_s1_q95": (1, 1920, 1080, 95),
    "synth_3840x2160_s0_q90": (0, 3840, 2160, 90),
    # bench.py verifies every timed frame (seeds 0..7 at 1080p q95)
    "synth_1920x1080_s2_q95": (2, 1920, 1080, 95),
    "synth_1920x1080_s3_q95": (3, 1920, 1080, 95),
    "synth_1920x1080_s4_q95": (4, 1920, 1080, 95),
    "synth_1920x1080_s5_q95": (5, 1920, 1080, 95),
    "synth_1920x1080_s6_q95": (6, 1920, 1080, 95),
    "synth_1920x1080_s7_q95": (7, 1920, 1080, 95),
    # configs[4]: ~35 min of reference CPU time, ~7 GB host memory
    "synth_8192x8192_s0_q84": (0, 8192, 8192, 84),
    # other qualities at 1080p, and gray content (R = G = B: the chroma the
    # search sees is all zero, SaveToJpegData keeps one component) through
    # the device bulk prefix and the tracked-histogram coder
    "synth_1920x1080_s0_q90": (0, 1920, 1080, 90),
    "gray_1920x1080_s0_q95": (0, 1920, 1080, 95, "gray"),
    "gray_640x360_s3_q90": (3, 640, 360, 90, "gray"),
    # round 6: configs[2]'s size at the headline quality, and sizes off the
    # 16-pixel grid (partial blocks and MCUs) at other qualities
    "synth_3840x2160_s1_q95": (1, 3840, 2160, 95),
    "synth_2560x1440_s2_q92": (2, 2560, 1440, 92),
    "synth_1366x768_s5_q88": (5, 1366, 768, 88),
    "synth_1283x721_s4_q84": (4, 1283, 721, 84),
}


def case_rgb(seed, w, h, *mode):
    """The case's input: the generator's frame, or its green channel in all
    three (mode "gray")."""
    rgb = guetzli_amd.synthetic_frame(seed, w, h)
    if mode and mode[0] == "gray":
        rgb = rgb.reshape(h, w, 3)[:, :, 1:2].repeat(3, axis=2).reshape(rgb.shape).copy()
    return rgb


def main():
    names = sys.argv[1:] or list(CASES)
    path = os.path.join(HERE, "manifest.json")
    for name in names:
        seed, w, h, q = CASES[name][:4]
        mode = CASES[name][4:]
        rgb = case_rgb(seed, w, h, *mode).tobytes()
        inp = "/tmp/gz_%s.rgb" % name
        open(inp, "wb").write(rgb)
        jpg = "/tmp/gz_%s.jpg" % name
        res = subprocess.run([REF, "encode", inp, str(w), str(h), str(q), jpg, "c"], check=True,
                             capture_output=True, text=True)
        info = json.loads(res.stdout)
        entry = {
            "seed": seed, "w": w, "h": h, "quality": q, **({"mode": mode[0]} if mode else {}),
            "input_sha256": hashlib.sha256(rgb).hexdigest(),
            "sha256": hashlib.sha256(open(jpg, "rb").read()).hexdigest(),
            "bytes": info["bytes"], "iters": info["iters"], "ref_seconds": info["seconds"]}
        os.unlink(inp)
        # several generators may run concurrently: read-modify-write under a lock
        with open(path + ".lock", "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            manifest = json.load(open(path))
            manifest.setdefault("synthetic", {})[name] = entry
            json.dump(manifest, open(path, "w"), indent=1, sort_keys=True)
        manifest["synthetic"][name] = entry
        print(name, manifest["synthetic"][name], flush=True)


if __name__ == "__main__":
    main()
