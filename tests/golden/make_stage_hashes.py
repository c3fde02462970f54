#!/usr/bin/env python3
"""Butteraugli intermediates of the reference (`--c`, oracle/_ref) at the
BASELINE frame sizes, as sha256 of each stage plane: configs[1] (1920x1080,
seed 0) and configs[2] (3840x2160, seed 0) from the product's synthetic
generator, the stage candidate of oracle/ref_driver.cc (EncodeRGBToJpeg, the
q = 1 coefficients globally quantized by MakeQ(qseed)).  The planes are
tens of MB each, so only their hashes are committed; tests/test_gpu.py
(test_compare_stages_at_frame_size) hashes the device's planes the same way.
Build container only; writes tests/golden/manifest.json["stage_hashes"].

  python tests/golden/make_stage_hashes.py [name ...]
"""
import fcntl
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
import guetzli_amd  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "guetzli_ref")
CASES = {
    "synth_1920x1080_s0": (0, 1920, 1080, 5),
    "synth_3840x2160_s0": (0, 3840, 2160, 6),
}
# the planes tests/test_gpu.py compares (STAGES; file names of ref_driver's dump)
FILES = {"cand_coeffs": "cand_coeffs.i16", "cand_linear": "cand_linear.f32", "cand_xyb": "cand_xyb.f32",
         "mhic0": "mhic0.f32", "mhic1": "mhic1.f32", "edge": "edge.f32", "block_dc": "block_dc.f32",
         "block_ac": "block_ac.f32", "block_ac_lf": "block_ac_lf.f32", "mask": "mask.f32",
         "mask_dc": "mask_dc.f32", "combined": "combined.f32", "distmap": "distmap.f32"}


def main():
    names = sys.argv[1:] or list(CASES)
    path = os.path.join(HERE, "manifest.json")
    for name in names:
        seed, w, h, qseed = CASES[name]
        rgb = guetzli_amd.synthetic_frame(seed, w, h).tobytes()
        tmp = tempfile.mkdtemp(prefix="gz_stage_")
        try:
            inp = os.path.join(tmp, "in.rgb")
            open(inp, "wb").write(rgb)
            subprocess.run([REF, "stages", inp, str(w), str(h), str(qseed), tmp, "nozero"], check=True)
            meta = dict(line.split() for line in open(os.path.join(tmp, "meta.txt")) if line.strip())
            entry = {"seed": seed, "w": w, "h": h, "qseed": qseed,
                     "input_sha256": hashlib.sha256(rgb).hexdigest(),
                     "distance": float(meta["distance"]), "target": float(meta["target"]),
                     "sha256": {k: hashlib.sha256(open(os.path.join(tmp, f), "rb").read()).hexdigest()
                                for k, f in FILES.items()}}
        finally:
            shutil.rmtree(tmp)
        with open(path + ".lock", "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            manifest = json.load(open(path))
            manifest.setdefault("stage_hashes", {})[name] = entry
            json.dump(manifest, open(path, "w"), indent=1, sort_keys=True)
        print(name, entry["distance"], flush=True)


if __name__ == "__main__":
    main()
