#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ from the REFERENCE.

Runs only in the build container (needs oracle/_ref, i.e. `make -C oracle`
with /root/reference present).  The outputs are data (inputs + the
reference's outputs) and are committed; nothing here ships to the GPU box
except those files.

  stages_<case>/   stage-level dumps of the reference `--c` path for a small
                   image (oracle/ref_driver.cc `stages`): reference/candidate
                   XYB, MHIC planes, edge / block-diff / low-freq / mask /
                   combined maps, distmap, block weights, per-block zeroing
                   orders (+ zero_order_la*_m*_nm*.bin: lookahead / comp_mask /
                   zeroing-model variants).
  manifest.json    end-to-end known answers: sha256 / size / iterations of
                   `guetzli --c` on bees.png and on synthetic frames.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref", "guetzli_ref")


def texture_image(w, h, seed):
    """Smooth colour field + sinusoids + filtered noise (numpy, seeded)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.zeros((h, w, 3))
    for c in range(3):
        v = 120.0 + 30.0 * rng.uniform(-1, 1)
        for _ in range(3):
            a = rng.uniform(8, 30)
            fx, fy = rng.uniform(0.02, 0.4, size=2)
            v = v + a * np.sin(fx * xx + fy * yy + rng.uniform(0, 6.28))
        noise = rng.normal(0, 10, size=(h, w))
        k = np.array([1, 4, 6, 4, 1], dtype=np.float64) / 16
        noise = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, noise)
        img[:, :, c] = v + noise
    for _ in range(3):
        x0, y0 = rng.integers(0, w - 8), rng.integers(0, h - 8)
        x1, y1 = x0 + rng.integers(4, max(5, w // 3)), y0 + rng.integers(4, max(5, h // 3))
        img[y0:y1, x0:x1, :] = 0.5 * img[y0:y1, x0:x1, :] + 0.5 * rng.uniform(40, 220, size=3)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def flat_image(w, h, seed):
    rng = np.random.default_rng(seed)
    base = rng.uniform(60, 200, size=3)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = base[None, None, :] + 0.05 * xx[:, :, None] + 0.03 * yy[:, :, None]
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def bees_crop(x0, y0, w, h):
    bees = np.fromfile(os.path.join(HERE, "bees.rgb"), dtype=np.uint8).reshape(258, 444, 3)
    return np.ascontiguousarray(bees[y0:y0 + h, x0:x0 + w])


STAGE_CASES = [
    # name, image factory, qseed
    ("tex_64x48", lambda: texture_image(64, 48, 1), 1),
    ("tex_100x77", lambda: texture_image(100, 77, 2), 2),
    ("tex_41x33", lambda: texture_image(41, 33, 3), 3),
    ("bees_88x64", lambda: bees_crop(200, 100, 88, 64), 4),
    ("flat_48x40", lambda: flat_image(48, 40, 5), 5),
]


def sha256(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def run_stages():
    for name, make, qseed in STAGE_CASES:
        img = make()
        h, w, _ = img.shape
        d = os.path.join(HERE, "stages_" + name)
        os.makedirs(d, exist_ok=True)
        rgb = os.path.join(d, "input.rgb")
        img.tofile(rgb)
        subprocess.run([REF, "stages", rgb, str(w), str(h), str(qseed), d], check=True)
        print("stages", name, w, h)


def run_zero_variants():
    """zero_order_la<L>_m<M>_nm<N>.bin next to each stage fixture: the
    per-block zeroing orders for lookahead 1/2, comp_mask 1/6 and the old
    zeroing model (oracle/ref_driver.cc ZeroVariants)."""
    for name, _, qseed in STAGE_CASES:
        d = os.path.join(HERE, "stages_" + name)
        meta = dict(l.split() for l in open(os.path.join(d, "meta.txt")) if len(l.split()) == 2)
        subprocess.run([REF, "zero_variants", os.path.join(d, "input.rgb"), meta["w"], meta["h"],
                        str(qseed), d], check=True)
        print("zero variants", name)


def run_e2e(manifest, cases, section="e2e"):
    """cases: (name, rgb path, w, h, quality[, {Params overrides}]).  A case
    whose reference run returns false (guetzli::Process, exit status 3 of the
    driver) is recorded as {"fail": true}."""
    out = manifest.setdefault(section, {})
    for case in cases:
        name, rgb, w, h, q = case[:5]
        params = case[5] if len(case) > 5 else {}
        jpg = "/tmp/gz_fixture_%s.jpg" % name
        res = subprocess.run([REF, "encode", rgb, str(w), str(h), str(q), jpg, "c"] +
                             ["%s=%d" % kv for kv in sorted(params.items())],
                             capture_output=True, text=True)
        if res.returncode == 3:
            out[name] = {"w": w, "h": h, "quality": q, "fail": True,
                         "input": os.path.relpath(rgb, HERE) if rgb.startswith(HERE) else rgb}
            if params:
                out[name]["params"] = params
            print(section, name, out[name])
            continue
        res.check_returncode()
        info = json.loads(res.stdout)
        out[name] = {"w": w, "h": h, "quality": q, "sha256": sha256(jpg), "bytes": info["bytes"],
                     "iters": info["iters"], "ref_seconds": info["seconds"],
                     "input": os.path.relpath(rgb, HERE) if rgb.startswith(HERE) else rgb}
        if params:
            out[name]["params"] = params
        print(section, name, out[name])


def main():
    manifest_path = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(manifest_path)) if os.path.exists(manifest_path) else {}
    what = sys.argv[1:] or ["stages", "e2e-small"]
    if "stages" in what:
        run_stages()
    if "stages" in what or "zero-variants" in what:
        run_zero_variants()
    if "e2e-small" in what:
        cases = [("bees_q95", os.path.join(HERE, "bees.rgb"), 444, 258, 95)]
        for name, _, _ in STAGE_CASES:
            d = os.path.join(HERE, "stages_" + name)
            meta = dict(l.split() for l in open(os.path.join(d, "meta.txt")) if len(l.split()) == 2)
            cases.append(("%s_q95" % name, os.path.join(d, "input.rgb"), int(meta["w"]),
                          int(meta["h"]), 95))
        cases.append(("bees_q90", os.path.join(HERE, "bees.rgb"), 444, 258, 90))
        cases.append(("bees_q84", os.path.join(HERE, "bees.rgb"), 444, 258, 84))
        run_e2e(manifest, cases)
    if "e2e-params" in what:
        # Params variants: old zeroing model, lookahead 1 / 2 (processor.cc:400-405, :416)
        bees = os.path.join(HERE, "bees.rgb")
        tex = os.path.join(HERE, "stages_tex_100x77", "input.rgb")
        run_e2e(manifest, [
            ("bees_q95_oldmodel", bees, 444, 258, 95, {"new_model": 0}),
            ("bees_q90_lookahead1", bees, 444, 258, 90, {"lookahead": 1}),
            ("tex_100x77_q95_oldmodel", tex, 100, 77, 95, {"new_model": 0}),
            ("tex_100x77_q95_lookahead2", tex, 100, 77, 95, {"lookahead": 2}),
        ], section="e2e_params")
    if "e2e-params-la" in what:
        # lookahead above 3 (the 4:4:4 search evaluates a step's candidates in
        # batches of three: 4 is a full batch and a short one, 7 three batches)
        tex = os.path.join(HERE, "stages_tex_100x77", "input.rgb")
        run_e2e(manifest, [("tex_100x77_q95_lookahead4", tex, 100, 77, 95, {"lookahead": 4}),
                           ("tex_100x77_q90_lookahead7", tex, 100, 77, 90, {"lookahead": 7})],
                section="e2e_params")
    if "e2e-420" in what:
        # the 4:2:0 pass (Params::try_420 / force_420 / use_silver_screen,
        # processor.cc:986-1016): downsampled search alone, both passes, the
        # silver-screen downsampler, odd sizes (partial 16x16 chroma blocks)
        bees = os.path.join(HERE, "bees.rgb")

        def stage(name):
            d = os.path.join(HERE, "stages_" + name)
            meta = dict(l.split() for l in open(os.path.join(d, "meta.txt")) if len(l.split()) == 2)
            return os.path.join(d, "input.rgb"), int(meta["w"]), int(meta["h"])

        cases = [("bees_q95_force420", bees, 444, 258, 95, {"force_420": 1}),
                 ("bees_q90_try420", bees, 444, 258, 90, {"try_420": 1}),
                 ("bees_q95_force420_silver", bees, 444, 258, 95, {"force_420": 1, "silver": 1})]
        for name, q, params in [("tex_64x48", 95, {"force_420": 1}), ("tex_100x77", 95, {"force_420": 1}),
                                ("tex_41x33", 95, {"force_420": 1}), ("bees_88x64", 95, {"try_420": 1}),
                                ("tex_100x77", 90, {"force_420": 1, "new_model": 0}),
                                ("tex_64x48", 95, {"force_420": 1, "lookahead": 1})]:
            rgb, w, h = stage(name)
            tag = "_".join("%s%d" % kv for kv in sorted(params.items()) if kv[0] not in ("force_420", "try_420"))
            cases.append(("%s_q%d_%s%s" % (name, q, "try420" if "try_420" in params else "force420",
                                           "_" + tag if tag else ""), rgb, w, h, q, params))
        run_e2e(manifest, cases, section="e2e_420")
    if "e2e-420-la" in what:
        # lookahead other than 3 in the 4:2:0 chroma search (k_block_zeroing420
        # evaluates a step's candidates three at a time: 2 is one short group,
        # 4 and 5 a full group and a short one)
        cases = []
        for name, q, la in [("tex_64x48", 95, 2), ("tex_64x48", 95, 4), ("tex_100x77", 95, 5)]:
            d = os.path.join(HERE, "stages_" + name)
            meta = dict(l.split() for l in open(os.path.join(d, "meta.txt")) if len(l.split()) == 2)
            cases.append(("%s_q%d_force420_lookahead%d" % (name, q, la), os.path.join(d, "input.rgb"),
                          int(meta["w"]), int(meta["h"]), q, {"force_420": 1, "lookahead": la}))
        run_e2e(manifest, cases, section="e2e_420")
    if "e2e-edge" in what:
        # the reference's edge paths (processor.cc):
        #  - images under 32 px in either dimension: no comparator, the q=1
        #    encode is the output (:1170-1181 -> :971-977);
        #  - quality below 84 (target above 2.0): Process returns false (:939-945);
        #  - force_420 on content whose chroma is all zero: Downsample leaves
        #    the image at 4:4:4 (output_image.cc:535-539), SaveToJpegData keeps
        #    one component, and the pass runs the downsampling quantization
        #    generator with comp_mask 1 and ymul 1.0 (:991-1016);
        #  - try_420 on such content: IsGrayscale skips the 4:2:0 pass (:986-988).
        d = os.path.join(HERE, "edge")
        os.makedirs(d, exist_ok=True)

        def save(name, img):
            path = os.path.join(d, name + ".rgb")
            np.ascontiguousarray(img).tofile(path)
            h, w, _ = img.shape
            return path, w, h

        def gray(img):
            g = img[:, :, 1:2]
            return np.repeat(g, 3, axis=2)

        cases = []
        for name, (w, h), seed in [("tex_24x24", (24, 24), 21), ("tex_300x20", (300, 20), 22),
                                   ("tex_20x300", (20, 300), 23), ("tex_31x64", (31, 64), 24),
                                   ("tex_1x1", (1, 1), 25)]:
            path, w, h = save(name, texture_image(w, h, seed) if w * h > 1 else
                              np.full((1, 1, 3), 77, np.uint8))
            cases.append(("%s_q95" % name, path, w, h, 95))
        tex = save("tex_64x48", texture_image(64, 48, 26))
        cases.append(("tex_64x48_q80", tex[0], tex[1], tex[2], 80))
        small = os.path.join(d, "tex_24x24.rgb")
        cases.append(("tex_24x24_q83", small, 24, 24, 83))
        g1 = save("gray_96x64", gray(texture_image(96, 64, 27)))
        g2 = save("gray_bees_88x64", gray(bees_crop(120, 60, 88, 64)))
        cases += [("gray_96x64_q95_force420", g1[0], g1[1], g1[2], 95, {"force_420": 1}),
                  ("gray_96x64_q90_force420", g1[0], g1[1], g1[2], 90, {"force_420": 1}),
                  ("gray_bees_88x64_q95_force420", g2[0], g2[1], g2[2], 95, {"force_420": 1}),
                  ("gray_96x64_q95_try420", g1[0], g1[1], g1[2], 95, {"try_420": 1}),
                  ("gray_bees_88x64_q95", g2[0], g2[1], g2[2], 95)]
        run_e2e(manifest, cases, section="e2e_edge")
    if "e2e-420-1080" in what:
        # the 4:2:0 pass at full size: synthetic 1920x1080 seed 0 (the bench's
        # frame), q95, force_420 -- about 7 minutes of reference CPU time
        sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
        import guetzli_amd as gz
        rgb = "/tmp/gz_fixture_synth_1080_s0.rgb"
        gz.synthetic_frame(0, 1920, 1080).tofile(rgb)
        run_e2e(manifest, [("synth_1920x1080_s0_q95_force420", rgb, 1920, 1080, 95, {"force_420": 1})],
                section="e2e_420")
        manifest["e2e_420"]["synth_1920x1080_s0_q95_force420"]["input"] = "synthetic:0"
    if "e2e-420-synth" in what:
        # the 4:2:0 pass on a frame off the 16-pixel grid (partial chroma
        # blocks on both edges): synthetic 1366x768 seed 5, q90, force_420
        sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
        import guetzli_amd as gz
        rgb = "/tmp/gz_fixture_synth_1366x768_s5.rgb"
        gz.synthetic_frame(5, 1366, 768).tofile(rgb)
        run_e2e(manifest, [("synth_1366x768_s5_q90_force420", rgb, 1366, 768, 90, {"force_420": 1})],
                section="e2e_420")
        manifest["e2e_420"]["synth_1366x768_s5_q90_force420"]["input"] = "synthetic:5"
    json.dump(manifest, open(manifest_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
