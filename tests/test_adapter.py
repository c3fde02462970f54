"""The drop-in adapters (guetzli-cuda-opencl_amd/adapters/) compiled against
the reference's own headers and linked with the reference's own Processor
(oracle/Makefile -> oracle/_ref/adapter_e2e; built where /root/reference is
present, and shipped prebuilt to the GPU box).

* comparator: the reference's unmodified search loop (processor.cc, CPU_OPT
  mode, per-block SwitchBlock / CompareBlock calls) driving
  guetzli::HipButteraugliComparator -- every Compare, CompareBlock and
  distmap() on the GPU -- must reproduce the reference's bytes;
* process: guetzli::ProcessHip (gz_process_rgb) likewise.
Without a GPU both must fail loudly (no CPU fallback)."""
import hashlib
import json
import os
import subprocess

import pytest

from oracle_lib import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "adapter_e2e")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))


def _need_bin():
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/adapter_e2e not built (needs /root/reference at build time)")


def _run(mode, name, tmp_path, timeout=600, section="e2e"):
    e = MANIFEST[section][name]
    out = tmp_path / ("%s_%s.jpg" % (mode, name))
    kv = ["%s=%d" % p for p in sorted(e.get("params", {}).items())]
    r = subprocess.run([BIN, mode, os.path.join(GOLDEN, e["input"]), str(e["w"]), str(e["h"]),
                        str(e["quality"]), str(out)] + kv, capture_output=True, text=True,
                       timeout=timeout)
    return e, out, r


@pytest.mark.parametrize("mode", ["comparator", "process"])
def test_adapters_fail_loudly_without_gpu(gz, mode, tmp_path):
    _need_bin()
    if gz.device_count() > 0:
        pytest.skip("a HIP device is visible")
    e, out, r = _run(mode, "bees_q95", tmp_path, timeout=120)
    assert r.returncode != 0 and not out.exists()
    assert "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode,name", [("comparator", "bees_q95"), ("comparator", "tex_64x48_q95"),
                                       ("process", "bees_q95"), ("process", "bees_q84")])
def test_adapters_reproduce_reference(mode, name, tmp_path):
    _need_bin()
    e, out, r = _run(mode, name, tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["iterations", str(e["iters"])], r.stdout
    assert hashlib.sha256(out.read_bytes()).hexdigest() == e["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode,name", [("comparator", "tex_64x48_q95_force420"),
                                       ("comparator", "tex_41x33_q95_force420"),
                                       ("process", "bees_q90_try420")])
def test_adapters_reproduce_reference_420(mode, name, tmp_path):
    """The 4:2:0 search: in comparator mode the reference's own factor-2
    loop (SwitchBlock(.., 2, 2), CompareBlock at the four luma offsets, the
    stateful SetCoeffBlock on the reference's OutputImage) drives the
    comparator through the sRGB entries (gz_comparator_compare_rgb /
    _compare_blocks_rgb)."""
    _need_bin()
    e, out, r = _run(mode, name, tmp_path, section="e2e_420")
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["iterations", str(e["iters"])], r.stdout
    assert hashlib.sha256(out.read_bytes()).hexdigest() == e["sha256"]
