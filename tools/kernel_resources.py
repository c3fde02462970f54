#!/usr/bin/env python3
"""VGPRs / scratch / occupancy / LDS of every gfx950 kernel in gz_device.hip
(compiler resource-usage remarks; no GPU needed).  The compiler's occupancy
does not see that gfx950 allocates LDS in 1,280-byte granules (a residency
census of k_block_zeroing, tools/zeroing_trace.py: at most 21 workgroups per
CU at 6,616 B = 6 granules, 24 at 6,256 B = 5): wg/CU(lds) is that limit.

  python tools/kernel_resources.py [name-filter]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "guetzli-cuda-opencl_amd", "csrc")


def main():
    flt = sys.argv[1] if len(sys.argv) > 1 else ""
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-I.",
           "-I../../include", "--offload-arch=gfx950", "-fno-gpu-flush-denormals-to-zero",
           "--cuda-device-only", "-c", "kernels/gz_device.hip", "-o", "/tmp/gz_dev_res.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    for r in rows:
        if flt in r["name"]:
            lds = r.get("lds") or 0
            gran = -(-lds // 1280)
            wg_lds = 163840 // (gran * 1280) if gran else "-"
            print("%-70s vgpr %3s scratch %3s occ %2s lds %6s wg/CU(lds) %s" % (
                r["name"][:70], r.get("vgpr"), r.get("scratch"), r.get("occ"), lds, wg_lds))


if __name__ == "__main__":
    main()
