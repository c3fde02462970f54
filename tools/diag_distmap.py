"""Diagnostic: where does the GPU distance map differ from the fixture?"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import guetzli_amd as gz
from oracle_lib import Fixture
for case in sys.argv[1:] or ["tex_41x33", "tex_100x77"]:
    F = Fixture(case)
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    st = cmp.compare_stages(F.i16("cand_coeffs.i16"))
    a = st["distmap"].reshape(F.h, F.w)
    b = F.f32("distmap.f32").reshape(F.h, F.w)
    bad = np.argwhere(a.view(np.uint32) != b.view(np.uint32))
    print(case, F.w, F.h, "mismatches", len(bad))
    ys = sorted(set(bad[:, 0])); xs = sorted(set(bad[:, 1]))
    print(" rows", ys)
    print(" cols", xs)
    for y, x in bad[:12]:
        print("  (%d,%d) gpu %.9g ref %.9g" % (y, x, a[y, x], b[y, x]))
    c = st["combined"]; print(" combined equal:", np.array_equal(c.view(np.uint32), F.f32("combined.f32").view(np.uint32)))
