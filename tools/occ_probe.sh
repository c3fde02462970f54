cd $GRAFT_REPO_ROOT
for pad in ${GZ_PADS:-0 4000 8000}; do
  GZ_BZ_LDS_PAD=$pad timeout -k 10 120 python - <<'PY'
import os, sys, json
sys.path.insert(0, "guetzli-cuda-opencl_amd/python")
import guetzli_amd as gz
import numpy as np
w, h = 1920, 1080
rgb = gz.synthetic_frame(0, w, h)
orig = gz.rgb_to_coeffs(rgb, w, h).reshape(3, -1, 64).astype(np.int32)
q = np.array([[1 + (k % 9) for k in range(64)]] * 3)[:, None, :]
r = np.fmod(orig, q)
cur = (orig + np.where(2 * r > q, q - r, np.where(-2 * r > q, -q - r, -r))).astype(np.int16)
cmp = gz.ButteraugliComparator(w, h, rgb, 1.0)
cmp.compare(cur.reshape(-1))
gz.profile_reset(); gz.profile_enable(True)
for _ in range(3):
    cmp.block_zeroing_orders(cur.reshape(-1), orig.astype(np.int16).reshape(-1), 1.0)
gz.profile_enable(False)
p = gz.profile_read()
print("pad", os.environ["GZ_BZ_LDS_PAD"], "zeroing ms", p["block_zeroing"][1] / p["block_zeroing"][0])
PY
done
