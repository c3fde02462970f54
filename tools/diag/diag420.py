import faulthandler, sys, time, os, json, hashlib
import numpy as np
faulthandler.dump_traceback_later(50, exit=True)
sys.path.insert(0, "guetzli-cuda-opencl_amd/python")
import guetzli_amd as gz
print("imported", flush=True)
m = json.load(open("tests/golden/manifest.json"))["e2e_420"]
for name in ["tex_41x33_q95_force420", "bees_88x64_q95_try420"]:
    e = m[name]
    rgb = np.fromfile(os.path.join("tests/golden", e["input"]), np.uint8) if not e["input"].startswith("synthetic") else gz.synthetic_frame(int(e["input"].split(":")[1]), e["w"], e["h"])
    p = gz.Params.for_quality(e["quality"]); pr = e["params"]
    p.force_420 = bool(pr.get("force_420", 0)); p.try_420 = bool(pr.get("try_420", 0))
    t0 = time.time()
    print("start", name, flush=True)
    data, st = gz.process(rgb, e["w"], e["h"], p, return_stats=True)
    print(name, time.time() - t0, st.iterations, e["iters"], hashlib.sha256(data).hexdigest() == e["sha256"], flush=True)
