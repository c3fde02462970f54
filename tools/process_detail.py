import sys, time, json
sys.path.insert(0, 'guetzli-cuda-opencl_amd/python')
import guetzli_amd as gz
w, h, q = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rgb = gz.synthetic_frame(0, w, h)
t0 = time.time()
d, st = gz.process(rgb, w, h, gz.Params.for_quality(q), return_stats=True)
print(json.dumps({"s": time.time() - t0, "iters": st.iterations, "up": st.iterations_up, "down": st.iterations_down, "backend": st.seconds_backend, "detail": gz.last_process_detail()}))
