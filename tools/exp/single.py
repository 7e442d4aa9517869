"""Single-frame latency probe (configs[1]): ms per sift_batch_device call of
one device-resident 1920x1080 frame, results kept on the device, plus the
serialised pass's pyramid ms.  Env knobs of the library apply (A/B)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))
import numpy as np, torch
import pkg_loader, synth
pkg = pkg_loader.load()
W, H = int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
n = int(os.environ.get("N", 1))
fr = synth.frames_torch(n, W, H, seed0=1000, device="cuda")
c = pkg.Context(0, pkg.OpenCVProcessing)
if os.environ.get("LANES"): c.set_pipeline_lanes(int(os.environ["LANES"]))
if os.environ.get("CHUNK"): c.set_chunk(int(os.environ["CHUNK"]))
call = (fr.data_ptr(), n, W, H, fr.stride(1), fr.stride(0))
def go(): return int(c.sift_batch_device(*call, fetch=False)[0][-1])
for _ in range(3): go()
torch.cuda.synchronize()
ts = []
for _ in range(30):
    t = time.perf_counter(); k = go(); ts.append(time.perf_counter() - t)
c.reset_stats()
for _ in range(10): go()
st = c.stats()
print(json.dumps({"tag": os.environ.get("TAG", ""), "ms_median": 1e3 * float(np.median(ts)), "ms_min": 1e3 * min(ts),
                  "kp": k, "pyramid_ms": st["pyramid_ms"] / 10, "detect_ms": st["detect_ms"] / 10,
                  "orient_ms": st["orient_ms"] / 10, "order_ms": st["order_ms"] / 10,
                  "descriptor_ms": st["descriptor_ms"] / 10, "total_ms": st["total_ms"] / 10}))
c.close()
