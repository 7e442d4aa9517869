"""bench.run_config's single-frame timing in a fresh process (A/B of what
precedes it: PRE=1 runs and closes a 128-frame batch context first, as
bench.py does before its configs)."""
import os, sys, json
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))
import torch, pkg_loader, synth, bench
pkg = pkg_loader.load()
if os.environ.get("PRE"):
    fr = synth.frames_torch(128, 1920, 1080, seed0=0, device="cuda")
    c = pkg.Context(0, pkg.OpenCVProcessing)
    for _ in range(5):
        c.sift_batch_device(fr.data_ptr(), 128, 1920, 1080, fr.stride(1), fr.stride(0), fetch=False)
    c.close()
    del fr
    torch.cuda.empty_cache()
r = bench.run_config(pkg, synth, "cuda", 0, 1, 1920, 1080, 30)
print(json.dumps({"pre": os.environ.get("PRE"), "q": os.environ.get("GPU_MAX_HW_QUEUES")} | {k: r[k] for k in ("ms_per_call", "ms_per_call_median", "pyramid_ms_per_call")}))
