"""One row band of an 8192^2 frame, repeated (for rocprofv3 --kernel-trace):
which launches of a band's call do not shrink with the band (VERDICT r05
item 7).  python tools/band_trace.py [--bands 8] [--band 3] [--calls 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--bands", type=int, default=8)
    ap.add_argument("--band", type=int, default=3)
    ap.add_argument("--calls", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    import pkg_loader
    from test_gpu_large import _tiled
    pkg = pkg_loader.load()
    ctx = pkg.Context(0, pkg.OpenCVProcessing)
    img = _tiled(a.size, 47)
    d = torch.from_numpy(img).cuda()
    H, W = img.shape
    ctx.set_row_band(a.band, a.bands)
    ts = []
    for i in range(a.calls + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.sift_batch_device(d.data_ptr(), 1, W, H, W, W * H, fetch=False)
        ts.append(time.perf_counter() - t0)
    print(f"band {a.band} of {a.bands}: median {1e3 * float(np.median(ts[2:])):.3f} ms per call")
    ctx.close()


if __name__ == "__main__":
    main()
