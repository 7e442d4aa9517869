"""Latency of ONE large frame split by row bands.

For n in {1, 2, 4, 8}: time each band's sift() of the same device-resident
frame on this one GPU (results fetched to host, as a caller needs them).  In
an n-GPU split every rank runs one band concurrently, so the slowest band is
the per-rank compute latency (each band computes only its rows of the
pyramid plus margins; `reruns` counts calls that fell back to the whole
pyramid); the all-gather of the bands' results (~156 B
per keypoint) comes on top.  Frames are the tiled synthetic frames of
tests/test_gpu_large.py (8192 x 8192 by default, configs #5).

    python tools/bench_bands.py [--size 8192] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import pkg_loader
    from test_gpu_large import _tiled
    pkg = pkg_loader.load()
    ctx = pkg.Context(0, pkg.OpenCVProcessing)
    img = _tiled(a.size, 47)
    d = torch.from_numpy(img).cuda()
    torch.cuda.synchronize()
    H, W = img.shape

    def run(band, n):
        ctx.set_row_band(band, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, r = ctx.sift_batch_device(d.data_ptr(), 1, W, H, W, W * H)
        dt = time.perf_counter() - t0
        return dt, len(r)

    run(0, 1)  # warm-up: plan + arenas
    out = {"frame": f"{W}x{H}", "reps": a.reps, "bands": {}}
    for n in (1, 2, 4, 8):
        ctx.reset_stats()
        per = []
        for b in range(n):
            ts, nk = [], 0
            for _ in range(a.reps):
                dt, nk = run(b, n)
                ts.append(dt)
            per.append((float(np.median(ts)) * 1e3, nk))
        out["bands"][n] = {"band_ms": [round(t, 3) for t, _ in per], "band_keypoints": [k for _, k in per],
                           "max_band_ms": round(max(t for t, _ in per), 3),
                           "reruns": int(ctx.stats()["band_reruns"]), "calls": n * a.reps}
        print(n, out["bands"][n], flush=True)
    ctx.set_row_band(0, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
