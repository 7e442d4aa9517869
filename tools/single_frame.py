#!/usr/bin/env python3
"""Single-frame latency probe (configs[1]: one 1920x1080 frame per call,
results left in HBM), for rocprofv3 --kernel-trace runs of the per-call
critical path.
    python tools/single_frame.py [--calls 50] [--width 1920] [--height 1080] [--octaves 0]
Prints the mean / median ms per call of the timed calls (after 10 warm-up
calls), the same measurement as bench.py's configs.single_1080p.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--octaves", type=int, default=0)
    ap.add_argument("--frames", type=int, default=1, help="frames per call (batch A/B runs)")
    ap.add_argument("--opt", action="append", default=[], help="path option name=value (A/B runs)")
    a = ap.parse_args()
    import torch
    import pkg_loader
    import synth
    pkg = pkg_loader.load()
    W, H = a.width, a.height
    fr = synth.frames_torch(a.frames, W, H, seed0=1000, device=torch.device("cuda", 0))
    torch.cuda.synchronize()
    c = pkg.Context(0, pkg.OpenCVProcessing)
    if a.octaves:
        c.set_max_octaves(a.octaves)
    opts = {}
    for kv in a.opt:
        k, v = kv.split("=")
        opts[k] = int(v)
        c.set_path_option(k, int(v))
    call = (fr.data_ptr(), a.frames, W, H, fr.stride(1), fr.stride(0))
    for _ in range(10):
        c.sift_batch_device(*call, fetch=False)
    torch.cuda.synchronize()
    ts, kp = [], 0
    for _ in range(a.calls):
        t = time.perf_counter()
        kp += int(c.sift_batch_device(*call, fetch=False)[0][-1])
        ts.append(time.perf_counter() - t)
    c.close()
    print(json.dumps({"frame": f"{W}x{H}", "frames_per_call": a.frames, "calls": a.calls, "ms_per_call": 1e3 * float(np.mean(ts)),
                      "ms_per_call_median": 1e3 * float(np.median(ts)), "keypoints_per_call": kp / a.calls, "path_options": opts}))


if __name__ == "__main__":
    main()
