#!/usr/bin/env python3
"""End-to-end JPEG bytes -> keypoints throughput on one MI355X (SURVEY.md
8(f) row 2; not the bench.py metric).

128 synthetic 1920x1080 RGB JPEGs (4:2:0, quality 90, PIL-encoded from the
bench's synthetic frames) in host memory.  One step = sift_mi_decode_jpeg_batch
(host-threaded entropy decoding + GPU reconstruction into a device batch)
then sift_batch_device over that batch (results kept on the device).
Reports decode-only, decode-then-sift (serial) and pipelined (a second
context decodes batch k + 1 while batch k runs through sift()) frames/s and
keypoints/s.
    python tools/bench_jpeg.py [--frames 128] [--steps 3] [--threads 16]
"""
import argparse
import io
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
    ap.add_argument("--frames", type=int, default=128)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch
    from PIL import Image
    import pkg_loader
    import synth
    pkg = pkg_loader.load()
    W, H = 1920, 1080
    base = synth.frames(8, W, H, seed0=0)
    datas = []
    for i in range(a.frames):
        f = np.roll(base[i % 8], 17 * i, 1)
        rgb = np.stack([f, np.roll(f, 5, 1), 255 - f], -1)
        b = io.BytesIO()
        Image.fromarray(rgb).save(b, "JPEG", quality=90, subsampling=2)
        datas.append(b.getvalue())
    ctx = pkg.Context(0, pkg.OpenCVProcessing)
    t = torch.empty((a.frames, H, W), dtype=torch.uint8, device="cuda")
    fp, rs = t.stride(0), t.stride(1)

    def decode():
        ctx.decode_jpeg_batch_device(datas, t.data_ptr(), fp, rs, a.threads)

    def step():
        decode()
        offs, _ = ctx.sift_batch_device(t.data_ptr(), a.frames, W, H, rs, fp, fetch=False)
        return int(offs[-1])

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        decode()
    torch.cuda.synchronize()
    dec = (time.perf_counter() - t0) / a.steps
    t0 = time.perf_counter()
    nkp = sum(step() for _ in range(a.steps))
    torch.cuda.synchronize()
    e2e = (time.perf_counter() - t0) / a.steps

    # pipelined: a second context decodes batch k + 1 (host threads + its own
    # stream) while this one runs sift() on batch k (ctypes drops the GIL)
    import threading
    dctx = pkg.Context(0, pkg.OpenCVProcessing)
    bufs = [t, torch.empty_like(t)]

    def dec_into(buf):
        dctx.decode_jpeg_batch_device(datas, buf.data_ptr(), fp, rs, a.threads)

    dec_into(bufs[0])
    t0 = time.perf_counter()
    nkp_p = 0
    for k in range(a.steps):
        th = threading.Thread(target=dec_into, args=(bufs[(k + 1) % 2],))
        th.start()
        offs, _ = ctx.sift_batch_device(bufs[k % 2].data_ptr(), a.frames, W, H, rs, fp, fetch=False)
        nkp_p += int(offs[-1])
        th.join()
    torch.cuda.synchronize()
    pipe = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"what": "JPEG bytes -> keypoints (decode_jpeg_batch + sift_batch_device)",
                      "frames": a.frames, "frame": f"{W}x{H}", "jpeg_mean_bytes": float(np.mean([len(d) for d in datas])),
                      "host_threads": a.threads, "decode_frames_per_s": a.frames / dec,
                      "serial_frames_per_s": a.frames / e2e, "serial_keypoints_per_s": nkp / a.steps / e2e,
                      "pipelined_frames_per_s": a.frames / pipe,
                      "pipelined_keypoints_per_s": nkp_p / a.steps / pipe}))
    dctx.close()
    ctx.close()


if __name__ == "__main__":
    main()
