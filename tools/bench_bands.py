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
    python tools/bench_bands.py --gloo-from /tmp/sift_bands_parts   (no GPU)

Each band is timed twice: results left in HBM (`device_ms`, as a GPU
consumer -- matching, the all-gather over RCCL -- takes them; n = 1 is then
the whole-frame call of bench.py's configs.giant_8192) and fetched to host
arrays (`band_ms`, PCIe + host copy: 148 B per keypoint).  Then the
all-gather of the bands' real results (shard.allgather_bands: sizes, then
one padded all_gather per array, merge by emission key) is timed on gloo
with n CPU processes (`allgather_gloo_ms`, for the record: the product path
gathers over RCCL / xGMI, which this box cannot run with one GPU).
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
    # outside gpurun_out/: the parts are ~45 MB per band count
    ap.add_argument("--parts-dir", default="/tmp/sift_bands_parts")
    ap.add_argument("--gloo-from", default=None, help="time the gloo all-gather of saved band results (no GPU)")
    a = ap.parse_args()
    if a.gloo_from:
        gloo_main(a.gloo_from, a.reps)
        return
    import torch
    import pkg_loader
    from test_gpu_large import _tiled
    pkg = pkg_loader.load()
    ctx = pkg.Context(0, pkg.OpenCVProcessing)
    img = _tiled(a.size, 47)
    d = torch.from_numpy(img).cuda()
    torch.cuda.synchronize()
    H, W = img.shape

    def run(band, n, fetch):
        ctx.set_row_band(band, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        offs, r = ctx.sift_batch_device(d.data_ptr(), 1, W, H, W, W * H, fetch=fetch)
        dt = time.perf_counter() - t0
        return dt, int(offs[-1]), r

    run(0, 1, True)  # warm-up: plan + arenas
    run(0, 1, False)
    out = {"frame": f"{W}x{H}", "reps": a.reps, "bands": {}}
    results = {}
    for n in (1, 2, 4, 8):
        ctx.reset_stats()
        per, dev, res = [], [], []
        for b in range(n):
            ts, td, nk, r = [], [], 0, None
            for _ in range(a.reps):
                dt, nk, _ = run(b, n, False)
                td.append(dt)
            for _ in range(a.reps):
                dt, nk, r = run(b, n, True)
                ts.append(dt)
            per.append((float(np.median(ts)) * 1e3, nk))
            dev.append(float(np.median(td)) * 1e3)
            res.append((r.keypoints_array.copy(), r.descriptors.copy(), r.keys.copy()))
        results[n] = res
        out["bands"][n] = {"device_ms": [round(t, 3) for t in dev], "max_device_ms": round(max(dev), 3),
                           "band_ms": [round(t, 3) for t, _ in per], "band_keypoints": [k for _, k in per],
                           "max_band_ms": round(max(t for t, _ in per), 3),
                           "reruns": int(ctx.stats()["band_reruns"]), "calls": 2 * n * a.reps}
        print(n, out["bands"][n], flush=True)
    ctx.set_row_band(0, 1)
    ctx.close()
    # the bands' real results for the gloo all-gather timing, which runs in a
    # separate invocation that never initialises the GPU (--gloo-from)
    os.makedirs(a.parts_dir, exist_ok=True)
    for n in (2, 4, 8):
        np.savez(os.path.join(a.parts_dir, f"bands_{n}.npz"),
                 **{f"{f}{r}": x for r, p in enumerate(results[n]) for f, x in zip(("k", "d", "key"), p)})
    print(json.dumps(out))


def gloo_main(parts_dir, reps):
    """All-gather timing of saved band results on gloo (CPU processes only)."""
    out = {}
    for n in (2, 4, 8):
        z = np.load(os.path.join(parts_dir, f"bands_{n}.npz"))
        parts = [(z[f"k{r}"], z[f"d{r}"], z[f"key{r}"]) for r in range(n)]
        ms = gloo_allgather_ms(parts, reps)
        out[n] = {"allgather_gloo_ms": round(ms, 3), "keypoints": sum(len(p[0]) for p in parts),
                  "bytes": sum(len(p[0]) for p in parts) * (20 + 128 + 8)}
        print(n, out[n], flush=True)
    print(json.dumps({"allgather_gloo": out}))


def _gloo_rank(rank, world, port, parts, reps, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import shard
    k, dsc, key = parts[rank]
    shard.allgather_bands(k, dsc, key, dist)  # warm-up
    ts = []
    for _ in range(reps):
        dist.barrier()
        t = time.perf_counter()
        merged = shard.allgather_bands(k, dsc, key, dist)
        ts.append(time.perf_counter() - t)
    dist.barrier()
    if rank == 0:
        q.put((float(np.median(ts)) * 1e3, len(merged[0])))
    dist.destroy_process_group()


def gloo_allgather_ms(parts, reps):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + len(parts)
    procs = [ctx.Process(target=_gloo_rank, args=(r, len(parts), port, parts, reps, q)) for r in range(len(parts))]
    for p in procs:
        p.start()
    ms, n = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert n == sum(len(p[0]) for p in parts)
    return ms


if __name__ == "__main__":
    main()
