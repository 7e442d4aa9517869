#!/usr/bin/env python3
"""bench.py -- keypoints+descriptors/s of the MI355X SIFT path on 1920x1080 batches.

Contract (driver):  python bench.py --gpus N --steps K --warmup W
For N > 1 the driver launches one process per GPU with torch.distributed.run
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the env, RCCL backend).

Workload (BASELINE.json configs[3], per GPU): every rank owns its own batch of
`--frames` (default 128) synthetic 1920x1080 u8 frames generated on its GPU
(seeded, sift-features_amd/synth.py) -- images are independent, so the batch
shards with no data-path collective ("scaling": "weak").  One step = one full
`sift()` per frame of the batch: Gaussian pyramid + DoG, extrema, orientation,
emission-order sort and descriptors, with every frame's SiftResult
(keypoints + 128-byte descriptors) left in HBM (sift_mi_set_keep_on_device):
inputs are resident in HBM when the timed region starts and outputs stay
there.  `host_fetch` reports the same steps with the results copied to host
arrays (PCIe + host copy included) -- never `value`.  The octave count is the crate's formula (10
for 1080p), not the "5 octaves" wording of configs[1].

`value` = keypoints (each with its descriptor) produced by all ranks per
second, max-over-ranks wall time between barriers.
`roofline` = the pyramid stage (seed + blur kernels; HBM-bound): SURVEY.md
8(d)'s algorithmic bytes W*H + 44*sum(P_o) per frame (u8 read once, G_0..G_5
and D_0..D_4 written once -- nothing else; the batch path writes only
G_0..G_5 and forms D where detection reads it, and its kernels' actual HBM
traffic is the PMC `traffic` field) / the stage's HIP-event time on the
kernels' stream, vs 8 TB/s, from a second pass of the same steps with the
chunks serialised (one pipeline lane) so the stage runs alone;
`stage_ms_per_step` comes from that pass too.  The stage's time includes the
extremum scan of the octaves detected with their blur 5 (k_blur_detect);
`roofline_fused_stage` states the same time against the yardstick plus what
the reference's scan reads for those octaves (20 B per octave pixel), a
separately labelled figure.  `cpu_baseline` = the CPU oracle (a C port of
src/lib.rs, 1 thread) on a bounded sample of the same frames, rank 0 at N=1;
`cpu_baseline_all_cores` the same with one frame per thread on the host's
CPU share (OMP_NUM_THREADS, 16 per GPU on the GPU pool).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))

METRIC = "keypoints+descriptors/sec on 1920×1080 batch; HBM GB/s on pyramid stage"
HBM_PEAK_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--frames", type=int, default=128, help="frames per GPU per step")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--chunk", type=int, default=0, help="frames per pipeline chunk (0 = auto)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-latency", action="store_true")
    p.add_argument("--no-configs", action="store_true", help="skip the other single-GPU BASELINE configs")
    p.add_argument("--no-unfused", action="store_true",
                   help="skip the blur-kernels-only reference pass (profiles: product kernels only)")
    p.add_argument("--no-jpeg", action="store_true", help="skip the JPEG -> keypoints end-to-end field")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="N > 1 rehearsal on a one-GPU box: every rank on cuda:0, gloo transport (not a measurement)")
    p.add_argument("--opt", action="append", default=[],
                   help="path option name=value on every context (A/B runs; default: the product path)")
    a = p.parse_args()
    for kv in a.opt:
        k, v = kv.split("=")
        PATH_OPTS[k] = int(v)
    return a


PATH_OPTS = {}  # --opt name=value


def new_context(pkg, device_index, processing):
    c = pkg.Context(device_index, processing)
    for k, v in PATH_OPTS.items():
        c.set_path_option(k, v)
    return c


def run_config(pkg, synth, dev, device_index, n, W, H, steps, seed0=1000, max_octaves=0, processing=None):
    """One BASELINE config on one GPU: `n` device-resident W x H frames per
    call, results left in HBM; keypoints/s from two-lane calls, the pyramid
    stage's HIP-event time (and its roofline fraction) from a serialised pass.
    max_octaves > 0: the labelled octave-cap extension (not the crate).
    processing: the Processing profile (default OpenCVProcessing, the one the
    reference's snapshots pin; ImageprocProcessing is the crate's sift())."""
    import torch
    fr = synth.frames_torch(n, W, H, seed0=seed0, device=dev)
    torch.cuda.synchronize()
    c = new_context(pkg, device_index, processing or pkg.OpenCVProcessing)
    if max_octaves:
        c.set_max_octaves(max_octaves)
    call = (fr.data_ptr(), n, W, H, fr.stride(1), fr.stride(0))

    def go():
        return int(c.sift_batch_device(*call, fetch=False)[0][-1])

    for _ in range(10 if n == 1 else 3):  # warm: plan, arenas, clocks (single-frame calls: ~1 ms each)
        go()
    torch.cuda.synchronize()
    ts, kp = [], 0
    for _ in range(steps):  # each call returns after its results are in HBM (host waits per chunk)
        t = time.perf_counter()
        kp += go()
        ts.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    dt = sum(ts) / steps
    c.set_pipeline_lanes(1)
    go()
    torch.cuda.synchronize()
    c.reset_stats()
    for _ in range(steps):
        go()
    torch.cuda.synchronize()
    st = c.stats()
    c.close()
    del fr
    torch.cuda.empty_cache()
    gbs = st["pyramid_bytes"] / (st["pyramid_ms"] * 1e-3) / 1e9 if st["pyramid_ms"] > 0 else 0.0
    n_oct = int(round(np.log2(min(2 * W, 2 * H)) - 2)) + 1
    return {"frames_per_call": n, "frame": f"{W}x{H}",
            "profile": "imageproc" if processing is pkg.ImageprocProcessing else "opencv",
            "octaves": min(n_oct, max_octaves) if max_octaves else n_oct,
            "ms_per_call": 1e3 * dt, "ms_per_call_median": 1e3 * float(np.median(ts)),
            "keypoints_per_s": kp / steps / dt, "frames_per_s": n / dt,
            "keypoints_per_frame": kp / steps / n, "pyramid_ms_per_call": st["pyramid_ms"] / steps,
            "pyramid_gbs": gbs, "pyramid_frac": gbs / HBM_PEAK_GBS}


def run_jpeg_e2e(pkg, synth, device_index, n, W, H, steps, threads):
    """JPEG bytes -> keypoints (examples/run-sift.rs:8
    decodes with image::open + grayscale): n synthetic W x H RGB JPEGs (4:2:0,
    quality 90, PIL-encoded from the bench's frames) in host memory; one step
    = sift_mi_decode_jpeg_batch (host-threaded entropy decoding + GPU
    reconstruction into device frames) and sift_batch_device over them,
    pipelined: a second context decodes batch k + 1 while batch k runs."""
    import io
    import threading
    import torch
    from PIL import Image
    base = synth.frames(8, W, H, seed0=0)
    datas = []
    for i in range(n):
        f = np.roll(base[i % 8], 17 * i, 1)
        rgb = np.stack([f, np.roll(f, 5, 1), 255 - f], -1)
        b = io.BytesIO()
        Image.fromarray(rgb).save(b, "JPEG", quality=90, subsampling=2)
        datas.append(b.getvalue())
    ctx = new_context(pkg, device_index, pkg.OpenCVProcessing)
    dctx = new_context(pkg, device_index, pkg.OpenCVProcessing)
    bufs = [torch.empty((n, H, W), dtype=torch.uint8, device="cuda") for _ in range(2)]
    fp, rs = bufs[0].stride(0), bufs[0].stride(1)

    def dec_into(buf):
        dctx.decode_jpeg_batch_device(datas, buf.data_ptr(), fp, rs, threads)

    def run(k):
        th = threading.Thread(target=dec_into, args=(bufs[(k + 1) % 2],))
        th.start()
        offs, _ = ctx.sift_batch_device(bufs[k % 2].data_ptr(), n, W, H, rs, fp, fetch=False)
        th.join()
        return int(offs[-1])

    dec_into(bufs[0])
    run(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nkp = sum(run(k + 1) for k in range(steps))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    t0 = time.perf_counter()
    for _ in range(steps):
        dec_into(bufs[0])
    torch.cuda.synchronize()
    dec = (time.perf_counter() - t0) / steps
    dctx.close()
    ctx.close()
    return {"frames_per_step": n, "frame": f"{W}x{H}", "jpeg_mean_bytes": float(np.mean([len(d) for d in datas])),
            "host_threads": threads, "frames_per_s": n / dt, "keypoints_per_s": nkp / steps / dt,
            "decode_only_frames_per_s": n / dec,
            "note": "pipelined: decode of batch k+1 (second context, host threads) beside sift() of batch k; "
                    "JPEGs in host memory, results kept on the device"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_one_gpu:
        local = 0  # every rank shares the one card; the gather goes over gloo
    if world > 1:
        torch.cuda.set_device(local)
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import pkg_loader
    import synth
    pkg = pkg_loader.load()

    import shard
    B, W, H = args.frames, args.width, args.height
    # weak scaling: a global batch of world*B frames, rank r owns the
    # contiguous block shard_range(world*B, r, world) (frame i = seed i)
    f0, f1 = shard.shard_range(world * B, rank, world)
    frames = synth.frames_torch(f1 - f0, W, H, seed0=f0, device=dev)
    torch.cuda.synchronize()
    ctx = new_context(pkg, local, pkg.OpenCVProcessing)
    if args.chunk:
        ctx.set_chunk(args.chunk)
    ptr, stride, pitch = frames.data_ptr(), frames.stride(1), frames.stride(0)

    out = pkg.ResultBuffers()  # streaming caller: host result arrays reused across batches

    last = {}

    def step(fetch=False):
        offs, res = ctx.sift_batch_device(ptr, B, W, H, stride, pitch, fetch=fetch, out=out)
        last["offs"] = offs
        return int(offs[-1])

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    ctx.reset_stats()
    t0 = time.perf_counter()
    n_kp = 0
    for _ in range(args.steps):
        n_kp += step()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0

    # Stage timing pass: the same steps with the chunks run one after another
    # (one pipeline lane), so the HIP-event time of each stage -- and the
    # pyramid roofline below -- is its kernels' own, not shared with the
    # overlapped neighbour chunk of the two-lane run that `value` measures.
    ctx.set_pipeline_lanes(1)
    step()
    torch.cuda.synchronize()
    ctx.reset_stats()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    serial_ms = 1e3 * (time.perf_counter() - t1) / args.steps
    st = ctx.stats()
    # The blur kernels alone, for reference: the same serialised steps with
    # the octaves' last blur as a plain strip launch and the extremum scan in
    # the detect stage (path option fused_detect = 0; the same bits).  The
    # product path fuses them, so `roofline` above is the stage as it runs.
    st_unf = None
    if not args.no_unfused:
        with ctx.path_options(fused_detect=0):
            step()
            torch.cuda.synchronize()
            ctx.reset_stats()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            st_unf = ctx.stats()
    # one more (untimed) step with the measurement-only sample counters: the
    # gradient samples the orientation and descriptor kernels evaluate per
    # step, divided by their serialised-pass stage time above
    ctx.set_sample_counting(True)
    ctx.reset_stats()
    step()
    torch.cuda.synchronize()
    sc = ctx.stats()
    ctx.set_sample_counting(False)
    ctx.set_pipeline_lanes(2)
    kp_stages = {
        "extrema_per_step": sc["extrema"], "keypoints_per_step": sc["keypoints"],
        "orientation": {"ms_per_step": st["orient_ms"] / args.steps, "samples_per_step": sc["orient_samples"],
                        "samples_per_s": sc["orient_samples"] / (st["orient_ms"] / args.steps * 1e-3),
                        "extrema_per_s": sc["extrema"] / (st["orient_ms"] / args.steps * 1e-3)},
        "descriptor": {"ms_per_step": st["descriptor_ms"] / args.steps, "samples_per_step": sc["desc_samples"],
                       "samples_per_s": sc["desc_samples"] / (st["descriptor_ms"] / args.steps * 1e-3),
                       "keypoints_per_s": sc["keypoints"] / (st["descriptor_ms"] / args.steps * 1e-3)},
        "note": "samples = patch positions / rotated-region samples the kernels evaluate (rank 0, one step, "
                "sift_mi_set_sample_counting); times from the serialised stage-timing pass",
    }

    dt_max, total_kp, total_frames = shard.reduce_run(dt, n_kp, B * args.steps, dist if world > 1 else None)

    # N > 1: the keypoint gather of the throughput path -- every rank's
    # device-resident results to rank 0 over RCCL (shard.gather_device_results:
    # sizes, then point-to-point rows into one concatenated device tensor).
    # (1) alone, one step's results, timed on its own; (2) inside a timed
    # loop of the same steps: each step's results are snapshotted in HBM (the
    # context's result arena is rewritten by the next step) and gathered
    # while the next step computes -- `value_incl_gather` (configs[3] is
    # "sharded ... via RCCL/xGMI": this is the config's whole-job rate with
    # the results on rank 0).
    gather = None
    if world > 1:
        k_dev, d_dev = shard.device_results(ctx)
        torch.cuda.synchronize()
        barrier()
        t = time.perf_counter()
        g = shard.gather_device_results(k_dev, d_dev, last["offs"], dist, dst=0)
        torch.cuda.synchronize()
        barrier()
        gms = 1e3 * (time.perf_counter() - t)
        gms = shard.reduce_run(gms / 1e3, 0, 0, dist)[0] * 1e3
        nk = int(g[0].shape[0]) if rank == 0 else 0
        del g, k_dev, d_dev
        barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        n_kp_g, got = 0, 0
        for _ in range(args.steps):
            n_kp_g += step()
            k_dev, d_dev = shard.device_results(ctx)
            snap = (k_dev.clone(), d_dev.clone())
            torch.cuda.current_stream().synchronize()  # the next step rewrites the arena
            g = shard.gather_device_results(snap[0], snap[1], last["offs"], dist, dst=0)
            if rank == 0:
                got += int(g[0].shape[0])
        torch.cuda.synchronize()
        barrier()
        dtg = time.perf_counter() - tg
        dtg_max, total_kp_g, _ = shard.reduce_run(dtg, n_kp_g, 0, dist)
        if rank == 0:
            assert got == total_kp_g, (got, total_kp_g)  # every keypoint of every step arrived
            gather = {"ms": gms, "keypoints": nk, "bytes": nk * (20 + 128),
                      "note": "one step's results of all ranks to rank 0 (device to device, RCCL send/recv), "
                              "max over ranks; not inside ms_per_step",
                      "value_incl_gather": total_kp_g / dtg_max,
                      "ms_per_step_incl_gather": 1e3 * dtg_max / args.steps,
                      "incl_note": "the same steps with every step's results gathered on rank 0 (snapshot in "
                                   "HBM, RCCL send/recv overlapped with the next step), max over ranks"}

    pyr_gbs = st["pyramid_bytes"] / (st["pyramid_ms"] * 1e-3) / 1e9 if st["pyramid_ms"] > 0 else 0.0
    per_launch_bytes = st["pyramid_bytes"] / max(1, st["pyramid_launches"])
    per_launch_ms = st["pyramid_ms"] / max(1, st["pyramid_launches"])
    fused_bytes = st["pyramid_bytes"] + st["pyramid_scan_bytes"]
    unf_gbs = (st_unf["pyramid_bytes"] / (st_unf["pyramid_ms"] * 1e-3) / 1e9
               if st_unf and st_unf["pyramid_ms"] > 0 else 0.0)
    fused_gbs = fused_bytes / (st["pyramid_ms"] * 1e-3) / 1e9 if st["pyramid_ms"] > 0 else 0.0

    # the same steps with the results copied to host arrays (PCIe-inclusive)
    host_fetch = None
    if rank == 0 and world == 1:
        step(fetch=True)
        torch.cuda.synchronize()
        hs = max(1, args.steps)
        t = time.perf_counter()
        hk = sum(step(fetch=True) for _ in range(hs))
        he = time.perf_counter() - t
        host_fetch = {"value": hk / he, "unit": "keypoints/s", "ms_per_step": 1e3 * he / hs,
                      "note": "results copied to host arrays each step (device->host + host copy)"}

    latency_ms = None
    if not args.no_latency and rank == 0:
        one = frames[:1]
        for _ in range(2):
            ctx.sift_batch_device(one.data_ptr(), 1, W, H, stride, pitch, fetch=True)
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            ctx.sift_batch_device(one.data_ptr(), 1, W, H, stride, pitch, fetch=True)
            ts.append(time.perf_counter() - t)
        latency_ms = 1e3 * float(np.median(ts))

    cpu, cpu_all = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        host = frames.cpu().numpy()
        kps, nfr, t = 0, 0, time.perf_counter()
        while nfr < B and (nfr == 0 or time.perf_counter() - t < args.cpu_seconds):
            kps += len(oracle.sift(host[nfr])[0])
            nfr += 1
        el = time.perf_counter() - t
        cpu = {"value": kps / el, "unit": "keypoints/s", "cores": 1, "kind": "port",
               "sample": f"{nfr} of the {B} benchmark frames ({W}x{H}), full sift() each, "
                         f"single-threaded C oracle (oracle/sift_oracle.c), {el:.1f} s"}
        # the host cores this process may use, one frame per thread (the C
        # oracle releases the GIL; SURVEY.md 8(d) asks for both baselines)
        from concurrent.futures import ThreadPoolExecutor
        # the box's CPU share: OMP_NUM_THREADS (16 per GPU on the pool; the
        # affinity mask shows the whole machine)
        cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
        kps, nfr, t = 0, 0, time.perf_counter()
        with ThreadPoolExecutor(cores) as ex:
            while nfr < B and (nfr == 0 or time.perf_counter() - t < args.cpu_seconds):
                batch = range(nfr, min(B, nfr + cores))
                kps += sum(len(r[0]) for r in ex.map(lambda i: oracle.sift(host[i]), batch))
                nfr += len(batch)
        el = time.perf_counter() - t
        cpu_all = {"value": kps / el, "unit": "keypoints/s", "cores": cores, "kind": "port",
                   "sample": f"{nfr} of the {B} benchmark frames, one per thread on {cores} threads, {el:.1f} s"}

    # the other single-GPU configs of BASELINE.json (extra fields, rank 0 at
    # N = 1): configs[1] one 1080p frame per call, configs[2] 256 VGA frames
    # per call, configs[4] one 8192^2 frame per call (the crate's octave
    # count: 10 / 9 / 13 octaves, not the configs' "5" / "7" wording)
    configs = None
    if rank == 0 and world == 1 and not args.no_configs:
        ctx.close()
        ctx = None
        del frames
        torch.cuda.empty_cache()
        configs = {
            "single_1080p": run_config(pkg, synth, dev, local, 1, 1920, 1080, max(30, args.steps)),
            "vga_256": run_config(pkg, synth, dev, local, 256, 640, 480, max(3, args.steps)),
            "giant_8192": run_config(pkg, synth, dev, local, 1, 8192, 8192, max(3, args.steps)),
            # LABELLED EXTENSION (sift_mi_set_max_octaves, not the crate): the
            # configs' "5 octaves" (#2) and "7 octaves" (#5) wording
            "ext_single_1080p_5oct": run_config(pkg, synth, dev, local, 1, 1920, 1080, max(30, args.steps),
                                                max_octaves=5),
            "ext_giant_8192_7oct": run_config(pkg, synth, dev, local, 1, 8192, 8192, max(3, args.steps),
                                              max_octaves=7),
            # the crate's own default sift() profile (ImageprocProcessing,
            # src/lib.rs:71-73, 993-1007) on the headline batch
            "imageproc_batch_1080p": run_config(pkg, synth, dev, local, B, W, H, max(3, args.steps),
                                                processing=pkg.ImageprocProcessing),
        }
        configs["single_1080p"]["latency_host_fetch_ms"] = latency_ms
        if not args.no_jpeg:
            configs["jpeg_e2e"] = run_jpeg_e2e(pkg, synth, local, B, W, H, max(3, args.steps),
                                               min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))

    # HBM traffic of the same launch group from the committed PMC passes
    # (tools/round_profile.sh -> profiles/pmc_traffic.json), scaled to one
    # launch like `achieved`; null when no measurement matches this frame size
    traffic, traffic_src = None, None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            t = json.load(f)
        if t["frame"] == f"{W}x{H}":
            traffic = t["pyramid_hbm_bytes_per_launch"]
            traffic_src = t["source"]
    except (OSError, KeyError, ValueError):
        pass

    if rank == 0:
        n_oct = int(round(np.log2(min(2 * W, 2 * H)) - 2)) + 1
        out = {
            "metric": METRIC,
            "value": total_kp / dt_max,
            "unit": "keypoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * dt_max / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded procedural blob frames generated on device, synth.py)",
            "config": {"workload": f"batch of {B} x {W}x{H} u8 frames per GPU (configs[3] shard), full sift()",
                       "frames_per_gpu": B, "frame": f"{W}x{H}", "octaves": n_oct, "profile": "opencv",
                       "parallelism": f"dp{world} (frames sharded, no collective)",
                       "chunking": (f"--chunk {args.chunk}" if args.chunk else
                                    "auto (path option chunk_mode, default 1: as few chunks as ~64 GB of pyramid "
                                    "allows; 128 x 1080p runs as one chunk)"),
                       **({"path_options": dict(PATH_OPTS)} if PATH_OPTS else {}),
                       **({"rehearsal": "every rank on cuda:0, gloo transport: not a measurement"}
                          if args.rehearse_one_gpu else {})},
            "frames_per_s": total_frames / dt_max,
            "keypoints_per_frame": total_kp / max(1.0, total_frames),
            "stage_ms_per_step": {k: st[k] / args.steps for k in
                                  ("pyramid_ms", "detect_ms", "orient_ms", "order_ms", "descriptor_ms", "total_ms")},
            "serial_lane_ms_per_step": serial_ms,
            "latency_1frame_ms": latency_ms,
            "host_fetch": host_fetch,
            "roofline": {"bound": "hbm", "achieved": pyr_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": pyr_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "pyramid stage (k_seed_pair + k_blur2_strip + k_blur_strip<R> + k_octave_tail + "
                                   "k_blur_detect, whose time includes the extremum scan of the octaves it fuses), "
                                   "rank 0; yardstick SURVEY.md 8(d) W*H + 44*sum(P_o) per frame",
                         "algorithmic_bytes_per_frame": st["pyramid_bytes"] / max(1, st["frames"]),
                         "algorithmic_bytes_per_launch": per_launch_bytes,
                         "launches": st["pyramid_launches"],
                         "avg_launch_ms": per_launch_ms},
            "roofline_blur_kernels_only": None if st_unf is None else {
                "achieved": unf_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": unf_gbs / HBM_PEAK_GBS,
                "pyramid_ms_per_step": st_unf["pyramid_ms"] / args.steps,
                "detect_ms_per_step": st_unf["detect_ms"] / args.steps,
                "note": "not the product path: the same serialised steps with path option fused_detect=0 "
                        "(every octave's blur 5 a plain strip launch, its extremum scan in the detect stage), "
                        "so the stage holds only the blur kernels; same yardstick (SURVEY.md 8(d))"},
            "roofline_fused_stage": {"achieved": fused_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": fused_gbs / HBM_PEAK_GBS,
                                     "bytes_per_launch": fused_bytes / max(1, st["pyramid_launches"]),
                                     "note": "the same stage time against the 8(d) yardstick plus what the "
                                             "reference's extremum scan reads for the octaves k_blur_detect "
                                             "scans inside the stage (5 DoG planes, 20 B per octave pixel)"},
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "keypoint_stages": kp_stages,
            "gather": gather,
            "value_incl_gather": gather["value_incl_gather"] if gather else None,
            "configs": configs,
        }
        print(json.dumps(out), flush=True)
    if ctx is not None:
        ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
