"""Batch / device-resident / chunked paths equal per-image `sift()` results, and
edge cases (tiny, flat, strided inputs) match the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames():
    import synth
    return synth.frames(5, 160, 120, seed0=20)


def test_batch_equals_single(pkg, ctx):
    fr = _frames()
    batch = ctx.sift_batch(fr)
    for i in range(len(fr)):
        single = ctx.sift(fr[i])
        assert single == batch[i], i
        f = pkg.key_fields(batch[i].keys)
        assert np.all(f["frame"] == i)


def test_chunked_batch(pkg, ctx):
    fr = _frames()
    ref = ctx.sift_batch(fr)
    c2 = pkg.Context(0)
    c2.set_chunk(2)
    got = c2.sift_batch(fr)
    c2.close()
    assert all(a == b for a, b in zip(ref, got))


def test_device_batch_torch(pkg, ctx):
    import torch
    fr = _frames()
    t = torch.from_numpy(fr).cuda()
    torch.cuda.synchronize()
    offs, res = ctx.sift_batch_device(t.data_ptr(), t.shape[0], t.shape[2], t.shape[1], t.stride(1),
                                      t.stride(0))
    ref = ctx.sift_batch(fr)
    for i in range(len(fr)):
        a, b = int(offs[i]), int(offs[i + 1])
        assert np.array_equal(res.keypoints_array[a:b], ref[i].keypoints_array)
        assert np.array_equal(res.descriptors[a:b], ref[i].descriptors)


def test_deterministic(ctx):
    import synth
    img = synth.frame(640, 480, 9)
    assert ctx.sift(img) == ctx.sift(img)


@pytest.mark.parametrize("shape", [(1, 1), (2, 2), (3, 7), (10, 10), (20, 3), (21, 40), (33, 19)])
def test_tiny_images(pkg, ctx, oracle, shape):
    from test_gpu_parity import assert_parity
    rng = np.random.default_rng(sum(shape))
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    res = ctx.sift(img)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


def test_flat_image_no_keypoints(ctx, oracle):
    img = np.full((120, 160), 77, np.uint8)
    assert len(oracle.sift(img)[0]) == 0
    assert len(ctx.sift(img)) == 0


def test_strided_input(ctx):
    import synth
    big = synth.frame(200, 150, 4)
    view = big[10:130, 7:167]  # non-contiguous rows: row_stride 200 > width 160
    assert ctx.sift(view) == ctx.sift(np.ascontiguousarray(view))


@pytest.mark.parametrize("w,h,stride", [(241, 61, 241), (77, 45, 77), (161, 97, 163), (39, 30, 41)])
def test_odd_stride_batch(pkg, ctx, oracle, w, h, stride):
    """Odd widths / row strides and unaligned frame bases: the strip seed
    (source width >= 80) and the tile seed (narrower frames) read rows that do
    not start on 4-byte boundaries; the batch equals the oracle per frame."""
    from test_gpu_parity import assert_parity
    import synth
    import torch
    n = 3
    frames = np.stack([synth.frame(w, h, 40 + i) for i in range(n)])
    got = ctx.sift_batch(frames)  # host frames: packed, odd widths give unaligned rows
    buf = np.zeros(n * h * stride + 1, np.uint8)  # device frames: odd stride, base at byte 1
    view = np.lib.stride_tricks.as_strided(buf[1:], (n, h, w), (h * stride, stride, 1))
    view[:] = frames
    t = torch.from_numpy(buf).cuda()
    torch.cuda.synchronize()
    offs, res = ctx.sift_batch_device(t.data_ptr() + 1, n, w, h, stride, h * stride)
    for i in range(n):
        kp_o, desc_o, ext_o = oracle.sift(frames[i], internal=True)
        assert_parity(pkg, got[i], kp_o, desc_o, ext_o)
        a, b = int(offs[i]), int(offs[i + 1])
        assert np.array_equal(res.keypoints_array[a:b], got[i].keypoints_array), i
        assert np.array_equal(res.descriptors[a:b], got[i].descriptors), i


def test_random_noise(pkg, ctx, oracle):
    """White noise: many plateaus/ties and dense extrema (worst case for ordering)."""
    from test_gpu_parity import assert_parity
    img = np.random.default_rng(5).integers(0, 256, (96, 128), dtype=np.uint8)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    res = ctx.sift(img)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


@pytest.mark.parametrize("chunk", [0, 2, -1, -2])
def test_device_resident_results(pkg, ctx, chunk):
    """fetch=False keeps every frame's results in HBM (the bench's `value`
    path); copied back they equal the host-fetched batch, chunked or not.
    chunk -1: the whole batch in one chunk, -2: a single frame -- one chunk,
    whose results are handed out as the slot's own output buffers (no copy;
    host.cpp res_slot), then a fetch=True call on the same context must
    return its own results, not the slot's stale ones."""
    import torch
    fr = _frames()
    if chunk == -2:
        fr = fr[:1]
    t = torch.from_numpy(fr).cuda()
    c2 = pkg.Context(0)
    if chunk == -1:
        c2.set_chunk(len(fr))
    elif chunk:
        c2.set_chunk(chunk)
    offs, res = c2.sift_batch_device(t.data_ptr(), t.shape[0], t.shape[2], t.shape[1], t.stride(1), t.stride(0),
                                     fetch=False)
    assert res is None
    kp_ptr, desc_ptr, n = c2.device_results()
    assert n == int(offs[-1]) > 0
    # copy the device arrays back with hipMemcpy
    kp = np.empty((n, 5), np.float32)
    desc = np.empty((n, 128), np.uint8)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(kp.ctypes.data, kp_ptr, kp.nbytes, 2) == 0      # hipMemcpyDeviceToHost
    assert hip.hipMemcpy(desc.ctypes.data, desc_ptr, desc.nbytes, 2) == 0
    ref = ctx.sift_batch(fr)
    for i in range(len(fr)):
        a, b = int(offs[i]), int(offs[i + 1])
        assert np.array_equal(kp[a:b], ref[i].keypoints_array), i
        assert np.array_equal(desc[a:b], ref[i].descriptors), i
    if chunk < 0:
        # a fetched call after the direct-slot one: its own results
        fr2 = np.ascontiguousarray(fr[:, ::-1])
        t2 = torch.from_numpy(fr2).cuda()
        offs2, res2 = c2.sift_batch_device(t2.data_ptr(), t2.shape[0], t2.shape[2], t2.shape[1], t2.stride(1),
                                           t2.stride(0), fetch=True)
        ref2 = ctx.sift_batch(fr2)
        for i in range(len(fr2)):
            a, b = int(offs2[i]), int(offs2[i + 1])
            assert np.array_equal(res2.keypoints_array[a:b], ref2[i].keypoints_array), i
            assert np.array_equal(res2.descriptors[a:b], ref2[i].descriptors), i
        # and a device-resident call again
        offs3, _ = c2.sift_batch_device(t.data_ptr(), t.shape[0], t.shape[2], t.shape[1], t.stride(1), t.stride(0),
                                        fetch=False)
        kp_ptr3, desc_ptr3, n3 = c2.device_results()
        assert n3 == n
        assert hip.hipMemcpy(kp.ctypes.data, kp_ptr3, kp.nbytes, 2) == 0
        assert np.array_equal(kp[: int(offs[1])], ref[0].keypoints_array)
    c2.close()


def test_pipeline_lanes_equal(pkg, ctx):
    """Two-lane (overlapped chunks) and one-lane batches give identical results."""
    fr = _frames()
    out = []
    for lanes in (1, 2):
        c2 = pkg.Context(0)
        c2.set_chunk(2)
        c2.set_pipeline_lanes(lanes)
        out.append(c2.sift_batch(fr))
        c2.close()
    assert all(a == b for a, b in zip(out[0], out[1]))
    assert all(a == b for a, b in zip(out[0], ctx.sift_batch(fr)))


def test_device_results_views(pkg, ctx):
    """shard.device_results wraps the device result arena as torch cuda
    tensors without a copy; they equal the host-fetched batch."""
    import torch
    import shard
    fr = _frames()
    t = torch.from_numpy(fr).cuda()
    c2 = pkg.Context(0)
    offs, _ = c2.sift_batch_device(t.data_ptr(), t.shape[0], t.shape[2], t.shape[1], t.stride(1), t.stride(0),
                                   fetch=False)
    k, d = shard.device_results(c2)
    kp_ptr, desc_ptr, n = c2.device_results()
    assert k.is_cuda and d.is_cuda and k.shape == (n, 5) and d.shape == (n, 128)
    assert k.data_ptr() == kp_ptr and d.data_ptr() == desc_ptr  # views, not copies
    ref = ctx.sift_batch(fr)
    kh, dh = k.cpu().numpy(), d.cpu().numpy()
    for i in range(len(fr)):
        a, b = int(offs[i]), int(offs[i + 1])
        assert np.array_equal(kh[a:b], ref[i].keypoints_array), i
        assert np.array_equal(dh[a:b], ref[i].descriptors), i
    c2.close()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_worker(rank, world, port, q):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "sift-features_amd"))
    import torch
    import torch.distributed as dist
    import pkg_loader
    import shard
    import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = pkg_loader.load()
        ctx = pkg.Context(0, pkg.OpenCVProcessing)
        ctx.set_chunk(2)
        f0, f1 = shard.shard_range(5, rank, world)  # 3 + 2 frames, several chunks on rank 0
        t = torch.from_numpy(synth.frames(f1 - f0, 640, 480, seed0=f0)).cuda()  # the same u8 frames as the reference below
        torch.cuda.synchronize()
        offs, _ = ctx.sift_batch_device(t.data_ptr(), f1 - f0, 640, 480, t.stride(1), t.stride(0), fetch=False)
        k, d = shard.device_results(ctx)
        g = shard.gather_device_results(k, d, offs, dist, dst=0)
        ok = True
        if rank == 0:
            allf = synth.frames(5, 640, 480, seed0=0)
            ref = ctx.sift_batch(allf)
            kh, dh, oh = (x.cpu().numpy() for x in g)
            ok = len(oh) == 6 and int(oh[-1]) == sum(len(r) for r in ref)
            for i in range(5):
                a, b = int(oh[i]), int(oh[i + 1])
                ok = ok and np.array_equal(kh[a:b], ref[i].keypoints_array) and np.array_equal(dh[a:b], ref[i].descriptors)
        q.put(("ok", rank, bool(ok)))
        ctx.close()
    except Exception as e:  # pragma: no cover - surfaced by the assert below
        q.put(("err", rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_world2_gather_device_results(pkg):
    """The bench's N > 1 keypoint gather on real results: two ranks (sharing
    cuda:0, gloo transport) each run sift_batch_device on their frame shard
    with the results left in HBM; gather_device_results on rank 0 equals the
    whole batch run in one process, frame for frame."""
    import multiprocessing as mp
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(r[0] == "ok" and r[2] for r in res), res


def _nccl_worker(port, q):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "sift-features_amd"))
    import torch
    import torch.distributed as dist
    import pkg_loader
    import shard
    import synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        pkg = pkg_loader.load()
        ctx = pkg.Context(0, pkg.OpenCVProcessing)
        ctx.set_chunk(2)
        t = torch.from_numpy(synth.frames(3, 640, 480, seed0=7)).cuda()
        torch.cuda.synchronize()
        offs, _ = ctx.sift_batch_device(t.data_ptr(), 3, 640, 480, t.stride(1), t.stride(0), fetch=False)
        k, d = shard.device_results(ctx)
        g = shard.gather_device_results(k, d, offs, dist, dst=0)
        dist.barrier()
        ref = ctx.sift_batch(synth.frames(3, 640, 480, seed0=7))
        kh, dh, oh = (x.cpu().numpy() for x in g)
        ok = g[0].is_cuda and len(oh) == 4 and int(oh[-1]) == sum(len(r) for r in ref)
        for i in range(3):
            a, b = int(oh[i]), int(oh[i + 1])
            ok = ok and np.array_equal(kh[a:b], ref[i].keypoints_array) and np.array_equal(dh[a:b], ref[i].descriptors)
        # the bench's max-over-ranks reduction as a real RCCL all-reduce
        x = torch.tensor([1.5], dtype=torch.float64, device="cuda")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        ok = ok and float(x.item()) == 1.5
        q.put(("ok", 0, bool(ok)))
        ctx.close()
    except Exception as e:  # pragma: no cover - surfaced by the assert below
        q.put(("err", 0, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(120)
def test_nccl_world1_gather_device_results(pkg):
    """The RCCL (backend "nccl") side of the N > 1 path on the one card a
    test box has: a one-rank process group initialised the way bench.py does
    (device_id given), the size all-gather of gather_device_results, a
    barrier and an all-reduce on device tensors; the gathered device results
    equal sift_batch's.  (Two ranks cannot share one GPU under RCCL; the
    point-to-point rows are covered on gloo by the test above.)"""
    import multiprocessing as mp
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    p = mpc.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=110)
    p.join(timeout=30)
    assert p.exitcode == 0
    assert res[0] == "ok" and res[2], res


@pytest.mark.gpu
def test_batch_tail_planes_exact(pkg, oracle):
    """A one-chunk batch of 6 frames: every octave's planes of frames 0 and
    5, the tail octaves' from k_octave_tail (one workgroup per frame), equal
    the oracle's bit for bit."""
    import synth
    fr = synth.frames(6, 640, 480, seed0=60)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    c.set_chunk(6)
    try:
        c.sift_batch(fr)
        for i in (0, 5):
            opy = oracle.Pyramid(fr[i], 0)
            for o in range(opy.n_octaves):
                assert np.array_equal(c.read_batch_scale_space(i, o), opy.scale_space(o)), (i, o)
    finally:
        c.close()


@pytest.mark.gpu
def test_batch_fused_kernels_equal_single_launches(pkg):
    """The batch path (no DoG planes) with the pair and tail kernels equals the
    batch path with single-blur launches only, bit for bit (1080p frames:
    the pair covers octaves 0-4, the tail octaves 5-9)."""
    import synth
    frames = np.stack([synth.frame(1920, 1080, s) for s in range(2)])
    c = pkg.Context(0, pkg.OpenCVProcessing)
    try:
        fused = c.sift_batch(frames)
        with c.path_options(pair_blur=0, tail=0):
            single = c.sift_batch(frames)
    finally:
        c.close()
    for a, b in zip(fused, single):
        assert np.array_equal(a.keypoints_array, b.keypoints_array)
        assert np.array_equal(a.descriptors, b.descriptors)
        assert np.array_equal(a.keys, b.keys)


@pytest.mark.parametrize("fetch", [False, True])
def test_single_chunk_graph_replay(pkg, ctx, oracle, fetch):
    """Path option graph = 1: identical single-frame calls are captured once
    (the second call) and replayed as a HIP graph; every call's results equal
    the normal path's and the oracle's, also after the frame contents change
    in place (the graph reads the frame buffer anew), when the frame pointer
    changes (a new capture) and when a path option changes between calls (the
    options are part of the graph's key: ADVICE r04)."""
    import torch
    import synth
    from test_gpu_parity import assert_parity
    a = synth.frame(640, 480, 3)
    b = synth.frame(640, 480, 4)
    ref = {0: ctx.sift(a), 1: ctx.sift(b)}
    t = torch.from_numpy(a).cuda()
    c = pkg.Context(0)
    c.set_path_option("graph", 1)
    for i in range(5):
        src = a if i < 3 else b
        if i == 3:
            t.copy_(torch.from_numpy(b))  # same pointer, new contents
        torch.cuda.synchronize()
        offs, res = c.sift_batch_device(t.data_ptr(), 1, 640, 480, t.stride(0), t.numel(), fetch=fetch)
        want = ref[0 if i < 3 else 1]
        if fetch:
            assert res == want, i
        else:
            assert int(offs[-1]) == len(want), i
    t2 = torch.from_numpy(b).cuda()  # a new pointer: a new key
    for i in range(3):
        offs, res = c.sift_batch_device(t2.data_ptr(), 1, 640, 480, t2.stride(0), t2.numel(), fetch=True)
        assert res == ref[1], i
    kp_o, desc_o, ext_o = oracle.sift(b, internal=True)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)
    for opts in ({"early": 0}, {"fused_detect": 0, "desc_first": 0}, {}):
        with c.path_options(**opts):
            for i in range(3):
                offs, res = c.sift_batch_device(t2.data_ptr(), 1, 640, 480, t2.stride(0), t2.numel(), fetch=True)
                assert res == ref[1], (opts, i)
                assert np.array_equal(res.keys, ref[1].keys), (opts, i)
    c.close()


@pytest.mark.parametrize("knob,on", [("early", 1), ("desc_first", 1), ("large_first", 1), ("onesweep", 1)])
@pytest.mark.parametrize("profile", [0, 1])
def test_single_chunk_paths_equal(pkg, knob, on, profile):
    """One-chunk calls take latency paths of their own -- the octaves below
    the tail detected, refined and oriented on the aux stream beside the tail
    kernel with the tail octaves in a region of their own
    (Slot::early), the descriptors computed in keypoint index order beside
    the ordering stage, then gathered (Slot::desc_first) -- whose results
    must equal the general path's (the knob = 0) bit for bit, incl. keys.
    Each frame runs twice: the second call uses the bounds the first one
    learned."""
    import synth
    frames = [synth.frame(640, 480, 3), synth.frame(1000, 333, 5),
              np.random.default_rng(5).integers(0, 256, (96, 128), dtype=np.uint8)]
    prof = pkg.OpenCVProcessing if profile == 0 else pkg.ImageprocProcessing
    c = pkg.Context(0, prof)
    c.set_path_option(knob, on)
    got = [c.sift(f) for f in frames for _ in range(2)]
    c.set_path_option(knob, 0)
    ref = [c.sift(f) for f in frames for _ in range(2)]
    c.close()
    for a, b in zip(got, ref):
        assert a == b
        assert np.array_equal(a.keys, b.keys)


@pytest.mark.parametrize("limit", [None, 40])
def test_batch_onesweep_equal(pkg, ctx, limit):
    """Path option onesweep = 1 (rocprim's Onesweep radix sort for the
    emission-order and response sorts at every size) gives the same results
    as the default sort path, chunked batches and features_limit included."""
    fr = _frames()
    ref = ctx.sift_batch(fr, features_limit=limit)
    c = pkg.Context(0)
    c.set_chunk(2)
    c.set_path_option("onesweep", 1)
    got = c.sift_batch(fr, features_limit=limit)
    c.close()
    for a, b in zip(got, ref):
        assert a == b
        assert np.array_equal(a.keys, b.keys)
