"""Multi-GPU data parallelism for batches of frames.

Frames are independent, so a batch shards by contiguous frame blocks, one
process per GPU (torch.distributed, RCCL backend on MI355X), with no
data-path collective: every rank runs the whole path on its own frames.  The
only collectives are
  * `reduce_run`    -- the benchmark's max-over-ranks time and summed counts;
  * `gather_device_results` -- the "trivial keypoint gather" of the north
                        star on the throughput path: every rank's
                        device-resident results (`device_results`: zero-copy
                        views of the context's result arena) land in one
                        concatenated device tensor on rank `dst`, in global
                        frame order -- sizes all-gathered, then each rank's
                        exact rows sent point-to-point (RCCL send/recv over
                        xGMI) into their slice: no padding, no host round trip;
  * `gather_results` -- the same for host arrays (padded payloads in one
                        gather per array).
All run unchanged on gloo (CPU tensors; tests/test_shard.py) and RCCL (GPU
tensors).

One large frame splits by ROW BANDS instead:
`sift_row_bands` gives each rank band (rank, world) of the keypoint stages
(Context.set_row_band: every rank builds the frame's pyramid, detection and
everything after it covers only the rank's octave rows), then all-gathers
the bands' (emission key, keypoint, descriptor) rows and merges them by
emission key -- the one exchange step.  The bands partition every octave's
candidate rows, so the merge is exactly the whole-frame sift() result.
"""
import numpy as np


def shard_range(n_total, rank, world):
    """Contiguous block [start, stop) of frames owned by `rank`; blocks differ
    in size by at most one frame and cover 0..n_total exactly once."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    q, r = divmod(n_total, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def _device(dist):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def reduce_run(seconds, keypoints, frames, dist=None):
    """(max seconds over ranks, total keypoints, total frames)."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(seconds), int(keypoints), int(frames)
    dev = _device(dist)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=dev)
    c = torch.tensor([float(keypoints), float(frames)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), int(c[0].item()), int(c[1].item())


def gather_results(keypoints, descriptors, offsets, dist, dst=0):
    """Concatenate every rank's (keypoints (n,5) f32, descriptors (n,128) u8,
    per-frame offsets (m+1,)) on rank `dst`, in rank (= global frame) order.

    Returns (keypoints, descriptors, offsets) on `dst`, None elsewhere.
    """
    import torch
    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = _device(dist)
    kps = np.ascontiguousarray(keypoints, dtype=np.float32).reshape(-1, 5)
    desc = np.ascontiguousarray(descriptors, dtype=np.uint8).reshape(-1, 128)
    offs = np.asarray(offsets, dtype=np.int64)
    n, m = len(kps), len(offs) - 1
    if len(desc) != n or offs[-1] - offs[0] != n:
        raise ValueError("keypoints / descriptors / offsets disagree")
    sizes = torch.tensor([n, m], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes)
    ns = [int(s[0]) for s in all_sizes]
    ms = [int(s[1]) for s in all_sizes]
    n_max, m_max = max(max(ns), 1), max(ms)

    def padded(a, rows, dtype):
        t = torch.zeros((rows,) + a.shape[1:], dtype=dtype, device=dev)
        if len(a):
            t[: len(a)] = torch.from_numpy(a).to(dev)
        return t

    # keypoints as raw 32-bit words, descriptors as bytes (exact bits on any backend)
    payload = {
        "kps": padded(kps.view(np.int32), n_max, torch.int32),
        "desc": padded(desc, n_max, torch.uint8),
        "offs": padded(offs - offs[0], m_max + 1, torch.int64),
    }
    out = {}
    for key, t in payload.items():
        lst = [torch.zeros_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, gather_list=lst, dst=dst)
        out[key] = lst
    if rank != dst:
        return None
    k_all, d_all, o_all, base = [], [], [0], 0
    for r in range(world):
        k_all.append(out["kps"][r][: ns[r]].cpu().numpy().view(np.float32))
        d_all.append(out["desc"][r][: ns[r]].cpu().numpy())
        o = out["offs"][r][1: ms[r] + 1].cpu().numpy()
        o_all.extend((o + base).tolist())
        base += ns[r]
    return (np.concatenate(k_all).reshape(-1, 5), np.concatenate(d_all).reshape(-1, 128),
            np.asarray(o_all, dtype=np.int64))


class _DeviceArray:
    """__cuda_array_interface__ view of raw device memory (torch.as_tensor
    wraps it without a copy)."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 2, "strides": None}


def _wrap_device(ptr, shape, dtype, device):
    import torch
    if int(np.prod(shape)) == 0:
        return torch.empty(shape, dtype=dtype, device=device)
    typestr = {torch.float32: "<f4", torch.uint8: "|u1", torch.int64: "<i8"}[dtype]
    return torch.as_tensor(_DeviceArray(ptr, shape, typestr), device=device)


def device_results(ctx, device=None):
    """(keypoints (n, 5) f32, descriptors (n, 128) u8) torch tensors on the
    context's GPU over the results of its last sift_batch_device(...,
    fetch=False) call -- every frame's keypoints and descriptors in frame
    order (sift_mi_device_results), wrapped without a copy; valid until the
    context's next call."""
    import torch
    kp, desc, n = ctx.device_results()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    return _wrap_device(kp, (n, 5), torch.float32, dev), _wrap_device(desc, (n, 128), torch.uint8, dev)


def gather_device_results(keypoints, descriptors, offsets, dist, dst=0):
    """Gather every rank's results -- (keypoints (n, 5) f32, descriptors
    (n, 128) u8) tensors, e.g. `device_results(ctx)`, and the per-frame
    offsets (m + 1,) of its frames -- on rank `dst`, concatenated in rank
    (= global frame) order.

    Sizes are all-gathered first; then every other rank sends its exact rows
    (raw bits) and rank `dst` receives them straight into its slice of the
    concatenated output (one batch of point-to-point ops: RCCL send/recv over
    xGMI on the nccl backend, device memory end to end; on gloo the tensors
    travel through host memory).  Returns (keypoints, descriptors, offsets)
    tensors on `dst` -- on the GPU for nccl -- and None elsewhere.
    """
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = _device(dist)
    kps = keypoints.reshape(-1, 5).view(torch.int32)
    desc = descriptors.reshape(-1, 128)
    offs = torch.as_tensor(np.asarray(offsets, dtype=np.int64))
    n, m = kps.shape[0], offs.numel() - 1
    if desc.shape[0] != n or int(offs[-1] - offs[0]) != n:
        raise ValueError("keypoints / descriptors / offsets disagree")
    kps, desc, offs = kps.to(dev), desc.to(dev), (offs - offs[0]).to(dev)
    sizes = torch.tensor([n, m], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes)
    ns = [int(x[0]) for x in all_sizes]
    ms = [int(x[1]) for x in all_sizes]
    ops = []
    if rank == dst:
        K = torch.empty((sum(ns), 5), dtype=torch.int32, device=dev)
        D = torch.empty((sum(ns), 128), dtype=torch.uint8, device=dev)
        O = [torch.empty(ms[r] + 1, dtype=torch.int64, device=dev) for r in range(world)]
        start = 0
        for r in range(world):
            k, d = K[start:start + ns[r]], D[start:start + ns[r]]
            if r == dst:
                k.copy_(kps)
                d.copy_(desc)
                O[r].copy_(offs)
            else:
                ops.append(dist.P2POp(dist.irecv, O[r], r))
                if ns[r]:
                    ops += [dist.P2POp(dist.irecv, k, r), dist.P2POp(dist.irecv, d, r)]
            start += ns[r]
    else:
        ops.append(dist.P2POp(dist.isend, offs, dst))
        if n:
            ops += [dist.P2POp(dist.isend, kps.contiguous(), dst), dist.P2POp(dist.isend, desc.contiguous(), dst)]
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    if rank != dst:
        return None
    base, parts = 0, [torch.zeros(1, dtype=torch.int64, device=dev)]
    for r in range(world):
        parts.append(O[r][1:] + base)
        base += ns[r]
    return K.view(torch.float32), D, torch.cat(parts)


def merge_bands(parts):
    """Merge per-band results [(keypoints (n,5) f32, descriptors (n,128) u8,
    emission keys (n,) u64), ...] into one frame's result in the reference's
    emission order (ascending key; src/lib.rs:281-294, :397-431).  Keys are
    unique per keypoint, so the order is total; a key seen twice means two
    bands overlapped and raises."""
    kps = np.concatenate([np.asarray(p[0], np.float32).reshape(-1, 5) for p in parts])
    desc = np.concatenate([np.asarray(p[1], np.uint8).reshape(-1, 128) for p in parts])
    keys = np.concatenate([np.asarray(p[2], np.uint64).reshape(-1) for p in parts])
    if not (len(kps) == len(desc) == len(keys)):
        raise ValueError("keypoints / descriptors / keys disagree")
    order = np.argsort(keys, kind="stable")
    keys = keys[order]
    if len(keys) > 1 and np.any(keys[1:] == keys[:-1]):
        raise ValueError("duplicate emission key: bands overlap")
    return kps[order], desc[order], keys


def allgather_bands(keypoints, descriptors, keys, dist):
    """All-gather every rank's band result (sizes first, then one padded
    all_gather per array, raw bits) and merge them; every rank gets the
    whole frame's (keypoints, descriptors, keys)."""
    import torch
    world = dist.get_world_size()
    dev = _device(dist)
    kps = np.ascontiguousarray(keypoints, dtype=np.float32).reshape(-1, 5)
    desc = np.ascontiguousarray(descriptors, dtype=np.uint8).reshape(-1, 128)
    key = np.ascontiguousarray(keys, dtype=np.uint64).reshape(-1)
    n = len(kps)
    if len(desc) != n or len(key) != n:
        raise ValueError("keypoints / descriptors / keys disagree")
    size = torch.tensor([n], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(size) for _ in range(world)]
    dist.all_gather(sizes, size)
    ns = [int(s.item()) for s in sizes]
    n_max = max(max(ns), 1)

    def padded(a, dtype):
        t = torch.zeros((n_max,) + a.shape[1:], dtype=dtype, device=dev)
        if len(a):
            t[: len(a)] = torch.from_numpy(a).to(dev)
        return t

    gathered = {}
    for name, t in (("kps", padded(kps.view(np.int32), torch.int32)), ("desc", padded(desc, torch.uint8)),
                    ("keys", padded(key.view(np.int64), torch.int64))):
        lst = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(lst, t)
        gathered[name] = [x.cpu().numpy() for x in lst]
    parts = [(gathered["kps"][r][: ns[r]].view(np.float32), gathered["desc"][r][: ns[r]],
              gathered["keys"][r][: ns[r]].view(np.uint64)) for r in range(world)]
    return merge_bands(parts)


def sift_row_bands(ctx, img, dist=None, band=None, n_bands=None):
    """sift() of ONE frame split across ranks by row bands (see the module
    docstring).  With `dist` initialised, the band is (rank, world) and the
    merged whole-frame SiftResult is returned on every rank; without it,
    `band` / `n_bands` select one band and that band's SiftResult (with keys)
    is returned for the caller to merge (merge_bands)."""
    if dist is not None and dist.is_initialized():
        band, n_bands = dist.get_rank(), dist.get_world_size()
    elif band is None or n_bands is None:
        band, n_bands = 0, 1
    ctx.set_row_band(band, n_bands)
    try:
        r = ctx.sift(img)
    finally:
        ctx.set_row_band(0, 1)
    if dist is None or not dist.is_initialized() or n_bands == 1:
        return r
    return type(r)(*allgather_bands(r.keypoints_array, r.descriptors, r.keys, dist))  # a SiftResult
