"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 path
(sift-features_amd/shard.py, bench.py --gpus N): frame sharding, the
max-over-ranks / summed reporting, and the keypoint gather."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_result(rank, frames):
    """Deterministic per-rank result: frame f of rank r has 3 + f + r keypoints."""
    rng = np.random.default_rng(100 + rank)
    counts = [3 + f + rank for f in range(frames)]
    n = sum(counts)
    kps = rng.standard_normal((n, 5)).astype(np.float32)
    if n and rank % 2 == 1:
        kps[0, 0] = np.float32(np.nan)  # bit-exact transport, NaN included
    desc = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return kps, desc, offs


def _worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "sift-features_amd"))
    import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, stop = shard.shard_range(10, rank, world)
        kps, desc, offs = _fake_result(rank, stop - start)
        t, nk, nf = shard.reduce_run(0.5 + rank, len(kps), stop - start, dist)
        g = shard.gather_results(kps, desc, offs, dist, dst=0)
        if rank == 0:
            q.put(("ok", (start, stop), (t, nk, nf), g))
        else:
            q.put(("ok", (start, stop), (t, nk, nf), None))
    except Exception as e:  # pragma: no cover - surfaced by the assert below
        q.put(("err", repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_shard_reduce_gather():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(r[0] == "ok" for r in res), res
    ranges = sorted(r[1] for r in res)
    assert ranges == [(0, 5), (5, 10)]
    for r in res:
        t, nk, nf = r[2]
        assert t == 1.5  # max over ranks
        assert nf == 10
        assert nk == sum(3 + f for f in range(5)) + sum(4 + f for f in range(5))
    g = next(r[3] for r in res if r[3] is not None)
    kps, desc, offs = g
    k0, d0, o0 = _fake_result(0, 5)
    k1, d1, o1 = _fake_result(1, 5)
    assert np.array_equal(kps.view(np.uint32), np.concatenate([k0, k1]).view(np.uint32))
    assert np.array_equal(desc, np.concatenate([d0, d1]))
    assert np.array_equal(offs, np.concatenate([o0, o1[1:] + o0[-1]]))


def _dev_worker(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "sift-features_amd"))
    import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = [4, 0, 3][rank]  # rank 1 has no frames at all
        kps, desc, offs = _fake_result(rank, frames)
        g = shard.gather_device_results(torch.from_numpy(kps), torch.from_numpy(desc), offs, dist, dst=0)
        q.put(("ok", rank, None if g is None else tuple(t.numpy() for t in g)))
    except Exception as e:  # pragma: no cover - surfaced by the assert below
        q.put(("err", rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world3_gather_device_results():
    """shard.gather_device_results (the bench's N > 1 gather: sizes, then
    point-to-point rows into rank 0's concatenated output) on gloo with three
    ranks, one of them empty: exact bits (NaN included) in frame order."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dev_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(3)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(r[0] == "ok" for r in res), res
    kps, desc, offs = next(r[2] for r in res if r[1] == 0)
    parts = [_fake_result(r, [4, 0, 3][r]) for r in range(3)]
    assert np.array_equal(kps.view(np.uint32), np.concatenate([p[0] for p in parts]).view(np.uint32))
    assert np.array_equal(desc, np.concatenate([p[1] for p in parts]))
    want, base = [0], 0
    for p in parts:
        want += (p[2][1:] + base).tolist()
        base += len(p[0])
    assert np.array_equal(offs, np.asarray(want))
    assert all(r[2] is None for r in res if r[1] != 0)


def test_shard_range_partition():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "sift-features_amd"))
    import shard
    for n in (0, 1, 7, 8, 128, 1023):
        for w in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(4, 2, 2)


# ---------------------------------------------------------------------------
# row bands of one frame (shard.merge_bands / allgather_bands): SURVEY 8(f) row 4
# ---------------------------------------------------------------------------
def _shard_mod():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "sift-features_amd"))
    import shard
    return shard


def _fake_frame(n=300, seed=5):
    """A whole frame's result in emission order: unique ascending keys."""
    rng = np.random.default_rng(seed)
    keys = np.sort(rng.choice(np.uint64(1) << np.uint64(40), n, replace=False).astype(np.uint64))
    kps = rng.standard_normal((n, 5)).astype(np.float32)
    desc = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    return kps, desc, keys


def _split(kps, desc, keys, world, seed=9):
    """Random disjoint partition into `world` bands (each band keeps its own
    emission order, as one context's result does)."""
    owner = np.random.default_rng(seed).integers(0, world, len(keys))
    return [(kps[owner == r], desc[owner == r], keys[owner == r]) for r in range(world)]


def test_merge_bands_restores_emission_order():
    shard = _shard_mod()
    kps, desc, keys = _fake_frame()
    for world in (1, 2, 3, 8):
        parts = _split(kps, desc, keys, world)
        k, d, y = shard.merge_bands(parts)
        assert np.array_equal(y, keys)
        assert np.array_equal(k.view(np.uint32), kps.view(np.uint32))
        assert np.array_equal(d, desc)
    # empty bands and an empty frame
    k, d, y = shard.merge_bands([(kps[:0], desc[:0], keys[:0])] * 3)
    assert len(k) == len(d) == len(y) == 0
    parts = _split(kps, desc, keys, 2)
    with pytest.raises(ValueError):  # overlapping bands
        shard.merge_bands(parts + [parts[0]])


def _band_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "sift-features_amd"))
    import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kps, desc, keys = _fake_frame()
        mine = _split(kps, desc, keys, world)[rank]
        q.put(("ok", rank, shard.allgather_bands(*mine, dist)))
    except Exception as e:  # pragma: no cover - surfaced by the assert below
        q.put(("err", rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_allgather_bands():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert all(r[0] == "ok" for r in res), res
    kps, desc, keys = _fake_frame()
    for _, _, (k, d, y) in res:  # every rank holds the whole frame
        assert np.array_equal(y, keys)
        assert np.array_equal(k.view(np.uint32), kps.view(np.uint32))
        assert np.array_equal(d, desc)
