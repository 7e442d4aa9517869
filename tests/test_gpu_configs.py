"""The BASELINE.json configs on the HIP path, checked against the oracle.

* config #2: one 1920x1080 frame, `sift()` vs the oracle directly;
* config #3: 256 x 640x480 frames through the device-resident batch path
  (`sift_batch_device(..., fetch=False)`: one chunk of 256 under the default
  automatic chunking, or -- chunk_mode 0 -- 2 chunks of 128 over both
  pipeline lanes), frames spread over the chunks (the last included) vs the
  oracle, every frame vs per-frame `sift()`;
* chunks of more than 64 frames with a features_limit (the per-frame output
  plan is one 256-thread workgroup, k_limit_plan);
* config #4, one GPU's shard: bench.py's exact call (128 x 1920x1080, auto
  chunks -- one of 128, or two of 64 under chunk_mode 0 -- results kept in
  HBM), 2 frames vs the oracle, every frame vs per-frame `sift()`;
* the stage-bound overflow re-run (host.cpp finalize_chunk rc == 1): with
  path option bound_shrink every chunk enqueued before a high-water mark exists
  overflows; the re-run chunks must equal per-frame results.
Configs #1 (bird_small) and #5 (8192^2) are covered by test_gpu_parity /
test_oracle_golden and test_gpu_large.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device_results(ctx, n):
    kp_ptr, desc_ptr, m = ctx.device_results()
    assert m == n
    kp = np.empty((n, 5), np.float32)
    desc = np.empty((n, 128), np.uint8)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    if n:
        assert hip.hipMemcpy(kp.ctypes.data, kp_ptr, kp.nbytes, 2) == 0  # hipMemcpyDeviceToHost
        assert hip.hipMemcpy(desc.ctypes.data, desc_ptr, desc.nbytes, 2) == 0
    return kp, desc


def _parity_rows(kp, desc, kp_o, desc_o):
    """assert_parity on (keypoints, descriptors) rows without keys."""
    from test_gpu_parity import TOL_ANGLE, TOL_RESP, TOL_XY
    assert len(kp) == len(kp_o), (len(kp), len(kp_o))
    d = np.abs(kp - kp_o)
    assert d[:, :3].max() <= TOL_XY, d.max(0)
    dang = np.abs(((kp[:, 3] - kp_o[:, 3]) + 180.0) % 360.0 - 180.0)
    assert dang.max() <= TOL_ANGLE
    assert d[:, 4].max() <= TOL_RESP
    dd = np.abs(desc.astype(np.int32) - desc_o.astype(np.int32))
    assert dd.max() <= 1 and (dd == 0).mean() >= 0.99


def _device_batch(pkg, frames_t, ctx=None):
    c = ctx or pkg.Context(0, pkg.OpenCVProcessing)
    n, h, w = frames_t.shape
    offs, res = c.sift_batch_device(frames_t.data_ptr(), n, w, h, frames_t.stride(1), frames_t.stride(0),
                                    fetch=False)
    assert res is None
    kp, desc = _device_results(c, int(offs[-1]))
    return c, offs, kp, desc


def test_config2_single_1080p(pkg, ctx, oracle):
    import synth
    from test_gpu_parity import assert_parity
    img = synth.frame(1920, 1080, 0)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    res = ctx.sift(img)
    assert len(res) > 5000
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


@pytest.mark.parametrize("chunk_mode", [1, 0])
def test_config3_vga_256_device(pkg, ctx, oracle, chunk_mode):
    import synth
    import torch
    t = synth.frames_torch(256, 640, 480, seed0=0, device="cuda")
    torch.cuda.synchronize()
    host = t.cpu().numpy()
    c = pkg.Context(0, pkg.OpenCVProcessing)
    c.set_path_option("chunk_mode", chunk_mode)
    c, offs, kp, desc = _device_batch(pkg, t, c)
    st = c.stats()
    assert st["frames"] == 256
    c.close()
    assert np.all(np.diff(offs) > 0)
    for i in (0, 63, 64, 127, 128, 200, 255):  # both 128-frame chunks (mode 0: lanes), the last frame
        a, b = int(offs[i]), int(offs[i + 1])
        kp_o, desc_o = oracle.sift(host[i])
        _parity_rows(kp[a:b], desc[a:b], kp_o, desc_o)
    for i in range(256):
        a, b = int(offs[i]), int(offs[i + 1])
        r = ctx.sift(host[i])
        assert np.array_equal(kp[a:b].view(np.uint32), r.keypoints_array.view(np.uint32)), i
        assert np.array_equal(desc[a:b], r.descriptors), i


@pytest.mark.parametrize("chunk_mode", [1, 0])
def test_config4_bench_shard_1080p(pkg, ctx, oracle, chunk_mode):
    """bench.py's step: 128 device-resident 1080p frames, auto chunks (one
    128-frame chunk; chunk_mode 0: two 64-frame chunks, one per lane),
    results kept in the device arena."""
    import synth
    import torch
    t = synth.frames_torch(128, 1920, 1080, seed0=0, device="cuda")
    torch.cuda.synchronize()
    c = pkg.Context(0, pkg.OpenCVProcessing)
    c.set_path_option("chunk_mode", chunk_mode)
    c, offs, kp, desc = _device_batch(pkg, t, c)
    c.close()
    host = t.cpu().numpy()
    del t
    for i in (5, 127):
        a, b = int(offs[i]), int(offs[i + 1])
        kp_o, desc_o = oracle.sift(host[i])
        _parity_rows(kp[a:b], desc[a:b], kp_o, desc_o)
    for i in range(128):
        a, b = int(offs[i]), int(offs[i + 1])
        r = ctx.sift(host[i])
        assert np.array_equal(kp[a:b].view(np.uint32), r.keypoints_array.view(np.uint32)), i
        assert np.array_equal(desc[a:b], r.descriptors), i


@pytest.mark.parametrize("limit", [None, 0, 3, 40])
def test_large_chunk_features_limit(pkg, ctx, limit):
    """200 frames in one chunk: the output plan (per-frame counts, offsets,
    response truncation) covers frames past the first 64."""
    import synth
    fr = synth.frames(200, 96, 64, seed0=7)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    c.set_chunk(200)
    got = c.sift_batch(fr, features_limit=limit)
    c.close()
    ref = [ctx.sift(f, features_limit=limit) for f in fr]
    if limit is None:
        assert sum(len(r) for r in ref) > 200
    assert all(a == b for a, b in zip(got, ref))


@pytest.mark.parametrize("lanes", [1, 2])
def test_stage_bound_overflow_rerun(pkg, ctx, lanes):
    import synth
    fr = synth.frames(7, 320, 240, seed0=40)
    ref = [ctx.sift(f) for f in fr]
    c = pkg.Context(0, pkg.OpenCVProcessing)  # no high-water marks yet
    c.set_path_option("bound_shrink", 1000)
    c.set_chunk(2)
    c.set_pipeline_lanes(lanes)
    got = c.sift_batch(fr)
    st = c.stats()
    c.close()
    assert st["stage_reruns"] >= (2 if lanes == 2 else 1), st
    assert st["frames"] == 7 and st["keypoints"] == sum(len(r) for r in ref)
    assert all(a == b for a, b in zip(got, ref))


def test_stage_bound_overflow_rerun_one_frame(pkg, ctx):
    """The one-frame path (early detection, descriptors beside the ordering,
    the chunk's counters copied to the host by k_gather_out) overflows its
    first-call bounds (bound_shrink) and re-runs; the results equal a
    context's whose bounds were learned."""
    import synth
    frames = [synth.frame(640, 480, 11), synth.frame(1920, 1080, 12)]
    ref = [ctx.sift(f) for f in frames]
    for f, r in zip(frames, ref):
        c = pkg.Context(0, pkg.OpenCVProcessing)  # no high-water marks yet
        c.set_path_option("bound_shrink", 1000)
        got = c.sift(f)
        st = c.stats()
        again = c.sift(f)  # bounds learned now
        c.close()
        assert st["stage_reruns"] >= 1, st
        assert got == r and again == r
        assert np.array_equal(got.keys, r.keys)
