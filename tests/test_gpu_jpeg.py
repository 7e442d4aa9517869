"""JPEG input step on the GPU: sift_mi_decode_jpeg
against the restatement tests/golden/jpeg_decode.py with zune-jpeg's
arithmetic (the decode that reproduces the reference's snapshots,
tests/golden/make_golden.py), bit for bit.

* The reference's own test JPEGs decode to exactly the golden fixtures'
  input images, so JPEG bytes -> keypoints through this path reproduces the
  snapshot-pinned inputs (and the oracle's keypoints on them).
* PIL-encoded files cover 4:4:4 / 4:2:2 / 4:2:0 chroma, grayscale JPEGs,
  odd sizes (partial MCUs) and restart intervals.
"""
import io
import os
import sys

import numpy as np
import pytest
from conftest import GOLDEN, load_golden

pytestmark = pytest.mark.gpu
JPEG = os.path.join(GOLDEN, "jpeg")
sys.path.insert(0, GOLDEN)
ZUNE = dict(idct="zune", upsample="twopass", color="zune", edge="pad")


def _reference_decode(data, tmp_path):
    import jpeg_decode
    f = tmp_path / "x.jpg"
    f.write_bytes(data)
    out = jpeg_decode.decode(str(f), **ZUNE)
    return out if out.ndim == 2 else jpeg_decode.luma(out)


@pytest.mark.parametrize("name", ["tree_small", "bird_small", "bird"])
def test_reference_images_decode_to_golden(ctx, name):
    data = open(os.path.join(JPEG, name + ".jpg"), "rb").read()
    got = ctx.decode_jpeg(data)
    assert np.array_equal(got, load_golden(name)["image"])


def test_jpeg_to_keypoints_matches_oracle(pkg, ctx, oracle):
    """examples/run-sift.rs: sift(image::open(path).grayscale()) from bytes."""
    from test_gpu_parity import assert_parity
    data = open(os.path.join(JPEG, "tree_small.jpg"), "rb").read()
    res = ctx.sift_jpeg(data)
    kp_o, desc_o, ext_o = oracle.sift(load_golden("tree_small")["image"], internal=True)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


def _pil_jpeg(shape, seed, mode="RGB", **kw):
    from PIL import Image
    import synth
    h, w = shape
    base = synth.frame(w, h, seed)
    if mode == "RGB":
        rng = np.random.default_rng(seed)
        arr = np.stack([base, np.roll(base, 3, 1), 255 - base], -1).astype(np.int16)
        arr = np.clip(arr + rng.integers(-20, 21, arr.shape), 0, 255).astype(np.uint8)
    else:
        arr = base
    b = io.BytesIO()
    Image.fromarray(arr, mode).save(b, "JPEG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("shape,kw", [
    ((64, 64), dict(quality=90, subsampling=0)),
    ((61, 93), dict(quality=85, subsampling=1)),
    ((97, 131), dict(quality=75, subsampling=2)),
    ((240, 320), dict(quality=95, subsampling=2, restart_marker_blocks=7)),
    ((123, 77), dict(quality=60, subsampling=0, restart_marker_rows=1)),
    ((270, 480), dict(quality=90, subsampling=2)),
])
def test_pil_color_jpegs(ctx, tmp_path, shape, kw):
    data = _pil_jpeg(shape, sum(shape), **kw)
    got = ctx.decode_jpeg(data)
    assert got.shape == shape
    assert np.array_equal(got, _reference_decode(data, tmp_path))


@pytest.mark.parametrize("shape", [(8, 8), (33, 17), (200, 301)])
def test_pil_gray_jpegs(ctx, tmp_path, shape):
    data = _pil_jpeg(shape, 5, mode="L", quality=88)
    got = ctx.decode_jpeg(data)
    assert np.array_equal(got, _reference_decode(data, tmp_path))


def test_decode_to_device(ctx):
    import torch
    data = open(os.path.join(JPEG, "bird_small.jpg"), "rb").read()
    ref = load_golden("bird_small")["image"]
    h, w = ref.shape
    t = torch.zeros((h, w + 5), dtype=torch.uint8, device="cuda")
    ctx.decode_jpeg_device(data, t.data_ptr(), t.stride(0))
    torch.cuda.synchronize()
    assert np.array_equal(t[:, :w].cpu().numpy(), ref)
    assert int(t[:, w:].sum()) == 0  # the stride padding is untouched


def test_batch_decode_to_device(pkg, ctx):
    """sift_mi_decode_jpeg_batch (threaded entropy decoding, chunked uploads)
    equals per-frame decoding, in the device layout sift_batch_device reads,
    and the keypoints of the decoded batch equal per-frame sift()."""
    import torch
    datas = [_pil_jpeg((90, 120), 40 + i, quality=80 + i, subsampling=2) for i in range(37)]
    h, w = 90, 120
    t = torch.zeros((len(datas), h, w + 8), dtype=torch.uint8, device="cuda")
    ctx.decode_jpeg_batch_device(datas, t.data_ptr(), t.stride(0), t.stride(1), threads=4)
    torch.cuda.synchronize()
    got = t[:, :, :w].cpu().numpy()
    for i, d in enumerate(datas):
        assert np.array_equal(got[i], ctx.decode_jpeg(d)), i
    offs, res = ctx.sift_batch_device(t.data_ptr(), len(datas), w, h, t.stride(1), t.stride(0), fetch=True)
    for i in (0, 17, 36):
        single = ctx.sift(got[i])
        a, b = int(offs[i]), int(offs[i + 1])
        assert np.array_equal(res.keypoints_array[a:b], single.keypoints_array)
    with pytest.raises(pkg.SiftMiError):  # frames of different sizes
        ctx.decode_jpeg_batch_device([datas[0], _pil_jpeg((91, 120), 1)], t.data_ptr(), t.stride(0), t.stride(1))
