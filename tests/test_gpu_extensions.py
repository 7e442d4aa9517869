"""Labelled extensions and tooling around the path, on the GPU.

* `set_max_octaves` (LABELLED EXTENSION, not in the crate; for the configs'
  "5 octaves" / "7 octaves" wording): without a limit the capped result is
  exactly the uncapped result's keypoints of octaves < cap -- a prefix of the
  emission order (octave-major, src/lib.rs:281-294), since octave o's images
  depend only on octaves <= o (src/lib.rs:213-267).  With a limit, the limit
  ranks that prefix.  Checked bit for bit against the uncapped GPU result
  (itself oracle-checked in test_gpu_parity).
* sample counting (measurement only): counts are the closed-form patch sizes
  and leave the results unchanged.
* run_sift.py, the examples/run-sift.rs counterpart: prints the keypoint
  count of `sift()` on the reference's own test JPEGs, equal to the oracle's
  count on the decoded image (imageproc profile, the crate's `sift()`), and
  the snapshot counts with --processing opencv (src/snapshots: 225 / 1270).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JPEG = os.path.join(ROOT, "tests", "golden", "jpeg")


def _octaves(keys):
    return (np.asarray(keys, np.uint64) >> np.uint64(38)) & np.uint64(0xF)


@pytest.mark.parametrize("shape,cap", [((240, 320), 3), ((1080, 1920), 5), ((480, 640), 1)])
def test_max_octaves_is_a_prefix(pkg, synth, shape, cap):
    h, w = shape
    img = synth.frame(w, h, 11)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    try:
        full = c.sift(img)
        c.set_max_octaves(cap)
        capped = c.sift(img)
        c.set_max_octaves(0)
        again = c.sift(img)
    finally:
        c.close()
    octs = _octaves(full.keys)
    keep = octs < cap
    n = int(keep.sum())
    assert 0 < n < len(full)
    assert keep[:n].all() and not keep[n:].any()  # octave-major emission order
    assert len(capped) == n
    assert np.array_equal(capped.keypoints_array, full.keypoints_array[:n])
    assert np.array_equal(capped.descriptors, full.descriptors[:n])
    assert np.array_equal(again.keypoints_array, full.keypoints_array)


def test_max_octaves_batch(pkg, synth):
    frames = np.stack([synth.frame(640, 480, s) for s in range(3)])
    c = pkg.Context(0, pkg.OpenCVProcessing)
    try:
        full = c.sift_batch(frames)
        c.set_max_octaves(4)
        capped = c.sift_batch(frames)
    finally:
        c.close()
    for f, g in zip(full, capped):
        n = int((_octaves(f.keys) < 4).sum())
        assert np.array_equal(g.keypoints_array, f.keypoints_array[:n])
        assert np.array_equal(g.descriptors, f.descriptors[:n])


def test_max_octaves_with_limit(pkg, synth):
    """With features_limit the cap applies first: the result is the limit
    (response-descending stable sort, emission order on ties, then truncate;
    src/lib.rs:156-161) applied to the capped keypoint set, i.e. to the
    uncapped result's octave prefix."""
    img = synth.frame(640, 480, 5)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    try:
        full = c.sift(img)
        c.set_max_octaves(3)
        capped = c.sift(img)
        lim = c.sift(img, features_limit=40)
    finally:
        c.close()
    n = len(capped)
    assert 40 < n < len(full)
    kp = full.keypoints_array[:n]
    order = np.argsort(-kp[:, 4], kind="stable")[:40]
    assert np.array_equal(lim.keypoints_array, kp[order])
    assert np.array_equal(lim.descriptors, full.descriptors[:n][order])


def test_sample_counting(pkg, synth):
    img = synth.frame(640, 480, 3)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    try:
        ref = c.sift(img)
        c.set_sample_counting(True)
        c.reset_stats()
        res = c.sift(img)
        st = c.stats()
        c.set_sample_counting(False)
    finally:
        c.close()
    assert np.array_equal(res.keypoints_array, ref.keypoints_array)
    assert np.array_equal(res.descriptors, ref.descriptors)
    n_ext = st["extrema"]
    # every extremum's patch is (2r + 1)^2 <= 33^2 positions, r >= 1
    assert 9 * n_ext <= st["orient_samples"] <= 33 * 33 * n_ext
    # a descriptor window covers ~(5 * 3 * sigma)^2 samples, sigma >= 1.6
    assert st["desc_samples"] >= 100 * len(res)
    assert st["desc_samples"] <= 79 * 79 * len(res)


@pytest.mark.parametrize("name", ["bird_small", "tree_small"])
def test_run_sift_cli(pkg, oracle, name):
    path = os.path.join(JPEG, name + ".jpg")
    env = dict(os.environ)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "sift-features_amd", "run_sift.py"), path],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr
    c = pkg.Context(0, pkg.ImageprocProcessing)
    try:
        with open(path, "rb") as f:
            img = c.decode_jpeg(f.read())
    finally:
        c.close()
    kp_o, _ = oracle.sift(img, profile=oracle.PROFILE_IMAGEPROC)
    assert out.stdout.strip() == f"{len(kp_o)} keypoints"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "sift-features_amd", "run_sift.py"), path,
                          "--processing", "opencv"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == {"bird_small": "225 keypoints", "tree_small": "1270 keypoints"}[name]


def test_path_option_validation_and_restore(pkg):
    """sift_mi_set_path_option rejects the retired split-tail option (10) and
    out-of-range values of the round-6 options; Context.path_options()
    restores the values the options had before the block, not the defaults
    (ADVICE r05)."""
    c = pkg.Context(0)
    try:
        L = pkg.lib()
        assert L.sift_mi_set_path_option(c._h, 10, 0) != 0  # split tail: retired
        assert L.sift_mi_set_path_option(c._h, 13, 3) != 0  # bd_pair: 0..2
        assert L.sift_mi_set_path_option(c._h, 14, 100) != 0  # bd_waves: 1024..65536
        assert L.sift_mi_set_path_option(c._h, 15, 2) != 0  # chunk_mode: 0..1
        assert L.sift_mi_set_path_option(c._h, 99, 0) != 0
        c.set_path_option("graph", 1)
        c.set_path_option("bd_waves", 4096)
        with c.path_options(graph=0, bd_pair=2, bd_waves=16384):
            assert c.path_option("graph") == 0 and c.path_option("bd_pair") == 2
        assert c.path_option("graph") == 1
        assert c.path_option("bd_pair") == pkg.Context.PATH_OPTIONS["bd_pair"][1]
        assert c.path_option("bd_waves") == 4096
    finally:
        c.close()


@pytest.mark.gpu
def test_chunk_mode_results_equal(pkg):
    """Automatic chunking mode 1 (as few chunks as memory allows: the five
    640x480 frames in one chunk instead of 3 + 2 over both lanes) returns
    the same keypoints and descriptors, frame for frame."""
    import synth
    fr = synth.frames(5, 640, 480, seed0=40)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    try:
        ref = c.sift_batch(fr)
        with c.path_options(chunk_mode=1):
            got = c.sift_batch(fr)
        assert len(ref) == len(got) == 5
        for a, b in zip(ref, got):
            assert np.array_equal(a.keypoints_array, b.keypoints_array)
            assert np.array_equal(a.descriptors, b.descriptors)
    finally:
        c.close()


@pytest.mark.gpu
def test_chunk_mode1_multi_chunk_lanes(pkg, ctx):
    """Under the default automatic chunking (mode 1) a call larger than one
    chunk still splits into balanced chunks over both pipeline lanes: 300
    tiny frames exceed the 256-frame cap (two chunks of 150); every frame
    equals its per-frame sift()."""
    import synth
    fr = synth.frames(300, 64, 48, seed0=900)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    try:
        got = c.sift_batch(fr)
        st = c.stats()
    finally:
        c.close()
    assert st["frames"] == 300
    ref = [ctx.sift(f) for f in fr]
    assert all(a == b for a, b in zip(got, ref))
