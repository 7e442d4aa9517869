"""The fused blur-5 + extremum-scan pass (k_blur_detect, detect.hip) against
the oracle.

The batch path runs each octave's blur 5 (G_4 -> G_5) and the octave's
point_is_local_extremum scan (src/lib.rs:437-506) as one kernel; these tests
pin both of its outputs:
  * G_5 (and every other plane) of the batch path's own pyramid, read back
    from the context's arena after a single-chunk call
    (sift_mi_read_batch_scale_space), bit-identical to the oracle's
    build_gaussian_scale_space (src/lib.rs:213-267);
  * the keypoints of the same calls against the oracle with the fused pass
    on (forced onto every octave it applies to, at 32-row segments:
    path option fused_detect = 2), in its one-column (k_blur_detect) and
    two-strips-per-lane (k_blur_detect_pair, path option bd_pair) forms, and
    off (fused_detect = 0: launch_blur + k_detect_rows), across frame shapes that exercise partial strips, short
    row segments, reflect-101 / clamp-to-edge borders and both profiles, and
    white noise (dense extrema, plateaus).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = ["640x480", "301x207", "1000x333", "90x700", "2000x40", "97x61"]


def _frame(name, seed=7):
    import synth
    if name == "noise":
        return np.random.default_rng(5).integers(0, 256, (96, 128), dtype=np.uint8)
    w, h = map(int, name.split("x"))
    return synth.frame(w, h, seed)


MODES = {"pair": dict(fused_detect=2, bd_pair=1), "pair_u1": dict(fused_detect=2, bd_pair=2),
         "single": dict(fused_detect=2, bd_pair=0),
         "apart": dict(fused_detect=0)}


def _context(pkg, profile, mode):
    c = pkg.Context(0, pkg.OpenCVProcessing if profile == 0 else pkg.ImageprocProcessing)
    for k, v in MODES[mode].items():
        c.set_path_option(k, v)
    return c


@pytest.mark.parametrize("fused", list(MODES))
@pytest.mark.parametrize("profile", [0, 1])
@pytest.mark.parametrize("name", SHAPES)
def test_batch_pyramid_bit_exact(pkg, oracle, fused, profile, name):
    """Every Gaussian plane the batch path leaves in its arena (G_5 from
    k_blur_detect / k_blur_detect_pair when fused) equals the oracle's, bit
    for bit."""
    img = _frame(name)
    c = _context(pkg, profile, fused)
    c.sift(img)
    opy = oracle.Pyramid(img, profile)
    for o in range(opy.n_octaves):
        go = opy.scale_space(o)
        g = c.read_batch_scale_space(0, o, (go.shape[2], go.shape[1]))
        assert np.array_equal(g, go), (o, [s for s in range(6) if not np.array_equal(g[s], go[s])],
                                       np.argwhere(g != go)[:5])
    c.close()


@pytest.mark.parametrize("fused", list(MODES))
@pytest.mark.parametrize("profile", [0, 1])
@pytest.mark.parametrize("name", SHAPES + ["noise"])
def test_fused_detect_parity(pkg, oracle, fused, profile, name):
    """Keypoints (count, emission order, values) and descriptors vs the
    oracle with and without the fused pass."""
    from test_gpu_parity import assert_parity
    img = _frame(name)
    c = _context(pkg, profile, fused)
    res = c.sift(img)
    c.close()
    kp_o, desc_o, ext_o = oracle.sift(img, profile=profile, internal=True)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


@pytest.mark.parametrize("pair", [2, 1, 0])
def test_batch_pyramid_multi_frame(pkg, oracle, pair):
    """Frames of one chunk (the fused pass's frame index and image stride):
    every frame's planes of a 5-frame single-chunk batch equal the oracle's."""
    import synth
    fr = synth.frames(5, 320, 240, seed0=21)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    c.set_path_option("fused_detect", 2)
    c.set_path_option("bd_pair", pair)
    c.set_chunk(5)
    got = c.sift_batch(fr)
    for i in (0, 2, 4):
        opy = oracle.Pyramid(fr[i], 0)
        for o in range(opy.n_octaves):
            go = opy.scale_space(o)
            g = c.read_batch_scale_space(i, o, (go.shape[2], go.shape[1]))
            assert np.array_equal(g, go), (i, o)
    ref = [c.sift(f) for f in fr]
    assert all(a == b for a, b in zip(got, ref))
    c.close()


def test_read_batch_scale_space_state(pkg):
    """The read-back is refused when the last call ran as several chunks, and
    after any later call (a precompute rewrites the arena: ADVICE r04); a
    frame past the chunk and dims that are not the octave's are rejected."""
    import synth
    fr = synth.frames(4, 96, 64, seed0=3)
    c = pkg.Context(0, pkg.OpenCVProcessing)
    c.set_path_option("chunk_mode", 0)
    c.sift_batch(fr)  # auto chunking (mode 0): two chunks over both lanes
    with pytest.raises(pkg.SiftMiError):
        c.read_batch_scale_space(0, 0, (192, 128))
    c.sift(fr[0])
    assert c.read_batch_scale_space(0, 0, (192, 128)).shape == (6, 128, 192)
    assert c.read_batch_scale_space(0, 1).shape == (6, 64, 96)
    with pytest.raises(ValueError):
        c.read_batch_scale_space(0, 0, (96, 64))
    with pytest.raises(pkg.SiftMiError):
        c.read_batch_scale_space(1, 0)
    c.set_chunk(4)
    c.sift_batch(fr)  # one chunk of 4 frames
    assert c.read_batch_scale_space(3, 0).shape == (6, 128, 192)
    c.precompute_images(synth.frame(48, 40, 1))  # other size: the plan is rebuilt
    with pytest.raises(pkg.SiftMiError):
        c.read_batch_scale_space(3, 0)
    c.sift_batch(fr)
    c.precompute_images(fr[1])  # same size: arena 0 rewritten in place
    with pytest.raises(pkg.SiftMiError):
        c.read_batch_scale_space(0, 0)
    c.close()

