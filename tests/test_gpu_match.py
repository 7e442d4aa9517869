"""Descriptor matching (examples/sift-match.rs:30-35: cv::BFMatcher(NORM_L2,
crossCheck).match) on the MFMA units vs the CPU oracle: identical query /
train indices (lowest index on ties) and bit-identical f32 distances."""
import numpy as np
import pytest
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _check(ctx, oracle, q, t, cross):
    gq, gt, gd = ctx.match_descriptors(q, t, cross_check=cross)
    oq, ot, od = oracle.match(q, t, cross_check=cross)
    assert np.array_equal(gq, oq) and np.array_equal(gt, ot), (len(gq), len(oq))
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))
    return len(gq)


@pytest.mark.parametrize("nq,nt", [(1, 1), (37, 300), (128, 128), (257, 129), (1000, 700)])
@pytest.mark.parametrize("cross", [True, False])
def test_match_random(ctx, oracle, nq, nt, cross):
    rng = np.random.default_rng(nq * 7 + nt)
    q = rng.integers(0, 256, (nq, 128), dtype=np.uint8)
    t = rng.integers(0, 256, (nt, 128), dtype=np.uint8)
    t[: min(nq, nt) // 3] = q[: min(nq, nt) // 3]  # exact duplicates: distance 0
    _check(ctx, oracle, q, t, cross)


def test_match_ties_lowest_index(ctx, oracle):
    """Equal distances resolve to the lowest index (OpenCV's strict <)."""
    rng = np.random.default_rng(9)
    base = rng.integers(0, 200, (50, 128), dtype=np.uint8)
    t = np.concatenate([base, base, base])  # every train row appears 3 times
    q = base[::-1].copy()
    n = _check(ctx, oracle, q, t, True)
    assert n == 50
    gq, gt, gd = ctx.match_descriptors(q, t)
    assert np.all(gt < 50) and np.all(gd == 0)


def test_match_real_descriptors(pkg, ctx, oracle):
    """sift-match.rs flow: descriptors of two images (the OpenCV profile)."""
    a = ctx.sift(load_golden("bird_small")["image"])
    b = ctx.sift(load_golden("bird")["image"])
    n = _check(ctx, oracle, b.descriptors, a.descriptors, True)
    assert n > 20
    _check(ctx, oracle, a.descriptors, b.descriptors, False)


def test_match_empty(ctx):
    e = np.zeros((0, 128), np.uint8)
    x = np.ones((5, 128), np.uint8)
    for q, t in [(e, x), (x, e), (e, e)]:
        gq, gt, gd = ctx.match_descriptors(q, t)
        assert len(gq) == 0
