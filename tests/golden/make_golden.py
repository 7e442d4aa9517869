"""Generate the committed golden fixtures from the reference's own test data.

Run ONLY in the build container (it reads /root/reference, which does not
exist on the GPU box).  Outputs are plain data (npz: inputs + expected
outputs); no reference source is copied.

Sources (reference @ /root/reference):
  * src/snapshots/sift__sift_end2end{,-2,-3,-4}.snap  -- insta YAML written by
    the `sift_end2end` test (src/lib.rs:1009-1056): keypoints {x,y,size,angle,
    response} and u8x128 descriptors for tree_small.jpg and bird_small.jpg,
    already stably sorted by (x, y, size) (src/lib.rs:1020-1030).
  * images/*.jpg -- the test inputs (src/lib.rs:1038, :1047).  The reference
    decodes them with `image::load_from_memory(..).grayscale()` (image 0.25.2,
    whose JPEG backend is zune-jpeg; luma = (2126 R + 7152 G + 722 B) / 10000,
    integer division).  zune-jpeg is not in /root/reference, so the inputs are
    decoded here by tests/golden/jpeg_decode.py with the reconstruction
    arithmetic that reproduces the snapshots (selected by matching them; see
    DESIGN.md, "Oracle"):  idct="zune" (stb_image 12-bit integer IDCT with the
    row-pass bias 512 + 65536 + (128 << 17) and the DC-only shortcut
    (DC >> 3) + 128), upsample="twopass" (vertical then horizontal 3:1
    triangle, each (3a + b + 2) >> 2), color="zune" (45/32, 11/32, 23/32,
    113/64 fixed point), edge="pad".  With these inputs the oracle finds the
    snapshots' exact keypoint counts (1270, 225) with 96-99 % of keypoints at
    identical positions.  The same decoder with the libjpeg arithmetic
    reproduces PIL (libjpeg-turbo) bit-exactly on these files (checked below),
    which validates its entropy decoding.

Usage:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
from PIL import Image

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def parse_keypoints(path):
    rows, cur = [], {}
    body = open(path).read().split("---\n", 2)[2]
    for line in body.splitlines():
        line = line.strip()
        if not line:
            continue
        if line.startswith("- "):
            if cur:
                rows.append(cur)
            cur = {}
            line = line[2:]
        k, v = line.split(":", 1)
        cur[k.strip()] = np.float32(v.strip())
    if cur:
        rows.append(cur)
    cols = ["x", "y", "size", "angle", "response"]
    return np.array([[r[c] for c in cols] for r in rows], dtype=np.float32)


def parse_descriptors(path):
    rows, cur = [], None
    body = open(path).read().split("---\n", 2)[2]
    for line in body.splitlines():
        if line.startswith("- - "):
            if cur is not None:
                rows.append(cur)
            cur = [int(line[4:])]
        elif line.startswith("  - "):
            cur.append(int(line[4:]))
        elif line.strip():
            raise ValueError(line)
    if cur is not None:
        rows.append(cur)
    arr = np.array(rows, dtype=np.int64)
    assert arr.shape[1] == 128 and arr.min() >= 0 and arr.max() <= 255
    return arr.astype(np.uint8)


sys.path.insert(0, HERE)
import jpeg_decode  # noqa: E402

ZUNE = dict(idct="zune", upsample="twopass", color="zune", edge="pad")


def decode_gray(path):
    # entropy-decoding check: the libjpeg arithmetic must reproduce PIL exactly
    pil = np.asarray(Image.open(path).convert("RGB"))
    ours = jpeg_decode.decode(path, idct="islow", upsample="libjpeg", color="libjpeg", edge="clamp")
    assert np.array_equal(pil, ours), "jpeg_decode does not reproduce libjpeg-turbo"
    return jpeg_decode.luma(jpeg_decode.decode(path, **ZUNE))


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not mounted; fixtures are already committed")
    snap = os.path.join(REF, "src", "snapshots")
    cases = {
        "tree_small": ("sift__sift_end2end.snap", "sift__sift_end2end-2.snap"),
        "bird_small": ("sift__sift_end2end-3.snap", "sift__sift_end2end-4.snap"),
    }
    for name, (kf, df) in cases.items():
        kps = parse_keypoints(os.path.join(snap, kf))
        desc = parse_descriptors(os.path.join(snap, df))
        assert len(kps) == len(desc)
        img = decode_gray(os.path.join(REF, "images", name + ".jpg"))
        np.savez_compressed(os.path.join(HERE, name + ".npz"),
                            image=img, keypoints=kps, descriptors=desc)
        print(name, img.shape, kps.shape, desc.shape)
    # extra real-content input without expected outputs (GPU-vs-oracle parity)
    img = decode_gray(os.path.join(REF, "images", "bird.jpg"))
    np.savez_compressed(os.path.join(HERE, "bird.npz"), image=img)
    print("bird", img.shape)


if __name__ == "__main__":
    main()
