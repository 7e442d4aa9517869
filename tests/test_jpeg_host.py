"""JPEG input step, host side (no GPU): sift_mi_jpeg_dims parses the headers
of the reference's test JPEGs and of PIL-encoded files, and rejects what the
decoder does not support (progressive) or what is not a JPEG."""
import io
import os

import numpy as np
import pytest
from conftest import GOLDEN, load_golden

JPEG = os.path.join(GOLDEN, "jpeg")


@pytest.mark.parametrize("name", ["tree_small", "bird_small", "bird"])
def test_dims_of_reference_images(pkg, name):
    data = open(os.path.join(JPEG, name + ".jpg"), "rb").read()
    h, w = load_golden(name)["image"].shape
    assert pkg.jpeg_dims(data) == (w, h)


def test_dims_pil_and_rejections(pkg):
    from PIL import Image
    img = Image.fromarray(np.zeros((21, 37, 3), np.uint8))
    b = io.BytesIO()
    img.save(b, "JPEG")
    assert pkg.jpeg_dims(b.getvalue()) == (37, 21)
    p = io.BytesIO()
    img.save(p, "JPEG", progressive=True)
    with pytest.raises(pkg.SiftMiError):  # SOF2: progressive is not decoded
        pkg.jpeg_dims(p.getvalue())
    with pytest.raises(pkg.SiftMiError):
        pkg.jpeg_dims(b"\x89PNG\r\n\x1a\n" + b"\0" * 32)


def test_truncated_sos_rejected(pkg):
    """An SOS segment shorter than its component list (T.81 B.2.3) at the end
    of the buffer is rejected, not read past."""
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, "JPEG")
    data = b.getvalue()
    p = data.index(b"\xff\xda")
    assert pkg.jpeg_dims(data) == (16, 16)
    with pytest.raises(pkg.SiftMiError):
        pkg.jpeg_dims(data[:p] + b"\xff\xda\x00\x03\x03")  # Ns = 3, no component specs
