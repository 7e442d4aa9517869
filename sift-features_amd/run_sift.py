"""run-sift: the counterpart of the crate's examples/run-sift.rs (BASELINE.json
configs[0]) on the MI355X path.

    python sift-features_amd/run_sift.py <image.jpg> [--processing opencv|imageproc] [--device N]

examples/run-sift.rs:5-21 opens the image (`image::open(path)?.grayscale()`),
runs `sift_features::sift(&img, None)` and prints "<n> keypoints".  Here the
JPEG is decoded by the context's decoder (host entropy decode + GPU IDCT /
colour / luma, the zune-jpeg arithmetic of image 0.25.2: jpeg.hip), and
`sift()` runs on the GPU through the C ABI.  The crate's `sift()` uses
ImageprocProcessing (src/lib.rs:71-73), the default here too;
`--processing opencv` selects the OpenCVProcessing profile the reference's
snapshot test pins (src/lib.rs:1009-1056).  Exits non-zero (with the
library's error) when the HIP library or the device is missing: there is
no CPU fallback.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="run-sift", description=__doc__.split("\n\n")[0])
    ap.add_argument("path")
    ap.add_argument("--processing", choices=("imageproc", "opencv"), default="imageproc")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    import pkg_loader
    pkg = pkg_loader.load()
    proc = pkg.ImageprocProcessing if a.processing == "imageproc" else pkg.OpenCVProcessing
    with open(a.path, "rb") as f:
        data = f.read()
    ctx = pkg.Context(a.device, proc)
    try:
        res = ctx.sift_jpeg(data)
    finally:
        ctx.close()
    print(f"{len(res)} keypoints")
    return 0


if __name__ == "__main__":
    sys.exit(main())
