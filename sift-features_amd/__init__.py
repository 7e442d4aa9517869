"""sift_features_amd -- MI355X-native SIFT hot path (gfx950 HIP kernels behind a
C ABI, include/sift_mi.h), a drop-in for tnibler/sift-features' `sift()`.

See sift.py for the reference API mirror and DESIGN.md for the design.
"""
from ._lib import SiftMiError, lib  # noqa: F401
from .sift import (  # noqa: F401
    DESCRIPTOR_SIZE, Context, ImageprocProcessing, KeyPoint, OpenCVProcessing, PrecomputedImages, Processing,
    ResultBuffers,
    SiftResult, compute_descriptor, decode_jpeg, default_context, jpeg_dims, key_fields, match_descriptors,
    precompute_images, sift,
    sift_with_precomputed,
    sift_with_processing, stable_sort_xy_size)

__version__ = "0.1.0"
