"""ctypes binding of libsift_mi.so (include/sift_mi.h).

The HIP library is the product: there is no CPU fallback.  Loading fails
loudly when the shared object is missing (run ``python -c "import
__graft_entry__ as g; g.build()"`` or ``make -C sift-features_amd/csrc``).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SIFT_MI_LIB: an alternative build of the same library (performance
# experiments, tools/exp/variants.sh); the product loads the in-tree build.
LIB_PATH = os.environ.get("SIFT_MI_LIB") or os.path.join(HERE, "libsift_mi.so")

# every symbol declared in include/sift_mi.h
EXPORTS = [
    "sift_mi_create", "sift_mi_destroy", "sift_mi_set_stream", "sift_mi_set_chunk",
    "sift_mi_extract", "sift_mi_fetch", "sift_mi_fetch_keys", "sift_mi_extract_batch",
    "sift_mi_extract_batch_device", "sift_mi_set_exact_descriptors", "sift_mi_set_max_octaves", "sift_mi_set_sample_counting", "sift_mi_set_keep_on_device", "sift_mi_device_results",
    "sift_mi_set_pipeline_lanes", "sift_mi_set_row_band",
    "sift_mi_precompute", "sift_mi_octave_dims", "sift_mi_read_scale_space", "sift_mi_read_dog",
    "sift_mi_read_batch_scale_space", "sift_mi_batch_octave_dims", "sift_mi_set_path_option",
    "sift_mi_sift_with_precomputed", "sift_mi_compute_descriptor", "sift_mi_gaussian_blur",
    "sift_mi_resize_linear", "sift_mi_resize_nearest", "sift_mi_match_descriptors", "sift_mi_jpeg_dims",
    "sift_mi_decode_jpeg", "sift_mi_decode_jpeg_batch", "sift_mi_get_stats",
    "sift_mi_reset_stats",
    "sift_mi_version", "sift_mi_last_error",
]

STATUS = {0: "OK", -1: "EINVAL", -2: "ENOMEM", -3: "EHIP", -4: "ENODEV", -5: "EUNSUPPORTED", -6: "ESTATE"}


class SiftMiError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sift_mi error {STATUS.get(code, code)}: {msg}")
        self.code = code


class Match(ctypes.Structure):
    """include/sift_mi.h sift_mi_match (cv::DMatch without imgIdx)."""
    _fields_ = [("query_idx", ctypes.c_int32), ("train_idx", ctypes.c_int32), ("distance", ctypes.c_float)]


class Stats(ctypes.Structure):
    _fields_ = [("pyramid_ms", ctypes.c_double), ("detect_ms", ctypes.c_double),
                ("orient_ms", ctypes.c_double), ("order_ms", ctypes.c_double),
                ("descriptor_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("pyramid_bytes", ctypes.c_uint64), ("pyramid_launches", ctypes.c_uint64),
                ("frames", ctypes.c_uint64), ("extrema", ctypes.c_uint64),
                ("keypoints", ctypes.c_uint64), ("band_reruns", ctypes.c_uint64),
                ("stage_reruns", ctypes.c_uint64), ("orient_samples", ctypes.c_uint64),
                ("desc_samples", ctypes.c_uint64), ("pyramid_scan_bytes", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same
    # SONAME as /opt/rocm's).  If torch is importable, load it first so that
    # libsift_mi.so binds to the already-loaded runtime instead of pulling in a
    # second copy (which breaks torch.cuda initialisation afterwards).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run `make -C {os.path.join(HERE, 'csrc')}` "
                          "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_size_t
    f32, f64, i32 = ctypes.c_float, ctypes.c_double, ctypes.c_int
    P = ctypes.POINTER
    sig = {
        "sift_mi_create": [i32, i32, P(vp)],
        "sift_mi_destroy": [vp],
        "sift_mi_set_stream": [vp, vp],
        "sift_mi_set_chunk": [vp, u32],
        "sift_mi_extract": [vp, vp, u32, u32, sz, i64, P(sz)],
        "sift_mi_fetch": [vp, vp, vp, sz],
        "sift_mi_fetch_keys": [vp, vp, sz],
        "sift_mi_extract_batch": [vp, P(vp), u32, u32, u32, sz, i64, P(sz)],
        "sift_mi_extract_batch_device": [vp, vp, sz, u32, u32, u32, sz, i64, P(sz)],
        "sift_mi_set_keep_on_device": [vp, i32],
        "sift_mi_set_pipeline_lanes": [vp, i32],
        "sift_mi_set_row_band": [vp, ctypes.c_uint32, ctypes.c_uint32],
        "sift_mi_set_exact_descriptors": [vp, i32],
        "sift_mi_set_max_octaves": [vp, i32],
        "sift_mi_set_sample_counting": [vp, i32],
        "sift_mi_device_results": [vp, P(vp), P(vp), P(sz)],
        "sift_mi_precompute": [vp, vp, u32, u32, sz, P(sz)],
        "sift_mi_octave_dims": [vp, sz, P(u32), P(u32)],
        "sift_mi_read_scale_space": [vp, sz, vp],
        "sift_mi_read_batch_scale_space": [vp, ctypes.c_uint32, sz, vp, sz],
        "sift_mi_batch_octave_dims": [vp, sz, P(u32), P(u32)],
        "sift_mi_set_path_option": [vp, i32, i32],
        "sift_mi_read_dog": [vp, sz, vp],
        "sift_mi_sift_with_precomputed": [vp, i64, P(sz)],
        "sift_mi_compute_descriptor": [vp, vp, u32, u32, f32, f32, f32, f32, vp],
        "sift_mi_gaussian_blur": [vp, vp, u32, u32, f64, vp],
        "sift_mi_resize_linear": [vp, vp, u32, u32, u32, u32, vp],
        "sift_mi_resize_nearest": [vp, vp, u32, u32, u32, u32, vp],
        "sift_mi_match_descriptors": [vp, vp, sz, vp, sz, i32, vp, sz, P(sz)],
        "sift_mi_jpeg_dims": [vp, sz, P(u32), P(u32)],
        "sift_mi_decode_jpeg": [vp, vp, sz, vp, sz, i32],
        "sift_mi_decode_jpeg_batch": [vp, P(vp), P(sz), u32, vp, sz, sz, i32],
        "sift_mi_get_stats": [vp, P(Stats)],
        "sift_mi_reset_stats": [vp],
        "sift_mi_version": [],
        "sift_mi_last_error": [],
    }
    for name, args in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = i32
    L.sift_mi_destroy.restype = None
    L.sift_mi_version.restype = ctypes.c_char_p
    L.sift_mi_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().sift_mi_last_error()
        raise SiftMiError(rc, msg.decode() if msg else "")
    return rc
