"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  It restates /root/reference/src/lib.rs (see
oracle/sift_oracle.c for the per-function citations); it is the checker,
never the thing measured or shipped.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsift_oracle.so")

PROFILE_OPENCV = 0
PROFILE_IMAGEPROC = 1


class _Kp(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("x", "y", "size", "angle", "response")]


class _Ext(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("x", "y", "size", "angle", "response")] + [
        (n, ctypes.c_int32) for n in ("octave", "scale", "s_init", "y_init", "x_init", "peak")
    ]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, f32, f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_double
        L.oracle_sift.restype = vp
        L.oracle_sift.argtypes = [vp, i32, i32, i32, i32, ctypes.c_int64]
        L.oracle_precompute.restype = vp
        L.oracle_precompute.argtypes = [vp, i32, i32, i32, i32]
        L.oracle_sift_with_precomputed.restype = vp
        L.oracle_sift_with_precomputed.argtypes = [vp, ctypes.c_int64]
        L.oracle_pyramid_free.argtypes = [vp]
        L.oracle_pyramid_n_octaves.argtypes = [vp]
        L.oracle_pyramid_dims.argtypes = [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.oracle_pyramid_gauss.restype = ctypes.POINTER(f32)
        L.oracle_pyramid_gauss.argtypes = [vp, i32]
        L.oracle_pyramid_dog.restype = ctypes.POINTER(f32)
        L.oracle_pyramid_dog.argtypes = [vp, i32]
        L.oracle_result_n.restype = ctypes.c_size_t
        L.oracle_result_n.argtypes = [vp]
        L.oracle_result_keypoints.restype = ctypes.POINTER(_Kp)
        L.oracle_result_keypoints.argtypes = [vp]
        L.oracle_result_internal.restype = ctypes.POINTER(_Ext)
        L.oracle_result_internal.argtypes = [vp]
        L.oracle_result_descriptors.restype = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_result_descriptors.argtypes = [vp]
        L.oracle_result_free.argtypes = [vp]
        L.oracle_compute_descriptor.argtypes = [vp, i32, i32, f32, f32, f32, f32, vp]
        L.oracle_gaussian_blur.argtypes = [vp, i32, i32, f64, i32, vp]
        L.oracle_resize_linear.argtypes = [vp, i32, i32, i32, i32, i32, vp]
        L.oracle_resize_nearest.argtypes = [vp, i32, i32, i32, i32, i32, vp]
        L.oracle_n_octaves.argtypes = [i32, i32]
        L.oracle_cv_ksize.argtypes = [f64]
        L.oracle_cv_kernel.argtypes = [i32, f64, vp]
        L.oracle_octave_sigmas.argtypes = [vp]
        L.oracle_seed_sigma.restype = f64
        L.oracle_match.argtypes = [vp, i32, vp, i32, i32, vp, vp]
        _lib = L
    return _lib


def _u8(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    assert img.ndim == 2
    return img


def _result(r):
    L = lib()
    if not r:
        raise RuntimeError("oracle failed")
    try:
        n = L.oracle_result_n(r)
        if n == 0:
            return np.zeros((0, 5), np.float32), np.zeros((0, 128), np.uint8), np.zeros((0, 6), np.int32)
        kp = np.ctypeslib.as_array(ctypes.cast(L.oracle_result_keypoints(r), ctypes.POINTER(ctypes.c_float)),
                                   shape=(max(n, 1) * 5,))[: n * 5].reshape(n, 5).copy()
        ext = np.ctypeslib.as_array(ctypes.cast(L.oracle_result_internal(r), ctypes.POINTER(ctypes.c_int32)),
                                    shape=(max(n, 1) * 11,))[: n * 11].reshape(n, 11).copy()
        desc = np.ctypeslib.as_array(L.oracle_result_descriptors(r), shape=(max(n, 1) * 128,))[: n * 128]
        desc = desc.reshape(n, 128).copy()
    finally:
        L.oracle_result_free(r)
    # ext columns 5.. are int32: octave, scale, s_init, y_init, x_init, peak
    return kp, desc, ext[:, 5:].copy()


def sift(img, features_limit=None, profile=PROFILE_OPENCV, internal=False):
    """Oracle of `sift_with_processing::<P>` (src/lib.rs:76-81).

    Returns (keypoints[n,5] f32 (x,y,size,angle,response), descriptors[n,128] u8)
    and, with internal=True, the (octave, scale, s_init, y_init, x_init, peak)
    table as a third element.
    """
    img = _u8(img)
    h, w = img.shape
    lim = -1 if features_limit is None else int(features_limit)
    r = lib().oracle_sift(img.ctypes.data, w, h, w, profile, lim)
    kp, desc, ext = _result(r)
    return (kp, desc, ext) if internal else (kp, desc)


class Pyramid:
    """Oracle of `precompute_images` / `PrecomputedImages` (src/lib.rs:123-143)."""

    def __init__(self, img, profile=PROFILE_OPENCV):
        img = _u8(img)
        h, w = img.shape
        self._p = lib().oracle_precompute(img.ctypes.data, w, h, w, profile)
        if not self._p:
            raise RuntimeError("oracle precompute failed")
        self.n_octaves = lib().oracle_pyramid_n_octaves(self._p)

    def dims(self, o):
        w, h = ctypes.c_int(), ctypes.c_int()
        lib().oracle_pyramid_dims(self._p, o, ctypes.byref(w), ctypes.byref(h))
        return w.value, h.value

    def scale_space(self, o):
        w, h = self.dims(o)
        return np.ctypeslib.as_array(lib().oracle_pyramid_gauss(self._p, o), shape=(6, h, w)).copy()

    def dog(self, o):
        w, h = self.dims(o)
        return np.ctypeslib.as_array(lib().oracle_pyramid_dog(self._p, o), shape=(5, h, w)).copy()

    def sift_with_precomputed(self, features_limit=None):
        lim = -1 if features_limit is None else int(features_limit)
        return _result(lib().oracle_sift_with_precomputed(self._p, lim))[:2]

    def __del__(self):
        if getattr(self, "_p", None):
            lib().oracle_pyramid_free(self._p)
            self._p = None


def compute_descriptor(img, x, y, scale, orientation):
    """Oracle of `compute_descriptor` (src/lib.rs:785-990)."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape
    out = np.zeros(128, np.uint8)
    lib().oracle_compute_descriptor(img.ctypes.data, w, h, x, y, scale, orientation, out.ctypes.data)
    return out


def gaussian_blur(img, sigma, profile=PROFILE_OPENCV):
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape
    out = np.empty_like(img)
    if lib().oracle_gaussian_blur(img.ctypes.data, w, h, float(sigma), profile, out.ctypes.data):
        raise RuntimeError("unsupported profile")
    return out


def resize_linear(img, w2, h2, profile=PROFILE_OPENCV):
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape
    out = np.empty((h2, w2), np.float32)
    if lib().oracle_resize_linear(img.ctypes.data, w, h, w2, h2, profile, out.ctypes.data):
        raise RuntimeError("unsupported profile")
    return out


def resize_nearest(img, w2, h2, profile=PROFILE_OPENCV):
    img = np.ascontiguousarray(img, dtype=np.float32)
    h, w = img.shape
    out = np.empty((h2, w2), np.float32)
    if lib().oracle_resize_nearest(img.ctypes.data, w, h, w2, h2, profile, out.ctypes.data):
        raise RuntimeError("unsupported profile")
    return out


def n_octaves(w, h):
    return lib().oracle_n_octaves(w, h)


def cv_kernel(sigma):
    n = lib().oracle_cv_ksize(float(sigma))
    out = np.zeros(n, np.float32)
    lib().oracle_cv_kernel(n, float(sigma), out.ctypes.data)
    return out


def octave_sigmas():
    out = np.zeros(6, np.float64)
    lib().oracle_octave_sigmas(out.ctypes.data)
    return out


def seed_sigma():
    return lib().oracle_seed_sigma()


def stable_sort_xy_size(kps):
    """The snapshot order of `sift_end2end` (src/lib.rs:1020-1030): stable sort
    by (x, y, size) with f32::total_cmp."""
    return np.lexsort((kps[:, 2], kps[:, 1], kps[:, 0]), axis=0) if len(kps) else np.zeros(0, np.int64)


def match(query, train, cross_check=True):
    """Oracle of cv::BFMatcher(NORM_L2, crossCheck).match (examples/sift-match.rs:30-35).
    Returns (query_idx, train_idx, distance) arrays of the matches, in query order."""
    q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, 128)
    t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, 128)
    ti = np.zeros(max(len(q), 1), np.int32)
    di = np.zeros(max(len(q), 1), np.float32)
    lib().oracle_match(q.ctypes.data, len(q), t.ctypes.data, len(t), 1 if cross_check else 0, ti.ctypes.data,
                       di.ctypes.data)
    ti, di = ti[: len(q)], di[: len(q)]
    keep = np.nonzero(ti >= 0)[0]
    return keep.astype(np.int32), ti[keep], di[keep]
