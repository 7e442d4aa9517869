"""Host-side mirror of the reference crate's public API over libsift_mi.so.

Reference: /root/reference/src/lib.rs (tnibler/sift-features @ 2024-10-22)

    pub fn sift(img: &GrayImage, features_limit: Option<usize>) -> SiftResult   (:71)
    pub fn sift_with_processing::<P: Processing>(img, features_limit)           (:76)
    pub trait Processing { gaussian_blur, resize_linear, resize_nearest }       (:86-90)
    pub struct SiftResult { keypoints: Vec<KeyPoint>, descriptors: Array2<u8> } (:41-46)
    pub struct KeyPoint { x, y, size, angle, response: f32 }                    (:50-56)
    #[doc(hidden)] precompute_images / sift_with_precomputed / compute_descriptor (:131, :147, :785)

Names, argument meaning and output layout follow the reference; the
computation is the HIP path (no CPU fallback).  Differences, all documented
in DESIGN.md:
  * `sift()` uses `ImageprocProcessing`, as the crate does (src/lib.rs:71-73);
    that profile restates imageproc 0.25 / image 0.25 arithmetic, which no
    reference test pins (parity unpinned).  `sift_with_processing(
    OpenCVProcessing, ...)` is the profile the reference's golden snapshots
    pin.
  * with a features_limit, ties in response keep emission order (the
    reference's `sort_unstable_by` leaves their order unspecified).
  * errors raise SiftMiError where the reference panics.
"""
import contextlib
import ctypes
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import SiftMiError, check, lib

PROFILE_OPENCV = 0
PROFILE_IMAGEPROC = 1
DESCRIPTOR_SIZE = 128


@dataclass
class KeyPoint:
    """src/lib.rs:50-56"""
    x: float
    y: float
    size: float
    angle: float
    response: float


class SiftResult:
    """src/lib.rs:41-46.  `keypoints_array` is the (n, 5) f32 table
    (x, y, size, angle, response); `descriptors` the (n, 128) u8 array whose
    row i belongs to keypoint i."""

    __slots__ = ("keypoints_array", "descriptors", "keys")

    def __init__(self, keypoints_array, descriptors, keys=None):
        self.keypoints_array = keypoints_array
        self.descriptors = descriptors
        self.keys = keys

    @property
    def keypoints(self):
        return [KeyPoint(*map(float, r)) for r in self.keypoints_array]

    def __len__(self):
        return len(self.keypoints_array)

    def __eq__(self, other):
        return (isinstance(other, SiftResult) and np.array_equal(self.keypoints_array, other.keypoints_array)
                and np.array_equal(self.descriptors, other.descriptors))

    def __repr__(self):
        return f"SiftResult(n={len(self)})"


class ResultBuffers:
    """Reusable host arrays for batch results (streaming callers: avoids a
    fresh allocation -- and its page faults -- per batch).  Grows on demand."""

    def __init__(self, capacity=0):
        self._alloc(capacity)

    def _alloc(self, n):
        self.kps = np.empty((n, 5), np.float32)
        self.desc = np.empty((n, DESCRIPTOR_SIZE), np.uint8)
        self.keys = np.empty(n, np.uint64)

    def views(self, n):
        if n > len(self.kps):
            self._alloc(max(n, 2 * len(self.kps)))
        return self.kps[:n], self.desc[:n], self.keys[:n]


def _u8_image(img):
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 2:
        raise TypeError("expected a 2-D uint8 GrayImage array (height, width)")
    if a.strides[1] != 1 or a.strides[0] < a.shape[1]:
        a = np.ascontiguousarray(a)
    return a


def _f32_image(img):
    a = np.ascontiguousarray(img, dtype=np.float32)
    if a.ndim != 2:
        raise TypeError("expected a 2-D f32 image (LumaFImage)")
    return a


def _limit(features_limit):
    if features_limit is None:
        return -1
    if features_limit < 0:
        raise ValueError("features_limit must be >= 0 or None")
    return int(features_limit)


class Context:
    """One device context (libsift_mi `sift_mi_ctx`): one HIP stream, pooled
    device buffers.  Not thread-safe; use one per thread / GPU."""

    def __init__(self, device=0, processing=None):
        processing = processing or OpenCVProcessing
        self.profile = processing.profile
        self.device = device
        h = ctypes.c_void_p()
        check(lib().sift_mi_create(device, self.profile, ctypes.byref(h)))
        self._h = h
        self._generation = 0
        self._keep_dev = False  # sift_mi_set_keep_on_device state
        self._path_values = {}  # sift_mi_set_path_option values set through this object

    def close(self):
        if getattr(self, "_h", None):
            lib().sift_mi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- configuration ----------------------------------------------------
    def set_stream(self, hip_stream_handle):
        check(lib().sift_mi_set_stream(self._h, ctypes.c_void_p(hip_stream_handle or 0)))

    def set_exact_descriptors(self, exact=True):
        """Bit-exact descriptor accumulation order (slower); default off."""
        check(lib().sift_mi_set_exact_descriptors(self._h, 1 if exact else 0))

    def set_max_octaves(self, max_octaves):
        """LABELLED EXTENSION (not in the crate): cap the octave count (0 = the
        crate's formula, src/lib.rs:133-134).  The result is the uncapped
        result's keypoints of octaves < max_octaves."""
        check(lib().sift_mi_set_max_octaves(self._h, int(max_octaves)))

    def set_sample_counting(self, on=True):
        """Measurement only: count the gradient samples the orientation and
        descriptor kernels evaluate (stats() orient_samples / desc_samples)."""
        check(lib().sift_mi_set_sample_counting(self._h, 1 if on else 0))

    def set_row_band(self, band, n_bands):
        """Keypoint stages over octave rows [H_o*band/n_bands, H_o*(band+1)/n_bands)
        only (include/sift_mi.h); band 0 of 1 = the whole frame.  Merge the
        bands' results with shard.merge_bands."""
        check(lib().sift_mi_set_row_band(self._h, int(band), int(n_bands)))

    def set_chunk(self, images_per_chunk):
        check(lib().sift_mi_set_chunk(self._h, int(images_per_chunk)))

    def stats(self):
        s = _lib.Stats()
        check(lib().sift_mi_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        check(lib().sift_mi_reset_stats(self._h))

    # -- results ------------------------------------------------------------
    def _keep(self, on):
        """Results to host buffers (False: every host-returning call) or left
        in HBM (True: sift_batch_device(..., fetch=False))."""
        if bool(on) != self._keep_dev:
            check(lib().sift_mi_set_keep_on_device(self._h, 1 if on else 0))
            self._keep_dev = bool(on)

    def _fetch(self, n, with_keys=True, out=None):
        if out is not None:
            kps, desc, keys = out.views(n)
        else:
            kps = np.empty((n, 5), np.float32)
            desc = np.empty((n, DESCRIPTOR_SIZE), np.uint8)
            keys = np.empty(n, np.uint64) if with_keys else None
        check(lib().sift_mi_fetch(self._h, kps.ctypes.data, desc.ctypes.data, n))
        if with_keys:
            check(lib().sift_mi_fetch_keys(self._h, keys.ctypes.data, n))
        else:
            keys = None
        return kps, desc, keys

    # -- sift (src/lib.rs:71-81) ---------------------------------------------
    def sift(self, img, features_limit=None):
        a = _u8_image(img)
        n = ctypes.c_size_t()
        self._keep(False)
        check(lib().sift_mi_extract(self._h, a.ctypes.data, a.shape[1], a.shape[0], a.strides[0],
                                    _limit(features_limit), ctypes.byref(n)))
        return SiftResult(*self._fetch(n.value))

    def sift_batch(self, frames, features_limit=None):
        """One `sift()` per frame of an (n, h, w) u8 array; returns a list."""
        f = np.ascontiguousarray(frames, dtype=np.uint8)
        if f.ndim != 3:
            raise TypeError("expected (n, height, width) uint8 frames")
        n, h, w = f.shape
        ptrs = (ctypes.c_void_p * n)(*[f[i].ctypes.data for i in range(n)])
        offs = (ctypes.c_size_t * (n + 1))()
        self._keep(False)
        check(lib().sift_mi_extract_batch(self._h, ptrs, n, w, h, w, _limit(features_limit), offs))
        kps, desc, keys = self._fetch(offs[n])
        return [SiftResult(kps[offs[i]:offs[i + 1]], desc[offs[i]:offs[i + 1]], keys[offs[i]:offs[i + 1]])
                for i in range(n)]

    def sift_batch_device(self, d_frames_ptr, n, width, height, row_stride, frame_pitch,
                          features_limit=None, fetch=True, out=None):
        """Device-resident frames (e.g. a torch.uint8 cuda tensor's data_ptr()).
        Returns per-frame offsets and, with fetch, the concatenated results.
        `out` (a ResultBuffers) receives the results in reused host arrays;
        the returned SiftResult then holds views into it, valid until the
        buffers are reused."""
        offs = (ctypes.c_size_t * (n + 1))()
        self._keep(not fetch)
        check(lib().sift_mi_extract_batch_device(self._h, ctypes.c_void_p(d_frames_ptr), frame_pitch, n, width,
                                                 height, row_stride, _limit(features_limit), offs))
        offsets = np.array(offs[:], dtype=np.int64)
        if not fetch:
            return offsets, None
        return offsets, SiftResult(*self._fetch(int(offsets[-1]), out=out))

    def set_pipeline_lanes(self, lanes):
        """2 (default): consecutive batch chunks overlap on two streams; 1: serial."""
        check(lib().sift_mi_set_pipeline_lanes(self._h, int(lanes)))

    def device_results(self):
        """(keypoints device pointer, descriptors device pointer, n) of the last
        sift_batch_device(..., fetch=False): every frame's results, concatenated
        in frame order, in HBM."""
        kp, desc, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_size_t()
        check(lib().sift_mi_device_results(self._h, ctypes.byref(kp), ctypes.byref(desc), ctypes.byref(n)))
        return kp.value, desc.value, n.value

    def read_batch_scale_space(self, frame, octave, dims=None):
        """(6, h, w) f32 Gaussians of `octave` of `frame` of the last call, as
        its pyramid left them (valid when that call ran as one chunk; a
        validation read-back, sift_mi_read_batch_scale_space).  The octave's
        (w, h) come from the library (sift_mi_batch_octave_dims); `dims`, if
        given, must equal them."""
        w, h = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().sift_mi_batch_octave_dims(self._h, int(octave), ctypes.byref(w), ctypes.byref(h)))
        if dims is not None and tuple(dims) != (w.value, h.value):
            raise ValueError(f"dims {tuple(dims)} != the batch octave's {(w.value, h.value)}")
        out = np.empty((6, h.value, w.value), np.float32)
        check(lib().sift_mi_read_batch_scale_space(self._h, int(frame), int(octave), out.ctypes.data, out.size))
        return out

    # kernel-path switches (include/sift_mi.h sift_mi_path_option): test /
    # diagnostic only; the defaults are the product path
    PATH_OPTIONS = {"tile_blur": (0, 0), "pair_blur": (1, 1), "seed_pair": (2, 1), "tail": (3, 1),
                    "fused_detect": (4, 1), "early": (5, 1), "desc_first": (6, 1), "graph": (7, 0),
                    "band_drift": (8, 24), "bound_shrink": (9, 1),
                    "large_first": (11, 1),
                    "onesweep": (12, 0), "bd_pair": (13, 1), "bd_waves": (14, 8192),
                    "chunk_mode": (15, 1)}

    def set_path_option(self, name, value):
        """One kernel-path switch (sift_mi_set_path_option), e.g.
        set_path_option("pair_blur", 0)."""
        check(lib().sift_mi_set_path_option(self._h, self.PATH_OPTIONS[name][0], int(value)))
        self._path_values[name] = int(value)

    def path_option(self, name):
        """The switch's current value (as last set through this object, else
        its default)."""
        return self._path_values.get(name, self.PATH_OPTIONS[name][1])

    @contextlib.contextmanager
    def path_options(self, **opts):
        """Kernel-path switches for the duration of a with-block, then the
        values they had before it."""
        before = {k: self.path_option(k) for k in opts}
        try:
            for k, v in opts.items():
                self.set_path_option(k, v)
            yield self
        finally:
            for k, v in before.items():
                self.set_path_option(k, v)

    # -- precompute_images / sift_with_precomputed (src/lib.rs:123-177) ------
    def precompute_images(self, img):
        a = _u8_image(img)
        n = ctypes.c_size_t()
        check(lib().sift_mi_precompute(self._h, a.ctypes.data, a.shape[1], a.shape[0], a.strides[0],
                                       ctypes.byref(n)))
        self._generation += 1
        return PrecomputedImages(self, n.value, self._generation)

    def sift_with_precomputed(self, pre, features_limit=None):
        pre._check()
        n = ctypes.c_size_t()
        self._keep(False)
        check(lib().sift_mi_sift_with_precomputed(self._h, _limit(features_limit), ctypes.byref(n)))
        return SiftResult(*self._fetch(n.value))

    # -- compute_descriptor (src/lib.rs:785) -----------------------------------
    def compute_descriptor(self, img, x, y, scale, orientation):
        a = _f32_image(img)
        out = np.zeros(DESCRIPTOR_SIZE, np.uint8)
        check(lib().sift_mi_compute_descriptor(self._h, a.ctypes.data, a.shape[1], a.shape[0], float(x),
                                               float(y), float(scale), float(orientation), out.ctypes.data))
        return out

    # -- matching (examples/sift-match.rs:30-35) -----------------------------
    def match_descriptors(self, query, train, cross_check=True):
        """cv::BFMatcher(NORM_L2, crossCheck).match(query, train) on the GPU.
        query / train: (n, 128) u8 descriptors.  Returns (query_idx, train_idx,
        distance) arrays in query order."""
        q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, DESCRIPTOR_SIZE)
        t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, DESCRIPTOR_SIZE)
        out = (_lib.Match * max(len(q), 1))()
        n = ctypes.c_size_t()
        check(lib().sift_mi_match_descriptors(self._h, q.ctypes.data, len(q), t.ctypes.data, len(t),
                                              1 if cross_check else 0, out, len(q), ctypes.byref(n)))
        a = np.ctypeslib.as_array(out)[: n.value]
        return (a["query_idx"].astype(np.int32), a["train_idx"].astype(np.int32),
                a["distance"].astype(np.float32))

    # -- the input step ------------------------------
    def decode_jpeg(self, data):
        """Baseline JPEG bytes -> (h, w) u8 luma, as the reference makes its
        inputs: `image::open(..)` (zune-jpeg) then `.grayscale()`
        (examples/run-sift.rs:8, src/lib.rs:1012).  Entropy decoding on the
        host, IDCT / upsampling / colour on the GPU."""
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        w, h = jpeg_dims(buf)
        out = np.empty((h, w), np.uint8)
        check(lib().sift_mi_decode_jpeg(self._h, buf.ctypes.data, len(buf), out.ctypes.data, w, 0))
        return out

    def decode_jpeg_device(self, data, out_ptr, out_stride):
        """The same into device memory (e.g. a torch.uint8 CUDA tensor's
        data_ptr(), row stride in bytes), ordered on the context stream."""
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        check(lib().sift_mi_decode_jpeg(self._h, buf.ctypes.data, len(buf), out_ptr, out_stride, 1))

    def decode_jpeg_batch_device(self, datas, out_ptr, frame_pitch, row_stride, threads=0):
        """Equal-size JPEGs -> device frames (frame i at out_ptr + i *
        frame_pitch), ready for sift_batch_device; host threads decode the
        entropy-coded data."""
        bufs = [np.frombuffer(bytes(d), dtype=np.uint8) for d in datas]
        ptrs = (ctypes.c_void_p * max(1, len(bufs)))(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * max(1, len(bufs)))(*[len(b) for b in bufs])
        check(lib().sift_mi_decode_jpeg_batch(self._h, ptrs, lens, len(bufs), out_ptr, frame_pitch, row_stride,
                                              int(threads)))

    def sift_jpeg(self, data, features_limit=None):
        """`sift(image::open(path)?.grayscale())` of examples/run-sift.rs on
        JPEG bytes."""
        return self.sift(self.decode_jpeg(data), features_limit)

    # -- Processing ops (src/lib.rs:86-90) ---------------------------------
    def gaussian_blur(self, img, sigma):
        a = _f32_image(img)
        out = np.empty_like(a)
        check(lib().sift_mi_gaussian_blur(self._h, a.ctypes.data, a.shape[1], a.shape[0], float(sigma),
                                          out.ctypes.data))
        return out

    def resize_linear(self, img, width, height):
        a = _f32_image(img)
        out = np.empty((height, width), np.float32)
        check(lib().sift_mi_resize_linear(self._h, a.ctypes.data, a.shape[1], a.shape[0], width, height,
                                          out.ctypes.data))
        return out

    def resize_nearest(self, img, width, height):
        a = _f32_image(img)
        out = np.empty((height, width), np.float32)
        check(lib().sift_mi_resize_nearest(self._h, a.ctypes.data, a.shape[1], a.shape[0], width, height,
                                           out.ctypes.data))
        return out


class PrecomputedImages:
    """src/lib.rs:123-128: scale_space[o] is (6, h, w) f32, dog[o] (5, h, w)."""

    def __init__(self, ctx, n_octaves, generation):
        self._ctx = ctx
        self.n_octaves = n_octaves
        self._gen = generation

    def _check(self):
        if self._gen != self._ctx._generation:
            raise SiftMiError(-6, "PrecomputedImages superseded by a later precompute on this context")

    def dims(self, o):
        w, h = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().sift_mi_octave_dims(self._ctx._h, o, ctypes.byref(w), ctypes.byref(h)))
        return w.value, h.value

    def scale_space_octave(self, o):
        self._check()
        w, h = self.dims(o)
        out = np.empty((6, h, w), np.float32)
        check(lib().sift_mi_read_scale_space(self._ctx._h, o, out.ctypes.data))
        return out

    def dog_octave(self, o):
        self._check()
        w, h = self.dims(o)
        out = np.empty((5, h, w), np.float32)
        check(lib().sift_mi_read_dog(self._ctx._h, o, out.ctypes.data))
        return out

    @property
    def scale_space(self):
        return [self.scale_space_octave(o) for o in range(self.n_octaves)]

    @property
    def dog(self):
        return [self.dog_octave(o) for o in range(self.n_octaves)]


# ---------------------------------------------------------------------------
# Processing backends (src/lib.rs:86-90, :993-1007; src/opencv_processing.rs)
# ---------------------------------------------------------------------------
class Processing:
    profile = None

    @classmethod
    def gaussian_blur(cls, img, sigma):
        return default_context(processing=cls).gaussian_blur(img, sigma)

    @classmethod
    def resize_linear(cls, img, width, height):
        return default_context(processing=cls).resize_linear(img, width, height)

    @classmethod
    def resize_nearest(cls, img, width, height):
        return default_context(processing=cls).resize_nearest(img, width, height)


class OpenCVProcessing(Processing):
    """cv::GaussianBlur / cv::resize arithmetic (src/opencv_processing.rs:38-74)."""
    profile = PROFILE_OPENCV


class ImageprocProcessing(Processing):
    """imageproc gaussian_blur_f32 / image::imageops::resize arithmetic
    (src/lib.rs:993-1007): the crate's default backend.  Restated from
    imageproc 0.25.0 / image 0.25.2 (not in the reference tree); parity
    against the reference is unpinned (no reference test runs it)."""
    profile = PROFILE_IMAGEPROC


_tls = threading.local()


def default_context(device=0, processing=None):
    processing = processing or ImageprocProcessing
    cache = getattr(_tls, "ctx", None)
    if cache is None:
        cache = _tls.ctx = {}
    key = (device, processing.profile)
    if key not in cache:
        cache[key] = Context(device, processing)
    return cache[key]


def sift(img, features_limit=None):
    """src/lib.rs:71: sift_with_processing::<ImageprocProcessing>."""
    return default_context(processing=ImageprocProcessing).sift(img, features_limit)


def sift_with_processing(processing, img, features_limit=None):
    """src/lib.rs:76"""
    return default_context(processing=processing).sift(img, features_limit)


def precompute_images(processing, img):
    """src/lib.rs:131"""
    return default_context(processing=processing).precompute_images(img)


def sift_with_precomputed(pre, features_limit=None):
    """src/lib.rs:147"""
    return pre._ctx.sift_with_precomputed(pre, features_limit)


def compute_descriptor(img, x, y, scale, orientation):
    """src/lib.rs:785"""
    return default_context().compute_descriptor(img, x, y, scale, orientation)


def jpeg_dims(data):
    """(width, height) of a baseline JPEG from its headers (host only)."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    w, h = ctypes.c_uint32(), ctypes.c_uint32()
    check(lib().sift_mi_jpeg_dims(buf.ctypes.data, len(buf), ctypes.byref(w), ctypes.byref(h)))
    return w.value, h.value


def decode_jpeg(data):
    return default_context().decode_jpeg(data)


def match_descriptors(query, train, cross_check=True):
    """examples/sift-match.rs:30-35: BFMatcher(NORM_L2, crossCheck).match."""
    return default_context().match_descriptors(query, train, cross_check)


def stable_sort_xy_size(keypoints_array):
    """Order of the reference test's snapshots (src/lib.rs:1020-1030): stable
    sort by (x, y, size)."""
    k = np.asarray(keypoints_array)
    if not len(k):
        return np.zeros(0, np.int64)
    return np.lexsort((k[:, 2], k[:, 1], k[:, 0]))


def key_fields(keys):
    """Decode emission keys (include/sift_mi.h sift_mi_fetch_keys)."""
    k = np.asarray(keys, dtype=np.uint64)
    f = lambda s, b: ((k >> np.uint64(s)) & np.uint64((1 << b) - 1)).astype(np.int64)
    return {"frame": f(42, 22), "octave": f(38, 4), "s_init": f(36, 2), "y_init": f(21, 15),
            "x_init": f(6, 15), "peak": f(0, 6)}
