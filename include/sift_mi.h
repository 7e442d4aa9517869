/*
 * sift_mi.h -- C ABI of the MI355X-native SIFT hot path (libsift_mi.so).
 *
 * Drop-in boundary for tnibler/sift-features (src/lib.rs @ 2024-10-22).
 * Plain pointers and sizes only (no HIP, torch or Rust types), so that the
 * crate's `sift()` can be re-implemented as a thin `extern "C"` shim (see
 * INTEGRATION.md for the Rust binding a maintainer would add).
 *
 * Every entry point names the reference interface it replaces (file:line).
 * All functions return 0 (SIFT_MI_OK) on success or a negative
 * sift_mi_status; sift_mi_last_error() describes the last failure of the
 * calling thread.  The reference is infallible (it panics); the Rust shim
 * panics with sift_mi_last_error() to keep that signature.
 *
 * Threading: a context is not thread-safe; use one context per thread (and
 * per GPU).  Distinct contexts run concurrently.
 * Ownership: inputs are borrowed for the duration of a call.  Results live
 * in context-owned buffers until the next extraction call or destroy.
 */
#ifndef SIFT_MI_H
#define SIFT_MI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIFT_MI_DESCRIPTOR_SIZE 128

/* src/lib.rs:48-56 `KeyPoint` (the Rust struct is not repr(C); the shim
 * converts field by field).  x, y, size are in input-image pixels (the
 * reference's final `* DELTA_MIN`, src/lib.rs:163-176, is applied). */
typedef struct {
    float x, y, size, angle, response;
} sift_mi_keypoint;

/* src/lib.rs:86-90 `trait Processing`: which blur / resize arithmetic the
 * pyramid uses.  OPENCV = `OpenCVProcessing` (src/opencv_processing.rs:38-74,
 * the backend the reference's golden snapshots pin).  IMAGEPROC =
 * `ImageprocProcessing` (src/lib.rs:993-1007), the crate's default for
 * `sift()`: imageproc 0.25 gaussian_blur_f32 + image 0.25 resize arithmetic,
 * restated (those crates are not in the reference tree and no reference test
 * runs this profile: parity unpinned). */
typedef enum { SIFT_MI_PROFILE_OPENCV = 0, SIFT_MI_PROFILE_IMAGEPROC = 1 } sift_mi_profile;

typedef enum {
    SIFT_MI_OK = 0,
    SIFT_MI_EINVAL = -1,      /* bad argument (null pointer, zero size, stride < width ...) */
    SIFT_MI_ENOMEM = -2,      /* device or host allocation failed */
    SIFT_MI_EHIP = -3,        /* HIP runtime error (message in sift_mi_last_error) */
    SIFT_MI_ENODEV = -4,      /* no usable gfx950 device */
    SIFT_MI_EUNSUPPORTED = -5,/* profile / feature not implemented */
    SIFT_MI_ESTATE = -6       /* call sequence error (e.g. fetch before extract) */
} sift_mi_status;

typedef struct sift_mi_ctx sift_mi_ctx;

/* Create a context on HIP device `device_ordinal`; owns one HIP stream and
 * pooled device buffers.  Fails with SIFT_MI_ENODEV on a non-gfx950 device. */
int sift_mi_create(int device_ordinal, sift_mi_profile profile, sift_mi_ctx** out);
void sift_mi_destroy(sift_mi_ctx* ctx);

/* Run subsequent work on an external hipStream_t (e.g. torch's current
 * stream); NULL restores the context-owned stream. */
int sift_mi_set_stream(sift_mi_ctx* ctx, void* hip_stream);

/* Images per internal pipeline chunk for batch calls (0 = automatic). */
int sift_mi_set_chunk(sift_mi_ctx* ctx, uint32_t images_per_chunk);

/* ---- src/lib.rs:71 `sift(img, features_limit) -> SiftResult` ------------
 * `pixels`: row-major u8 GrayImage, `row_stride` >= width bytes per row.
 * features_limit < 0 == None.  With a limit the result is ordered by
 * response, descending (src/lib.rs:156-161); ties keep emission order (the
 * reference's sort_unstable_by leaves them unspecified).
 * Writes the keypoint count to *n_keypoints; fetch with sift_mi_fetch. */
int sift_mi_extract(sift_mi_ctx* ctx, const uint8_t* pixels, uint32_t width, uint32_t height,
                    size_t row_stride, int64_t features_limit, size_t* n_keypoints);

/* Copy the last result: `kps[cap]`, `desc[cap * 128]` (row i <-> keypoint i,
 * the (n,128) C-order `Array2<u8>` of SiftResult::descriptors).  Either
 * pointer may be NULL.  cap must be >= the result size. */
int sift_mi_fetch(sift_mi_ctx* ctx, sift_mi_keypoint* kps, uint8_t* desc, size_t cap);

/* Emission keys of the last result, for parity checks: bits
 * [42,64) image, [38,42) octave, [36,38) initial scale, [21,36) initial y,
 * [6,21) initial x, [0,6) orientation peak (x/y in octave pixels; octave 0
 * is the 2x seed, so frames up to 16384 px fit the 15-bit fields) -- the reference's emission order
 * (src/lib.rs:281-294, :324-332, :397-431). */
int sift_mi_fetch_keys(sift_mi_ctx* ctx, uint64_t* keys, size_t cap);

/* ---- batch of equal-size frames (throughput path; one `sift()` per frame)
 * `offsets[n+1]` receives the per-frame ranges in the concatenated result. */
int sift_mi_extract_batch(sift_mi_ctx* ctx, const uint8_t* const* frames, uint32_t n, uint32_t width,
                          uint32_t height, size_t row_stride, int64_t features_limit, size_t* offsets);

/* Same, frames already resident in device memory: frame i starts at
 * d_frames + i * frame_pitch (bytes).  The timed path of bench.py. */
int sift_mi_extract_batch_device(sift_mi_ctx* ctx, const uint8_t* d_frames, size_t frame_pitch, uint32_t n,
                                 uint32_t width, uint32_t height, size_t row_stride, int64_t features_limit,
                                 size_t* offsets);

/* Descriptor accumulation order.  0 (default): lane-private histograms summed
 * per bin -- components within +-1 of the reference.  1: bins accumulated in
 * the reference's sequential sample order (src/lib.rs:883-948) -- bit-exact
 * descriptors, slower.  Keypoints are identical in both modes. */
int sift_mi_set_exact_descriptors(sift_mi_ctx* ctx, int exact);

/* LABELLED EXTENSION (not in the crate): cap the octave count at max_octaves
 * (0 = the crate's formula round(log2(min(2W, 2H)) - 2) + 1, src/lib.rs:133-134,
 * the default).  The kept octaves are computed exactly as without the cap.
 * With features_limit None the result is the uncapped result's keypoints of
 * octaves < max_octaves (a prefix of the emission order).  With a limit, the
 * cap applies first: the limit ranks the capped keypoint set (src/lib.rs:156-161
 * on the prefix), which is not in general a subset of the uncapped limited
 * result.  For the "5 octaves" / "7 octaves" wording of BASELINE.json's
 * configs; parity runs leave it at 0. */
int sift_mi_set_max_octaves(sift_mi_ctx* ctx, int max_octaves);

/* Batch pipeline lanes: 2 (default) runs consecutive chunks on two streams
 * with their own pyramid arenas, so one chunk's kernels overlap the other's;
 * 1 runs the chunks one after another on the context's stream (half the
 * device memory; used to time kernels in isolation). */
int sift_mi_set_pipeline_lanes(sift_mi_ctx* ctx, int lanes);

/* Row band of the keypoint stages, for splitting ONE large frame across
 * contexts / GPUs (replaces nothing in the reference,
 * whose sift() is whole-frame: src/lib.rs:71-81).  With n_bands > 1,
 * detection (and so refinement, orientation and descriptors) covers only
 * octave rows [H_o*band/n_bands, H_o*(band+1)/n_bands) of each octave o,
 * and the pyramid is computed only on those rows plus the halos they read
 * (a refinement reaching beyond them re-runs the call on the whole pyramid:
 * sift_mi_stats.band_reruns; OpenCV profile, else the whole pyramid).  The bands
 * partition every octave's candidate rows, so the union of the n_bands
 * results, ordered by emission key (sift_mi_fetch_keys), is exactly the
 * whole-frame result.  features_limit is rejected (SIFT_MI_EINVAL) while
 * n_bands > 1: it ranks the whole frame's keypoints, so apply it after the
 * merge.  Default band 0 of 1 (the whole frame). */
int sift_mi_set_row_band(sift_mi_ctx* ctx, uint32_t band, uint32_t n_bands);

/* Skip the device->host copy of results in batch calls (results stay in
 * device memory; see sift_mi_device_results).  Default 0 = copy. */
int sift_mi_set_keep_on_device(sift_mi_ctx* ctx, int keep);

/* Device pointers of the last batch's results (keep_on_device = 1): the
 * keypoints and descriptors of every frame, concatenated in frame order
 * (frame i at offsets[i] .. offsets[i+1]); valid until the next call. */
int sift_mi_device_results(sift_mi_ctx* ctx, const sift_mi_keypoint** d_kps, const uint8_t** d_desc, size_t* n);

/* Validation read-back (extension, not the crate): the Gaussian planes
 * G_0..G_5 of octave `octave` of frame `frame` of the last batch / sift()
 * call, as that call's pyramid left them in the context's arena -- (6, h, w)
 * f32 like sift_mi_read_scale_space, with (w, h) from
 * sift_mi_batch_octave_dims; `out_floats` is the capacity of `out`
 * (SIFT_MI_EINVAL below 6 * w * h).  Valid only when the last call ran as
 * one chunk (one frame, or sift_mi_set_chunk >= its frames) and until the
 * next call of any kind (precompute included); SIFT_MI_ESTATE otherwise.
 * Lets tests check the batch path's planes (which no DoG is materialised
 * for) against precompute_images. */
int sift_mi_batch_octave_dims(sift_mi_ctx* ctx, size_t octave, uint32_t* width, uint32_t* height);
int sift_mi_read_batch_scale_space(sift_mi_ctx* ctx, uint32_t frame, size_t octave, float* out, size_t out_floats);

/* Kernel-path switches (test / diagnostic, not configuration).  The default
 * of every option is the product path; each alternative computes the same
 * bits through a different kernel family, so the tests can hold every family
 * against the oracle.  Per context (no environment variables, no process-wide
 * state); waits for the context's work in flight.  SIFT_MI_EINVAL for an
 * unknown option or a value out of range. */
typedef enum {
    SIFT_MI_PATH_TILE_BLUR = 0,    /* 1: one-tile-per-workgroup blurs everywhere (default 0) */
    SIFT_MI_PATH_PAIR_BLUR = 1,    /* 0: no two-blur kernels (default 1) */
    SIFT_MI_PATH_SEED_PAIR = 2,    /* 0: seed and blur 1 as two launches (default 1) */
    SIFT_MI_PATH_TAIL = 3,         /* 0: per-blur launches for the small octaves (default 1) */
    SIFT_MI_PATH_FUSED_DETECT = 4, /* 0: blur 5 and the extremum scan apart; 2: fused wherever it
                                      applies, at 32-row segments (default 1: where it fills the chip) */
    SIFT_MI_PATH_EARLY = 5,        /* 0: one-chunk calls detect every octave after the tail (default 1) */
    SIFT_MI_PATH_DESC_FIRST = 6,   /* 0: one-frame calls order, then describe (default 1) */
    SIFT_MI_PATH_GRAPH = 7,        /* 1: identical single-chunk calls replayed as a HIP graph (default 0) */
    SIFT_MI_PATH_BAND_DRIFT = 8,   /* row bands: accepted refinement drift, -41..24 rows (default 24;
                                      smaller values force the whole-pyramid re-run) */
    SIFT_MI_PATH_BOUND_SHRINK = 9, /* k >= 1: first-chunk stage bounds / k (default 1; > 1 forces the
                                      bound-overflow re-run) */
    /* 10: retired (the round-5 split tail kernel, removed in round 6); setting it returns
       SIFT_MI_EINVAL */
    SIFT_MI_PATH_LARGE_FIRST = 11, /* 0: one-chunk calls orient the extrema in refinement order, not
                                      those with large windows first (default 1) */
    SIFT_MI_PATH_ONESWEEP = 12,    /* the emission-order sorts with rocprim's Onesweep radix sort: 1 at
                                      every size, 0 never, 2 from 524288 keys (default 0) */
    SIFT_MI_PATH_BD_PAIR = 13,     /* the fused blur 5 + extremum scan with two column strips per lane
                                      (packed f32): 1 (default) / 2 its two loop forms, 0 the one-column
                                      kernel */
    SIFT_MI_PATH_BD_WAVES = 14,    /* the pair kernel's fewest waves per launch when choosing its row
                                      segments, 1024..65536 */
    SIFT_MI_PATH_CHUNK_MODE = 15   /* automatic chunking: 1 (default) as few chunks as ~64 GB of pyramid
                                      (counted at 44 B per octave pixel) and ~1062 M seed pixels per chunk
                                      allow (128 x 1080p: one chunk); 0 at least two chunks per
                                      multi-frame call (both pipeline lanes busy), <= ~32 GB / ~531 M
                                      seed pixels each (rounds 1-5).  Either way a chunk is capped at
                                      40% of the device memory the context could use */
} sift_mi_path_option;
int sift_mi_set_path_option(sift_mi_ctx* ctx, int option, int value);

/* ---- src/lib.rs:123-143 `precompute_images` / `PrecomputedImages` ------- */
int sift_mi_precompute(sift_mi_ctx* ctx, const uint8_t* pixels, uint32_t width, uint32_t height,
                       size_t row_stride, size_t* n_octaves);
int sift_mi_octave_dims(sift_mi_ctx* ctx, size_t octave, uint32_t* width, uint32_t* height);
/* scale_space[octave]: (6, h, w) f32; dog[octave]: (5, h, w) f32 */
int sift_mi_read_scale_space(sift_mi_ctx* ctx, size_t octave, float* out);
int sift_mi_read_dog(sift_mi_ctx* ctx, size_t octave, float* out);

/* ---- src/lib.rs:147 `sift_with_precomputed(&PrecomputedImages, limit)` -- */
int sift_mi_sift_with_precomputed(sift_mi_ctx* ctx, int64_t features_limit, size_t* n_keypoints);

/* ---- src/lib.rs:785 `compute_descriptor(img, x, y, scale, orientation)` -
 * `img`: host f32 image (h, w); writes 128 bytes. */
int sift_mi_compute_descriptor(sift_mi_ctx* ctx, const float* img, uint32_t width, uint32_t height, float x,
                               float y, float scale, float orientation, uint8_t* out);

/* ---- src/lib.rs:86-90 `Processing` ops on host f32 images (op-level parity;
 * not the performance path) ------------------------------------------------ */
int sift_mi_gaussian_blur(sift_mi_ctx* ctx, const float* src, uint32_t width, uint32_t height, double sigma,
                          float* dst);
int sift_mi_resize_linear(sift_mi_ctx* ctx, const float* src, uint32_t width, uint32_t height, uint32_t dst_width,
                          uint32_t dst_height, float* dst);
int sift_mi_resize_nearest(sift_mi_ctx* ctx, const float* src, uint32_t width, uint32_t height, uint32_t dst_width,
                           uint32_t dst_height, float* dst);

/* ---- examples/sift-match.rs:30-35: cv::BFMatcher(NORM_L2, crossCheck)
 * .match(query, train) -- the step after the path.
 * query / train: (n, 128) u8 descriptor rows (SiftResult::descriptors).
 * distance = sqrt((float) exact integer L2^2); nearest = lowest index among
 * equal distances; cross_check != 0 keeps query i only when its nearest
 * train row's nearest query is i.  Matches are written in query order to
 * out[cap]; *n_matches = their count (SIFT_MI_EINVAL if cap is smaller, with
 * *n_matches set). */
typedef struct {
    int32_t query_idx, train_idx;
    float distance;
} sift_mi_match;
int sift_mi_match_descriptors(sift_mi_ctx* ctx, const uint8_t* query, size_t n_query, const uint8_t* train,
                              size_t n_train, int cross_check, sift_mi_match* out, size_t cap, size_t* n_matches);

/* ---- the input step before the path ---------------
 * Baseline (SOF0/SOF1) Huffman JPEG, 1 or 3 components -> 8-bit luma, with
 * the arithmetic of the reference's decode: image 0.25.2 `image::open` /
 * `load_from_memory` (zune-jpeg) then `.grayscale()` (examples/run-sift.rs:8,
 * src/lib.rs:1012).  Host entropy decoding, GPU IDCT / upsampling / colour.
 * sift_mi_jpeg_dims: frame size from the headers (host only, no device).
 * sift_mi_decode_jpeg: luma into out (row stride out_stride), a host buffer,
 * or device memory when out_on_device != 0 (ordered on the context stream;
 * the call returns once the frame is written). */
int sift_mi_jpeg_dims(const uint8_t* data, size_t len, uint32_t* width, uint32_t* height);
int sift_mi_decode_jpeg(sift_mi_ctx* ctx, const uint8_t* data, size_t len, uint8_t* out, size_t out_stride,
                        int out_on_device);
/* n JPEGs of one size and sampling -> device luma frames laid out as
 * sift_mi_extract_batch_device takes them (frame i at d_frames + i *
 * frame_pitch, rows row_stride apart).  Entropy decoding runs on `threads`
 * host threads (<= 0: up to 16), overlapped with the GPU reconstruction of
 * the previous chunk of frames; returns once every frame is written. */
int sift_mi_decode_jpeg_batch(sift_mi_ctx* ctx, const uint8_t* const* data, const size_t* len, uint32_t n,
                              uint8_t* d_frames, size_t frame_pitch, size_t row_stride, int threads);

/* ---- measurement ---------------------------------------------------------
 * Cumulative since the last reset.  The stage times (pyramid_ms ..
 * descriptor_ms, total_ms) come from HIP events that only the one-lane mode
 * records (sift_mi_set_pipeline_lanes(ctx, 1): the stage-timing mode; a
 * marker costs ~7 us of a stream's timeline, so the two-lane throughput mode
 * records none and leaves them at 0).  pyramid_* covers the seed + octave
 * blur kernels (the HBM-bound stage), which include the extremum scan of the
 * octaves detected with their last blur (k_blur_detect); pyramid_bytes is
 * SURVEY.md 8(d)'s algorithmic byte count W*H + 44*sum(P_o) per frame, and
 * pyramid_scan_bytes what the reference's scan reads for those fused
 * octaves (the five DoG planes once, 20 B per octave pixel), apart. */
typedef struct {
    double pyramid_ms;
    double detect_ms;
    double orient_ms;
    double order_ms;
    double descriptor_ms;
    double total_ms;
    uint64_t pyramid_bytes;
    uint64_t pyramid_launches;
    uint64_t frames;
    uint64_t extrema;
    uint64_t keypoints;
    uint64_t band_reruns;  /* row-band calls re-run on the whole-frame pyramid (sift_mi_set_row_band) */
    uint64_t stage_reruns; /* chunks re-run because a stage count exceeded its buffer bound */
    /* gradient samples evaluated (sift_mi_set_sample_counting on, else 0):
     * orientation = patch positions of gradient_direction_histogram
     * (src/lib.rs:657-757) inside the image, descriptors = samples of the
     * rotated 4x4 region that compute_descriptor (src/lib.rs:785-990) enumerates */
    uint64_t orient_samples;
    uint64_t desc_samples;
    uint64_t pyramid_scan_bytes;
} sift_mi_stats;
int sift_mi_get_stats(sift_mi_ctx* ctx, sift_mi_stats* out);
int sift_mi_reset_stats(sift_mi_ctx* ctx);
/* Measurement only: count the samples the orientation and descriptor kernels
 * evaluate (one device atomic per workgroup / per descriptor wave; off by
 * default, and off in every timed run).  Read with sift_mi_get_stats. */
int sift_mi_set_sample_counting(sift_mi_ctx* ctx, int on);

/* Library version string and last error (thread-local).
 * 0.4.0: sift_mi_set_path_option (replaces the environment knobs),
 *        sift_mi_batch_octave_dims, sift_mi_read_batch_scale_space takes the
 *        output capacity, sift_mi_stats gained pyramid_scan_bytes (pyramid_bytes
 *        no longer includes it).
 * 0.3.0: no ABI change from 0.2.
 * 0.2.0: emission keys (sift_mi_fetch_keys) widened x / y to 15 bits -- image
 *        field moved from bit 40 to bit 42; sift_mi_stats gained band_reruns,
 *        stage_reruns, orient_samples, desc_samples (a larger struct). */
const char* sift_mi_version(void);
const char* sift_mi_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SIFT_MI_H */
