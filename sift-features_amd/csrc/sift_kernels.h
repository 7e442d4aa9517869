// Host-side launch interface of the HIP kernels (internal to libsift_mi.so).
#pragma once

#include <string>

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "sift_common.h"

namespace siftmi {

// cv::resize coefficient tables (device pointers), resizeGeneric_ layout.
struct ResizeTab {
    const int* xofs;
    const float* xa0;
    const float* xa1;
    const int* yofs;
    const float* ya0;
    const float* ya1;
    int xmax;
};

// image::imageops::resize sampling tables (ImageprocProcessing profile),
// per destination index: first source tap and up to kIpTaps normalised f32
// weights (zero-padded; an extra zero-weight tap adds +0 and changes nothing).
constexpr int kIpTaps = 3;
struct IpResizeTab {
    const int* xl;
    const float* xw;  // [dst_w][kIpTaps]
    const int* yl;
    const float* yw;  // [dst_h][kIpTaps]
};

// Arithmetic profile of the Processing backend (src/lib.rs:86-90).
enum : int { kProfileOpenCV = 0, kProfileImageproc = 1 };

// Kernel-path switches of one context (sift_mi_set_path_option).  The
// defaults are the product path; every alternative computes the same bits and
// exists so the tests can hold each kernel family against the oracle.  They
// live in the context (no process-wide state, nothing read from the
// environment).
// Onesweep from this many sort keys (PathOpts::onesweep = 2): below it rocprim's
// block sort + merge path is faster.  One 1080p frame (~12 k keys): 0.578 vs
// 0.71 ms per call with Onesweep; 256 x VGA (128-frame chunks, ~206 k keys):
// 10.08-10.29 vs 9.93-10.15 ms; 128 x 1080p (64-frame chunks, ~715 k keys):
// 31.69-31.73 vs 31.68-31.89 ms (profiles/r05_batch35.log, r05_vga35.log)
constexpr uint32_t kOnesweepMinKeys = 1u << 19;

struct PathOpts {
    int tile_blur = 0;     // 1: one-tile-per-workgroup blurs everywhere (no strip / pair kernels)
    int pair = 1;          // 0: no pair kernels (k_blur2_strip, k_seed_pair)
    int seed_pair = 1;     // 0: k_seed_strip, then blur 1 like the other octaves
    int tail = 1;          // 0: per-blur launches for the small octaves (no k_octave_tail)
    int fused_detect = 1;  // 0: blur 5 and the extremum scan apart; 2: fused at 32-row segments wherever it applies
    int early = 1;         // one-chunk calls: detection of the octaves below the tail beside the tail kernel
    int desc_first = 1;    // one-frame calls: descriptors beside the ordering stage
    int graph = 0;         // 1: single-chunk calls captured once and replayed as a HIP graph
    int band_drift = 24;   // row bands: refinement drift accepted without a re-run (< 24 forces re-runs)
    int bound_shrink = 1;  // > 1: first-chunk stage bounds divided by it (forces the overflow re-run)
    int large_first = 1;   // one-chunk early path: two-ended extremum append (RefineLaunch::counter_hi)
    int bd_pair = 1;       // k_blur_detect_pair (two column strips per lane, packed f32): 1 its steady loop
                           // unrolled by 12 rows, 2 by 4; 0 the one-column k_blur_detect
    int bd_waves = 8192;   // k_blur_detect_pair: fewest waves per launch at the chosen row segments
    int chunk_mode = 1;    // automatic chunking (SIFT_MI_PATH_CHUNK_MODE)
    int onesweep = 0;      // emission-order sorts with rocprim's Onesweep: 1 always, 0 never (the
                           // library default path), 2 for bounds >= kOnesweepMinKeys
};

// Image planes are row-pitched: element (y, x) at plane[y * pitch + x].
struct BlurLaunch {
    const float* src;
    size_t src_img_stride;
    float* dst;
    size_t dst_img_stride;
    float* dog;  // may be null
    size_t dog_img_stride;
    float* nxt;  // may be null: next octave base (nearest 1/2)
    size_t nxt_img_stride;
    int pitch_n, wn, hn;
    int W, H, pitch;
    int n_img;
    int y0, y1;  // output rows [y0, y1) only (rounded out to tiles); y1 <= y0: all rows
    BlurTaps taps;
    int profile;  // kProfileOpenCV | kProfileImageproc
};

struct SeedLaunch {
    const uint8_t* frames;
    size_t frame_pitch, row_stride;
    int sh, sw;      // source height, width
    ResizeTab tab;   // 2x bilinear tables (OpenCV profile)
    IpResizeTab iptab;  // 2x Triangle tables (Imageproc profile)
    int profile;
    float* dst;      // octave 0, plane 0
    size_t dst_img_stride;
    int W, H, pitch;  // seed (2x) geometry
    int n_img;
    int y0, y1;  // output rows [y0, y1) only (rounded out to tiles); y1 <= y0: all rows
    BlurTaps taps;
    // k_seed_pair's first workgroup also resets a chunk's counters (k_chunk_init's
    // words: 4 zeros, init_m x ~0, init_words zeros) when init_cnt is set
    uint32_t* init_cnt = nullptr;
    int init_m = 0, init_words = 0;
};


// Host wait for an event (host.cpp): spins ~1 ms, then polls with short
// sleeps, so a thread waiting for a multi-ms chunk does not hold a CPU the
// decode threads (or a CPU quota) need.
hipError_t host_wait_event(hipEvent_t e);

// jpeg.hip: baseline JPEG -> 8-bit luma (zune-jpeg + image::grayscale arithmetic)
int jpeg_dims(const uint8_t* data, size_t len, uint32_t* w, uint32_t* h, std::string& err);
int jpeg_decode_luma(const uint8_t* data, size_t len, uint8_t* out, size_t out_stride, bool out_on_device,
                     hipStream_t st, std::string& err);
// pinned coefficient buffers and device scratch of the batch decoder, kept by
// the context across calls (grow-only)
struct JpegBatchCache {
    int16_t* pin[2] = {nullptr, nullptr};
    hipEvent_t up[2] = {nullptr, nullptr};
    size_t pin_bytes = 0;
    uint8_t* dev = nullptr;
    size_t dev_bytes = 0;
    void release();
};
int jpeg_decode_batch(const uint8_t* const* data, const size_t* len, uint32_t n, uint8_t* d_out, size_t frame_pitch,
                      size_t stride, int threads, hipStream_t st, JpegBatchCache& cache, std::string& err);

// Every octave from o0 on of n_img frames in one launch (k_octave_tail): a
// workgroup per frame, the octave's planes in LDS.  The octave G bases are
// the lane arena's; G_0 of octave o0 must be in place.
constexpr int kTailMaxOct = 16;
constexpr int kTailLdsFloats = 39680;  // 155 KB: A, B, T with halos + the next G_0 (pyramid.hip)
struct TailLaunch {
    float* gauss[kTailMaxOct];
    size_t gstride[kTailMaxOct];
    int ow[kTailMaxOct], oh[kTailMaxOct], pitch[kTailMaxOct];
    int o0, n_oct, n_img, profile;
    int r[kImagesPerOctave];
    BlurTaps taps[kImagesPerOctave];
};
// first octave that fits the tail kernel (n_oct: none); radii[1..5] = the
// octave's blur radii
int tail_octave_start(const int* ow, const int* oh, int n_oct, const int* radii);
void launch_octave_tail(const TailLaunch& L, hipStream_t st);

// pyramid.hip
// The next kernel a pyramid launcher enqueues from this host thread signals
// e on completion (no marker packet of its own); launch_done_pending() is
// true while no launch has taken it (the caller then clears it and records e)
void set_launch_done_event(hipEvent_t e);
bool launch_done_pending();
int launch_blur(int radius, const BlurLaunch& L, hipStream_t st, const PathOpts& o = PathOpts{});
// two consecutive blurs of an octave (A then B, B.src == A.dst) in one pass;
// -1 when the pair kernel does not apply (the caller launches them singly)
int launch_blur_pair(int ra, int rb, const BlurLaunch& A, const BlurLaunch& B, hipStream_t st,
                     const PathOpts& o = PathOpts{});
int launch_seed(int radius, const SeedLaunch& L, hipStream_t st, const PathOpts& o = PathOpts{});
// the seed (radius rs) and blur 1 (radius rb; B.src == L.dst) in one pass
// (k_seed_pair: G_0 never read back); -1 when it does not apply
int launch_seed_pair(int rs, int rb, const SeedLaunch& L, const BlurLaunch& B, hipStream_t st,
                     const PathOpts& o = PathOpts{});
// D_s = G_{s+1} - G_s (s < 5) of an octave's G stack, for n images
void launch_dog(const float* gauss, size_t plane, size_t g_img_stride, float* dog, size_t dog_img_stride, int W, int H,
                int pitch, int n_img, hipStream_t st);
void launch_resize_linear_f32(const float* src, int sw, int sh, const ResizeTab& tab, float* dst, int dw, int dh,
                              hipStream_t st);
// image::imageops::resize (Imageproc profile, op level): generic tap tables
// with up to `taps` entries per index ([n][taps] weights)
void launch_ip_resize_f32(const float* src, int sw, int sh, const int* xl, const float* xw, int xtaps, const int* yl,
                          const float* yw, int ytaps, float* tmp, float* dst, int dw, int dh, hipStream_t st);
void launch_resize_nearest_f32(const float* src, int sw, const int* xofs, const int* yofs, float* dst, int dw, int dh,
                               hipStream_t st);

// detect.hip
// One launch over several octaves: octave i's strips take the blocks
// [block0[i], block0[i + 1]).
struct DetectOctave {
    const float* gauss;  // octave G_0 base, image b at gauss + b*img_stride, plane s at + s*pitch*H
    size_t img_stride;   // (the DoG planes are formed from G_0..G_5 as they are read)
    int W, H, pitch, octave;
    int y_lo, y_hi;  // candidate rows [y_lo, y_hi) (a row band; 0, H for the whole octave)
};
struct DetectLaunch {
    DetectOctave oct[kTailMaxOct];
    uint32_t block0[kTailMaxOct + 1];
    int n_oct, n_img, img_base;
    int sh;          // rows per strip (filled by launch_detect)
    uint64_t* cand;  // packed candidate keys (frame, octave, scale, y, x)
    uint32_t* counter;
    uint32_t cap;
};
// octaves L.oct[0 .. n_oct) (block0 and sh are filled here)
void launch_detect(DetectLaunch& L, hipStream_t st);
// The octave's blur 5 (G_4 -> G_5, radius R, whole planes) and its
// detection in one pass (k_blur_detect); -1 when it does not apply (the
// caller then runs launch_blur and the octave's k_detect_rows).  nsx, nsy,
// seg are filled here.
struct BlurDetectLaunch {
    float* gauss;       // octave G_0 base of the launch's first frame
    size_t img_stride;  // floats between frames
    int W, H, pitch, octave, n_img, img_base, profile;
    int nsx, nsy, seg;
    BlurTaps taps;      // blur 5
    uint64_t* cand;
    uint32_t* counter;
    uint32_t cap;
};
int launch_blur_detect(int R, BlurDetectLaunch& L, hipStream_t st, const PathOpts& o = PathOpts{});
// whether launch_blur_detect would launch (the same test, nothing enqueued)
bool blur_detect_applies(int R, const BlurDetectLaunch& L, const PathOpts& o = PathOpts{});

// Stage sizes live in device counters (no host round trip between stages):
// every consumer reads its count from device memory, clamps it to the buffer
// bound, and walks the items with a grid-stride loop.
struct RefineLaunch {
    const uint64_t* cand;
    const uint32_t* n_cand;  // device count (may exceed cand_cap: overflow, clamped)
    uint32_t cand_cap;
    // row bands with a restricted pyramid (null flag: no check): octave o's
    // Gaussians are exact on rows [H_o*r/n - 1 - margin, H_o*(r+1)/n + 1 + margin)
    // (clipped); the flag is set when a refinement reads outside them or an
    // accepted keypoint's patch (+-patch rows) leaves them
    uint32_t* band_flag;
    int band_r, band_n, band_margin, band_patch;
    const float* const* gauss;   // device array [n_octaves] of octave G_0 bases (D formed from G)
    const size_t* g_img_stride;  // device array [n_octaves]
    const int* ow;
    const int* oh;
    const int* opitch;
    int n_oct;  // entries of the device arrays above
    int img_base;
    ExtRec* out;
    uint32_t* counter;
    uint32_t cap;
    // two-ended append (null: off): extrema whose windows will be large
    // (refined scale s + off_s >= kLargeWindowScale) from the front
    // (counter), the others from the back (out[cap - 1 - j], j from
    // counter_hi), so k_orient takes the large windows first (longest-first
    // scheduling of one frame's orientation: 0.574-0.576 vs 0.580-0.581 ms
    // per 1080p call; the descriptor kernel's duration did not change, its
    // keypoints are appended in orientation completion order)
    uint32_t* counter_hi;
};
constexpr float kLargeWindowScale = 2.0f;
void launch_refine(const RefineLaunch& L, hipStream_t st);

struct OrientLaunch {
    const ExtRec* ext;
    const uint32_t* n_ext;  // device count, clamped to ext_cap
    const uint32_t* n_ext_hi;  // two-ended ext (RefineLaunch::counter_hi; null: off): back-end count
    uint32_t ext_cap;
    const float* const* gauss;     // device array [n_octaves] of octave G bases
    const size_t* gauss_img_stride;  // device array [n_octaves]
    const int* ow;                 // device arrays [n_octaves]
    const int* oh;
    const int* opitch;
    KpRec* out;
    uint32_t* counter;
    int img_base;
    uint32_t cap;
    unsigned long long* samples;  // 8 counters (measurement only; null: off)
};
void launch_orient(const OrientLaunch& L, hipStream_t st);

// order.hip
// keys/vals for the emission-order sort; returns temp bytes when temp == null.
size_t sort_pairs_u64(void* temp, size_t temp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                      uint32_t* vout, uint32_t n, int end_bit, hipStream_t st,
                      bool onesweep = false);
// keys[i] = emission key of kp i for i < min(*n, bound); keys beyond are
// padded with `pad` (sorts last); vals[i] = i
void launch_chunk_init(uint32_t* cnt, int m, int work_words, hipStream_t st);
void launch_make_sort_keys(const KpRec* kp, const uint32_t* n, uint32_t bound, uint64_t pad, uint64_t* keys,
                           uint32_t* vals, hipStream_t st);
// starts[f] = first index of frame f in the sorted keys (0xffffffff if none);
// starts must be pre-filled with 0xff bytes
void launch_frame_starts(const uint64_t* sorted_keys, const uint32_t* n, uint32_t bound, uint32_t* starts,
                         hipStream_t st);
// Per-frame output plan (features_limit, src/lib.rs:156-161), one wave:
// out_cnt[f], seg_off[f] (first sorted index of frame f), out_off[f] (first
// output index), use_resp[f] (frame truncated by response) and *n_out.
void launch_limit_plan(const uint32_t* starts, const uint32_t* n_kp, uint32_t bound, int n_img, int64_t limit,
                       uint32_t* out_cnt, uint32_t* seg_off, uint32_t* out_off, uint8_t* use_resp, uint32_t* n_out,
                       hipStream_t st);
// key = (frame << 32) | ~bits(response) over the emission order; padded beyond *n
void launch_make_resp_keys(const KpRec* kp, const uint32_t* order, const uint32_t* n, uint32_t bound, int img_base,
                           uint64_t pad, uint64_t* keys, uint32_t* vals, hipStream_t st);
// final[i] = src index for i < *n_out: for frame f, if use_resp[f] the
// response order, else the emission order
// one-frame calls: descriptors computed in keypoint index order (desc_in),
// then row j of the outputs = keypoint order[j] (descriptor, KeyPoint, key)
void launch_gather_out(const KpRec* kp, const uint32_t* order, const uint32_t* n_out, uint32_t bound,
                       const uint8_t* desc_in, uint8_t* desc_out, OutKp* out_kp, uint64_t* out_key, uint64_t key_base,
                       const uint32_t* cnt, uint32_t* h_cnt, int cnt_words, hipStream_t st);
void launch_select(const uint32_t* emis_order, const uint32_t* resp_order, const uint32_t* seg_off,
                   const uint32_t* out_off, const uint8_t* use_resp, int n_img, const uint32_t* n_out, uint32_t bound,
                   uint32_t* final_idx, hipStream_t st);

// match.hip: per query the nearest train row (or -1), its distance
void launch_match(const uint8_t* q, int nq, const uint8_t* t, int nt, int cross_check, float* qn, float* tn,
                  unsigned long long* row_best, unsigned long long* col_best, int* train_idx, float* dist,
                  hipStream_t st);

// describe.hip
// Descriptor work queues: keypoint i belongs to queue i % kDescQueues, which
// hands out its keypoints in order; 8 counters on separate 128-B lines (one
// per XCD) keep the same-address atomic rate at an eighth.
constexpr int kDescQueues = 8;
constexpr int kDescQueueStride = 32;  // uint32 words
constexpr int kDescWorkWords = kDescQueues * kDescQueueStride;

struct DescLaunch {
    const KpRec* kp;
    const uint32_t* idx;  // final order -> kp index (may be null = identity)
    const uint32_t* n;    // device count, clamped to bound
    uint32_t bound;
    uint32_t* work;       // kDescQueues zeroed work counters, kDescQueueStride words apart: waves
                          // take keypoints dynamically (costs vary ~20x)
    uint64_t key_base;    // added to the emission keys (frame offset of the chunk)
    const float* const* gauss;
    const size_t* gauss_img_stride;
    const int* ow;
    const int* oh;
    const int* opitch;
    int img_base;
    OutKp* out_kp;     // may be null
    uint64_t* out_key; // may be null
    uint8_t* out_desc;
    int exact;         // 1: bit-exact bin-owner accumulation (describe_wave_exact)
    unsigned long long* samples;  // 8 counters (measurement only; null: off)
};
void launch_describe(const DescLaunch& L, hipStream_t st);

// single-keypoint compute_descriptor on an arbitrary f32 image
void launch_describe_one(const float* img, int w, int h, float x, float y, float scale, float orientation,
                         uint8_t* out, hipStream_t st);

}  // namespace siftmi
