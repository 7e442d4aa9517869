// Shared constants, device records and arithmetic helpers of the MI355X SIFT
// path.  Every constant cites the reference definition in
// /root/reference/src/lib.rs.
//
// Numerics: this code is compiled with -ffp-contract=off (the Rust reference
// never contracts a*b+c) and only fuses where the reference's OpenCV
// backend fuses (explicit __builtin_fmaf in the blur passes).  f32 division
// and sqrt are the IEEE correctly-rounded HIP defaults.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace siftmi {

// packed f32 pairs / quads (v_pk_* arithmetic, 8- and 16-byte LDS accesses)
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kScalesPerOctave = 3;                  // src/lib.rs:92
constexpr int kImagesPerOctave = kScalesPerOctave + 3;  // 6 Gaussian images (src/lib.rs:218-221)
constexpr int kDogPerOctave = kScalesPerOctave + 2;     // 5 DoG images (src/lib.rs:277)
constexpr float kContrastThreshold = 0.04f;          // src/lib.rs:93
constexpr float kEdgeThreshold = 10.0f;              // src/lib.rs:94
constexpr int kImageBorder = 5;                      // src/lib.rs:100
constexpr int kOriBins = 36;                         // src/lib.rs:102
constexpr float kLambdaOri = 1.5f;                   // src/lib.rs:104
constexpr float kLambdaDescr = 3.0f;                 // src/lib.rs:105
constexpr int kDescHist = 4;                         // src/lib.rs:108
constexpr int kDescBins = 8;                         // src/lib.rs:110
constexpr int kDescSize = 128;                       // src/lib.rs:111
constexpr float kOriPeakRatio = 0.8f;                // src/lib.rs:297
constexpr int kMaxInterpSteps = 5;                   // src/lib.rs:516
constexpr int kMaxBlurRadius = 31;                   // taps <= 63 per pass

// Emission key layout (see include/sift_mi.h, sift_mi_fetch_keys).  x_init
// and y_init are octave coordinates; octave 0 is the 2x seed, so a 16384-px
// frame needs 15 bits each (coordinates < 32768).
constexpr int kKeyImgShift = 42;    // [42,64): frame within the call (4M frames)
constexpr int kKeyOctShift = 38;    // [38,42)
constexpr int kKeyScaleShift = 36;  // [36,38)
constexpr int kKeyYShift = 21;      // [21,36)
constexpr int kKeyXShift = 6;       // [6,21)
constexpr uint32_t kKeyCoordMask = 0x7fff;
constexpr uint32_t kMaxFrameSide = 16384;  // 2*16384 - 5 < 2^15

__host__ __device__ inline uint64_t make_key(uint32_t img, uint32_t o, uint32_t s, uint32_t y, uint32_t x) {
    return ((uint64_t)img << kKeyImgShift) | ((uint64_t)o << kKeyOctShift) | ((uint64_t)s << kKeyScaleShift) |
           ((uint64_t)y << kKeyYShift) | ((uint64_t)x << kKeyXShift);
}

// Accepted extremum after interpolation + contrast + edge tests
// (src/lib.rs:334-367).  48 bytes.
struct ExtRec {
    uint64_t key;  // emission key without the peak field
    int32_t img, octave, scale, x, y;  // converged discrete point
    float off_s, off_x, off_y, response;
    int32_t pad;
};

// Keypoint with reference orientation (src/lib.rs:58-68 SiftKeyPoint), in
// 2x-seed pixel units.  48 bytes.  sin_d / cos_d: (sin, cos) of the
// descriptor's rotation, compute_descriptors' `360 - angle` in radians
// (src/lib.rs:771, :800-801), as compute_descriptor evaluates them -- computed
// once per keypoint by k_orient instead of by every lane of k_describe.
struct KpRec {
    uint64_t key;
    int32_t img, octave, scale;
    float sin_d;
    float x, y, size, angle, response;
    float cos_d;
};

// (sin, cos) of the descriptor rotation for a keypoint angle (degrees):
// orientation = 360 - angle (src/lib.rs:771), to_radians in f32, then f64
// sin / cos rounded to f32 (the reference's f32 sin / cos are correctly
// rounded glibc calls; up to rare near-midpoint ties this is the same value)
__device__ __forceinline__ void orientation_rotation(float orientation, float& s, float& c) {
    const float rad = orientation * (3.14159265358979323846f / 180.0f);  // f32::to_radians
    double sd, cd;
    sincos((double)rad, &sd, &cd);  // one argument reduction for both
    s = (float)sd;
    c = (float)cd;
}
__device__ __forceinline__ void desc_rotation(float angle, float& s, float& c) {
    orientation_rotation(360.0f - angle, s, c);
}

// Output keypoint (include/sift_mi.h sift_mi_keypoint).
struct OutKp {
    float x, y, size, angle, response;
};

// Blur taps, centre-indexed: k[0] = centre, k[t] = tap at distance t.
struct BlurTaps {
    float k[kMaxBlurRadius + 1];
};

// ---------------------------------------------------------------------------
// Rust-semantics helpers (saturating `as` casts, `.round()`)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t sat_i32(float v) {
    if (v != v) return 0;
    if (v >= 2147483647.0f) return INT32_MAX;
    if (v <= -2147483648.0f) return INT32_MIN;
    return (int32_t)v;
}
__device__ __forceinline__ int64_t sat_i64(float v) {
    if (v != v) return 0;
    if (v >= 9.2233720368547758e18f) return INT64_MAX;
    if (v <= -9.2233720368547758e18f) return INT64_MIN;
    return (int64_t)v;
}
__device__ __forceinline__ uint32_t sat_u32(float v) {  // `as usize` on small non-negative values
    if (!(v > 0.0f)) return 0;
    if (v >= 4294967295.0f) return 0xffffffffu;
    return (uint32_t)v;
}

// cv::borderInterpolate(BORDER_REFLECT_101)
__host__ __device__ __forceinline__ int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

// Global-address-space view of a pointer that the compiler only knows as
// generic (e.g. loaded from a device array of plane pointers): its loads
// become global_load (vmcnt only) instead of flat_load, which also counts
// against lgkmcnt and serialises with the kernel's LDS traffic.
typedef __attribute__((address_space(1))) const float gfloat;
__device__ __forceinline__ const gfloat* as_global(const float* p) { return (const gfloat*)p; }

// Buffer resource over `bytes` bytes at p (wave-uniform inputs: the halves of
// the pointer and the size go through readfirstlane so the descriptor lives
// in SGPRs).  Loads / stores then take a 32-bit per-lane voffset and a
// uniform soffset: no 64-bit address arithmetic per access.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* q = (void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ float buffer_load_f32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// XCD-aware tile order for (tx, ty, frames) grids.  The dispatcher deals
// workgroups round-robin over the 8 XCDs (each with a private 4 MB L2), so
// neighbouring tiles of a plain grid land on different XCDs and every halo
// row is re-read from HBM / Infinity Cache.  The bijective remap below gives
// each XCD a contiguous range of tile ids (cdna_hip_programming.md T1), walked
// row-major inside a frame: consecutive tiles of one XCD are horizontal
// neighbours (shared column halos, adjacent 256-B write segments), and the
// tile row above -- the vertical halo -- was loaded one tile row earlier
// (still in L2).
struct TileId {
    int x, y, z;
};
__device__ __forceinline__ TileId xcd_tile() {
    const uint32_t tx = gridDim.x, ty = gridDim.y;
    const uint32_t nwg = tx * ty * gridDim.z;
    const uint32_t orig = blockIdx.x + tx * (blockIdx.y + ty * blockIdx.z);
    const uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    const uint32_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
    const uint32_t per = tx * ty;
    const uint32_t z = t / per, rem = t - z * per;
    return {(int)(rem - (rem / tx) * tx), (int)(rem / tx), (int)z};
}

// The same bijection for a 1-D range of n items dealt round robin to the 8
// XCDs by index (item `orig` runs on XCD orig % 8): item orig becomes the
// returned index, so each XCD takes a contiguous range of [0, n).
__device__ __forceinline__ uint32_t xcd_remap(uint32_t orig, uint32_t n) {
    const uint32_t q = n / 8, r = n % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__host__ __device__ __forceinline__ int clamp_idx(int p, int len) { return p < 0 ? 0 : (p >= len ? len - 1 : p); }

// image 0.25.2 imageops::resize clamps every f32 output to [DEFAULT_MIN_VALUE,
// DEFAULT_MAX_VALUE] = [0, 1] (horizontal_sample's clamp), its Nearest 1/2
// included: the imageproc profile's next-octave base is the picked G_3 pixel
// clamped (a blur of values in [0, 1] can round a hair past 1)
__host__ __device__ __forceinline__ float ip_unit_clamp(float v) { return v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v); }

// Correctly rounded f32 transcendentals evaluated in f64 (the reference calls
// glibc expf/sinf/cosf/powf, which are correctly rounded in all but rare
// near-midpoint cases).
__device__ __forceinline__ float exp_f32(float x) { return (float)exp((double)x); }

// atan2(y, x) in radians in f32: |t| = min/max in [0, 1] (v_rcp_f32),
// atan(t) = t + t s P(s) (s = t^2, degree-7 minimax fitted in f64, |error| <
// 6e-8 on [0, 1] in f32), then the octant / quadrant reflections.  Measured
// against the correctly rounded f32 atan2 on 4M gradient pairs (f32 emulation
// with a 1-ulp reciprocal): |error| <= 2.4e-7 rad.  atan2(+0, +0) = 0 and
// atan2(+0, x < 0) = pi; callers pass gradient differences, never -0.
__device__ __forceinline__ float atan2_poly(float t) {
    const float sq = t * t;
    float p = 0.0025999427f;
    p = __builtin_fmaf(p, sq, -0.015042510f);
    p = __builtin_fmaf(p, sq, 0.040974170f);
    p = __builtin_fmaf(p, sq, -0.073540933f);
    p = __builtin_fmaf(p, sq, 0.10567977f);
    p = __builtin_fmaf(p, sq, -0.14184459f);
    p = __builtin_fmaf(p, sq, 0.19990212f);
    p = __builtin_fmaf(p, sq, -0.33332980f);
    return __builtin_fmaf(t * sq, p, t);
}
__device__ __forceinline__ float atan2_fast(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
    float v = atan2_poly(t);
    v = ay > ax ? 1.57079632679489662f - v : v;
    v = x < 0.0f ? 3.14159265358979324f - v : v;
    return y < 0.0f ? -v : v;
}
__device__ __forceinline__ float pow2_f32(float x) { return (float)exp2((double)x); }

}  // namespace siftmi
