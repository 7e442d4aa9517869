// Keypoint detection on MI355X: DoG extrema + sub-pixel refinement + contrast
// and edge rejection (k_detect_rows, k_refine), then 36-bin orientation histograms and
// reference orientations (k_orient).
//
// Reference: find_keypoints / find_extrema_in_dog_img / point_is_local_extremum
// / interpolate_extremum / extremum_contrast / extremum_is_on_edge /
// gradient_direction_histogram (src/lib.rs:281-757).
//
// Parity: every arithmetic expression keeps the reference's operand order
// (compiled with -ffp-contract=off).  The orientation histogram accumulates
// each bin in the reference's sequential row-major sample order (one lane
// per bin scanning the wave's LDS sample list), so bins are bit-identical to
// the CPU path and the keypoint count/order does not depend on reduction
// order.  Emission order (octave, s_init, y_init, x_init, peak) is restored
// by sorting the 64-bit emission keys afterwards (order.hip).
#include <algorithm>
#include <type_traits>

#include "launch_ext.h"
#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {

// ---------------------------------------------------------------------------
// interpolate_extremum (src/lib.rs:525-603) on the DoG stack of one frame.
// ---------------------------------------------------------------------------
// The batch path does not materialise the DoG planes: D_s = G_{s+1} - G_s is
// formed where it is read, with the same single f32 subtraction the blur
// epilogue uses when it does write D (pyramid.hip), so every value is
// bit-identical to the stored plane.
//
// One Newton step reads the 3x3x3 DoG neighbourhood of (s, y, x): the four
// Gaussians G_{s-1} .. G_{s+2} at rows y-1 .. y+1, columns x-1 .. x+1, i.e.
// twelve 12-byte row segments.  They are fetched as twelve 3-dword loads (one
// instruction each) instead of the 28 distinct single floats the expressions
// name: the kernel is bound by the address rate of its scattered loads (one
// candidate per lane, every lane a different row), not by arithmetic.  The
// unused corner values of the outer planes cost no extra cache line.
typedef float f3a __attribute__((ext_vector_type(3), aligned(4)));
typedef __attribute__((address_space(1))) const f3a gf3a;

struct Nbhd {
    float d[3][3][3];  // [prev / curr / next][row y-1 .. y+1][column x-1 .. x+1]
};

__device__ __forceinline__ void load_nbhd(const gfloat* g0, size_t P, int pitch, int s, int y, int x, Nbhd& n) {
    f3a g[4][3];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int r = 0; r < 3; r++)
            g[k][r] = *(const gf3a*)(g0 + (size_t)(s - 1 + k) * P + (size_t)(y - 1 + r) * pitch + (x - 1));
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int r = 0; r < 3; r++) {
            n.d[j][r][0] = g[j + 1][r].x - g[j][r].x;
            n.d[j][r][1] = g[j + 1][r].y - g[j][r].y;
            n.d[j][r][2] = g[j + 1][r].z - g[j][r].z;
        }
}

// ---------------------------------------------------------------------------
// k_refine: interpolate_extremum, extremum_contrast, extremum_is_on_edge
// (src/lib.rs:334-367, 525-653) for the candidate list.  A refinement is a
// STATE (candidate, current scale / row / column, steps taken, the octave's
// geometry) advanced by refine_step one Newton step at a time: exactly the
// reference's sequence of steps (same expressions, same order), decided after
// at most kMaxInterpSteps of them.
// ---------------------------------------------------------------------------
struct RefineState {
    uint64_t key;
    const gfloat* g0;    // G_0 of the candidate's frame and octave
    int W, H, pitch;     // the octave's geometry
    int vlo, vhi;        // rows of the octave's Gaussians that are exact (row bands)
    int sc, xi, yi, it;  // current scale, column, row; Newton steps taken
};

// The octaves' geometry, staged in LDS once per workgroup (a candidate's
// start then costs its key load only, not a second round trip for its
// octave's entries)
struct RefineOct {
    const float* g;
    size_t stride;
    int W, H, pitch;
};

// A new candidate's state: its key decoded and its octave's geometry looked
// up once (a Newton step then issues only the neighbourhood loads).
__device__ __forceinline__ void refine_start(const RefineLaunch& L, const RefineOct* geo, uint64_t key,
                                             RefineState& st) {
    const int b = (int)(key >> kKeyImgShift);
    const int o = (int)((key >> kKeyOctShift) & 15);
    const RefineOct& g = geo[o];
    st.key = key;
    st.W = g.W;
    st.H = g.H;
    st.pitch = g.pitch;
    st.g0 = as_global(g.g) + (size_t)(b - L.img_base) * g.stride;
    st.vlo = 0;
    st.vhi = st.H;
    if (L.band_flag) {
        st.vlo = max(0, (int)((uint64_t)st.H * L.band_r / L.band_n) - 1 - L.band_margin);
        st.vhi = min(st.H, (int)((uint64_t)st.H * (L.band_r + 1) / L.band_n) + 1 + L.band_margin);
    }
    st.sc = (int)((key >> kKeyScaleShift) & 3);
    st.yi = (int)((key >> kKeyYShift) & kKeyCoordMask);
    st.xi = (int)((key >> kKeyXShift) & kKeyCoordMask);
    st.it = 0;
}

// One step for state st.  Returns 1 (accepted: e filled), -1 (rejected) or 0
// (moved: another step follows).
__device__ __forceinline__ int refine_step(const RefineLaunch& L, RefineState& st, ExtRec& e) {
    const uint64_t key = st.key;
    const int W = st.W, H = st.H, pitch = st.pitch, vlo = st.vlo, vhi = st.vhi;
    const gfloat* g0 = st.g0;
    const size_t P = (size_t)pitch * H;
    const int x = st.xi, y = st.yi, scale = st.sc;
    // row bands with a restricted pyramid (host.cpp run_pyramid): the rows
    // read here must be computed ones, else the host recomputes the band on
    // the whole-frame pyramid
    if (L.band_flag && (y - 1 < vlo || y + 1 >= vhi)) atomicOr(L.band_flag, 1u);
    Nbhd n;
    load_nbhd(g0, P, pitch, scale, y, x, n);
    // interpolate_extremum (src/lib.rs:525-603), one iteration
    // AT(plane, dy, dx): plane 0 / 1 / 2 = prev / curr / next
#define AT(a, dy, dx) n.d[a][(dy) + 1][(dx) + 1]
    {
        const float g1 = (AT(2, 0, 0) - AT(0, 0, 0)) / 2.f;
        const float g2 = (AT(1, 1, 0) - AT(1, -1, 0)) / 2.f;
        const float g3 = (AT(1, 0, 1) - AT(1, 0, -1)) / 2.f;
        const float v2 = AT(1, 0, 0) * 2.f;
        const float h11 = AT(2, 0, 0) + AT(0, 0, 0) - v2;
        const float h12 = (AT(2, 1, 0) - AT(2, -1, 0) - AT(0, 1, 0) + AT(0, -1, 0)) / 4.f;
        const float h13 = (AT(2, 0, 1) - AT(2, 0, -1) - AT(0, 0, 1) + AT(0, 0, -1)) / 4.f;
        const float h22 = AT(1, 1, 0) + AT(1, -1, 0) - v2;
        const float h33 = AT(1, 0, 1) + AT(1, 0, -1) - v2;
        const float h23 = (AT(1, 1, 1) - AT(1, 1, -1) - AT(1, -1, 1) + AT(1, -1, -1)) / 4.f;
        const float det =
            h11 * h22 * h33 - h11 * h23 * h23 - h12 * h12 * h33 + 2.f * h12 * h13 * h23 - h13 * h13 * h22;
        const float i11 = (h22 * h33 - h23 * h23) / det;
        const float i12 = (h13 * h23 - h12 * h33) / det;
        const float i13 = (h12 * h23 - h13 * h22) / det;
        const float i22 = (h11 * h33 - h13 * h13) / det;
        const float i23 = (h12 * h13 - h11 * h23) / det;
        const float i33 = (h11 * h22 - h12 * h12) / det;
        const float s_ = -(i11 * g1 + i12 * g2 + i13 * g3);
        const float x_ = -(i13 * g1 + i23 * g2 + i33 * g3);
        const float y_ = -(i12 * g1 + i22 * g2 + i23 * g3);
        if (!(fabsf(s_) < 0.5f && fabsf(x_) < 0.5f && fabsf(y_) < 0.5f)) {
            // `x as isize + offset.round() as isize` (saturating), then bounds
            const int64_t LIM = (int64_t)1 << 40;
            const int64_t rx = sat_i64(roundf(x_)), ry = sat_i64(roundf(y_)), rs = sat_i64(roundf(s_));
            if (rx > LIM || rx < -LIM || ry > LIM || ry < -LIM || rs > LIM || rs < -LIM) return -1;
            const int64_t nx = x + rx, ny = y + ry, ns = scale + rs;
            if (!(ns >= 1 && ns <= kScalesPerOctave) || nx < kImageBorder || nx >= W - kImageBorder ||
                ny < kImageBorder || ny >= H - kImageBorder)
                return -1;
            st.xi = (int)nx;
            st.yi = (int)ny;
            st.sc = (int)ns;
            return ++st.it < kMaxInterpSteps ? 0 : -1;
        }
        e.off_s = s_;
        e.off_x = x_;
        e.off_y = y_;
    }
    // converged: extremum_contrast (src/lib.rs:606-626) on the same neighbourhood
    const float g1 = (AT(2, 0, 0) - AT(0, 0, 0)) / 2.f;
    const float g2 = (AT(1, 1, 0) - AT(1, -1, 0)) / 2.f;
    const float g3 = (AT(1, 0, 1) - AT(1, 0, -1)) / 2.f;
    const float interp = e.off_s * g1 + e.off_y * g2 + e.off_x * g3;
    const float contrast = fabsf(AT(1, 0, 0) + interp / 2.f);
    if (contrast * (float)kScalesPerOctave <= kContrastThreshold) return -1;
    // extremum_is_on_edge (src/lib.rs:630-653)
    const float v2 = AT(1, 0, 0) * 2.0f;
    const float h11 = AT(1, 1, 0) + AT(1, -1, 0) - v2;
    const float d22 = AT(1, 0, 1) + AT(1, 0, -1) - v2;
    const float h12 = (AT(1, 1, 1) - AT(1, 1, -1) - AT(1, -1, 1) + AT(1, -1, -1)) / 4.f;
#undef AT
    const float tr = d22 + h11;
    const float det = d22 * h11 - h12 * h12;
    if (det <= 0.f) return -1;
    if ((tr * tr * kEdgeThreshold) > (kEdgeThreshold + 1.0f) * (kEdgeThreshold + 1.0f) * det) return -1;
    // an accepted keypoint's orientation / descriptor patch must be exact too
    // (at the image's own top / bottom rows the patch reads clamp, so no limit)
    if (L.band_flag && ((vlo > 0 && y - L.band_patch < vlo) || (vhi < H && y + L.band_patch >= vhi)))
        atomicOr(L.band_flag, 1u);
    e.key = key;
    e.img = (int)(key >> kKeyImgShift);
    e.octave = (int)((key >> kKeyOctShift) & 15);
    e.scale = scale;
    e.x = x;
    e.y = y;
    e.response = contrast;
    e.pad = 0;
    return 1;
}

#ifndef SIFT_REFINE_WPE
#define SIFT_REFINE_WPE 1
#endif
// One candidate per lane for its whole refinement, the block's lanes
// grid-striding over the list.  (Round 5 also built persistent waves that
// refill a decided lane at once, so a wave never waits for its slowest
// lane's five steps -- with the next key prefetched and the geometry in LDS
// as here -- and measured them slower: 26.8-28.6 vs 23.3-25.4 us on octave 0
// of 64 frames, detect_ms 1.36-1.58 vs 1.19 per 128 frames.  The stage moves
// ~12 scattered 64-byte sectors per step; keeping more steps in flight per
// wave does not shorten that.)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_REFINE_WPE))) void k_refine(const RefineLaunch L) {
    __shared__ RefineOct geo[16];
    if ((int)threadIdx.x < L.n_oct && threadIdx.x < 16)
        geo[threadIdx.x] = RefineOct{L.gauss[threadIdx.x], L.g_img_stride[threadIdx.x], L.ow[threadIdx.x],
                                     L.oh[threadIdx.x], L.opitch[threadIdx.x]};
    __syncthreads();
    const uint32_t n = min(*L.n_cand, L.cand_cap);
    const int lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x * 256; base < n; base += gridDim.x * 256) {
        const uint32_t i = base + threadIdx.x;
        ExtRec e;
        int r = -1;
        if (i < n) {
            RefineState st;
            refine_start(L, geo, L.cand[i], st);
            do {
                r = refine_step(L, st, e);  // <= kMaxInterpSteps steps
            } while (r == 0);
        }
        const bool keep = r > 0;
        if (L.counter_hi) {  // two-ended: large windows from the front, the others from the back
            const bool large = keep && (float)e.scale + e.off_s >= kLargeWindowScale;
            const uint64_t ml = __ballot(large), ms = __ballot(keep && !large);
            uint32_t bl = 0, bs = 0;
            if (ml && lane == __ffsll((unsigned long long)ml) - 1) bl = atomicAdd(L.counter, (uint32_t)__popcll(ml));
            if (ms && lane == __ffsll((unsigned long long)ms) - 1) bs = atomicAdd(L.counter_hi, (uint32_t)__popcll(ms));
            if (ml) bl = __shfl(bl, __ffsll((unsigned long long)ml) - 1);
            if (ms) bs = __shfl(bs, __ffsll((unsigned long long)ms) - 1);
            const uint64_t below = (1ull << lane) - 1ull;
            if (large) {
                const uint32_t slot = bl + (uint32_t)__popcll(ml & below);
                if (slot < L.cap) L.out[slot] = e;
            } else if (keep) {
                const uint32_t j = bs + (uint32_t)__popcll(ms & below);
                if (j < L.cap) L.out[L.cap - 1 - j] = e;
            }
            continue;
        }
        const uint64_t mask = __ballot(keep);
        if (!mask) continue;
        const int leader = __ffsll((unsigned long long)mask) - 1;
        uint32_t b = 0;
        if (lane == leader) b = atomicAdd(L.counter, (uint32_t)__popcll(mask));
        b = __shfl(b, leader);
        const uint32_t slot = b + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
        if (keep && slot < L.cap) L.out[slot] = e;
    }
}

void launch_refine(const RefineLaunch& L, hipStream_t st) {
    if (L.cand_cap == 0) return;
    hipLaunchKernelGGL(k_refine, dim3(std::min<uint32_t>((L.cand_cap + 255) / 256, 2048)), dim3(256), 0, st, L);
}

// ---------------------------------------------------------------------------
// k_orient: one wave per accepted extremum (4 per workgroup).
// gradient_direction_histogram (src/lib.rs:657-757) + peak selection
// (src/lib.rs:369-431).  Samples are evaluated 64 at a time (one per lane) in
// the reference's row-major order; after each batch lane k < 36 adds the
// batch's bin-k samples in order (bit-identical to `raw_hist[bin + 2] +=
// w*mag`), while the next batch's gradient loads are in flight.
// ---------------------------------------------------------------------------
constexpr int OR_WT = 17 * 17;  // weight table (|yp|, |xp|) at the largest radius (16)

#ifndef SIFT_ORIENT_SUM_U
#define SIFT_ORIENT_SUM_U 1  // samples per step of the per-bin sums (batched kernel: 1 3.43 ms, 2 3.50, 3 3.62, 4 3.67 per 128 frames)
#endif
#ifndef SIFT_ORIENT_MIN_WAVES
#define SIFT_ORIENT_MIN_WAVES 8  // 8 waves per SIMD (64 VGPRs, 10 dwords spilled; no LDS limit since the sample list went): orientation 3.51 ms vs 3.54 at 7 waves, 3.57-3.62 at 6 (128 1080p frames)
#endif
// The correctly rounded angle of a near-tie sample, out of line: the f64
// atan2 needs ~50 VGPRs, which only the (rare) call site pays for.
__attribute__((noinline)) __device__ float orient_angle_f64(float dy, float dx) {
    return (float)atan2((double)dy, (double)dx);
}

__global__ __launch_bounds__(256, SIFT_ORIENT_MIN_WAVES) void k_orient(const OrientLaunch L) {
    __shared__ __attribute__((aligned(16))) float sval[4][64];  // the current batch of sample values
    __shared__ float swt[4][OR_WT];  // per-wave Gaussian weight table
    __shared__ uint32_t wcount[4], wbase, wsamp[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // two-ended ext (RefineLaunch::counter_hi): wave r < n_lo takes ext[r],
    // the next n_hi waves ext[cap - 1 - (r - n_lo)] (a total above the cap is
    // an overflow the host re-runs)
    const uint32_t n_lo = min(*L.n_ext, L.ext_cap);
    const uint32_t n_ext = L.n_ext_hi ? min(n_lo + min(*L.n_ext_hi, L.ext_cap), L.ext_cap) : n_lo;
    // one group of 4 extrema per workgroup; the grid covers the bound, the
    // device count ends it early (block-uniform).  (Round 5: the groups
    // remapped to contiguous ranges per XCD measured slower, together with
    // the same for the descriptor queues: 32.5-32.9 vs 32.2-32.4 ms per 128
    // 1080p frames, profiles/r05_xcd_local_ab.log.)
    {
        const uint32_t rg = blockIdx.x * 4;
        if (rg >= n_ext) return;
        const uint32_t r = rg + wave;
        const bool active = r < n_ext;
        ExtRec e;
        int W = 1, H = 1, pitch = 1, radius = 0, n = 1, N = 0;
        uint32_t nin = 0;  // patch positions inside the image (sample counting)
        float kp_scale = 0.f, kp_x = 0.f, kp_y = 0.f, osf = 1.f;
        float acc = 0.0f;  // lane k < 36: raw_hist[k + 2]
        if (active) {
            e = L.ext[r < n_lo ? r : L.ext_cap - 1 - (r - n_lo)];
            W = L.ow[e.octave];
            H = L.oh[e.octave];
            pitch = L.opitch[e.octave];
            const float* img = L.gauss[e.octave] + (size_t)(e.img - L.img_base) * L.gauss_img_stride[e.octave] +
                               (size_t)e.scale * pitch * H;
            osf = (float)(1u << e.octave);  // 2_f32.powi(octave)
            kp_scale = 0.8f * pow2_f32(((float)e.scale + e.off_s) / (float)kScalesPerOctave) * 2.f;
            kp_x = ((float)e.x + e.off_x) * osf;
            kp_y = ((float)e.y + e.off_y) * osf;
            radius = sat_i32(roundf(3.f * kLambdaOri * kp_scale));
            if (radius > 16) radius = 16;  // unreachable: kp_scale < 3.6 (assert-equivalent guard)
            if (radius < 0) radius = 0;
            n = 2 * radius + 1;
            N = n * n;
            const float sigma = kLambdaOri * kp_scale;
            const float gws = -1.0f / (2.0f * sigma * sigma);
            const float bin_step = (float)kOriBins / (3.14159265358979323846f * 2.f);
            const int x = e.x, y = e.y;
            // Gaussian weights: exp_f32((yp^2 + xp^2) * gws) depends on the
            // sample only through (max(|xp|,|yp|), min(|xp|,|yp|)): one
            // correctly rounded exp per triangle entry (<= 153) instead of one
            // per sample (<= 1089), looked up bit-identically below.
            // Stored at [a][b] and [b][a] of a 17 x 17 table: a sample's entry
            // is then |yp| * 17 + |xp| (one multiply-add).
            const int T = (radius + 1) * (radius + 2) / 2;
            for (int t = lane; t < T; t += 64) {
                int a = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
                a = (a + 1) * (a + 2) / 2 <= t ? a + 1 : (a * (a + 1) / 2 > t ? a - 1 : a);
                const int bb = t - a * (a + 1) / 2;
                const float wv = exp_f32((float)(a * a + bb * bb) * gws);
                swt[wave][a * 17 + bb] = wv;
                swt[wave][bb * 17 + a] = wv;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // The four neighbours of a sample, at clamped positions (samples
            // outside the image are dropped below); the loads of the lane's
            // next sample are in flight while the current batch is evaluated
            // and summed.  Buffer resource based one row and one column before
            // the plane: a sample's four neighbours are one 32-bit offset plus
            // a uniform soffset (one or two rows) and an immediate (0, 4, 8
            // bytes); the clamped position keeps every access inside the plane.
            // The resource starts at the row above the patch's first clamped
            // row and spans only the patch's rows, so offsets stay small
            // however large the plane (octave 0 of a 16384-px frame is 2^32
            // bytes: a plane-based 32-bit offset would wrap).
            const int rb = max(y - radius, 1);                    // first sample row (clamped)
            const int re = min(max(y + radius, 1), H - 2);        // last sample row (clamped)
            const __amdgpu_buffer_rsrc_t rs =
                uniform_rsrc(img + (ptrdiff_t)(rb - 1) * pitch - 1, (uint32_t)(re - rb + 3) * (uint32_t)pitch * 4u);
            const int s1 = __builtin_amdgcn_readfirstlane(4 * pitch), s2 = 2 * s1;
            auto fetch = [&](int iy, int ix, float& l, float& r, float& u, float& d) {
                const int yy = min(max(y + iy - radius, 1), H - 2), xx = min(max(x + ix - radius, 1), W - 2);
                const int vo = ((yy - rb) * pitch + xx) * 4;
                r = buffer_load_f32(rs, vo + 8, s1);
                l = buffer_load_f32(rs, vo, s1);
                u = buffer_load_f32(rs, vo + 4, 0);
                d = buffer_load_f32(rs, vo + 4, s2);
            };
            float nl = 0.f, nr = 0.f, nu = 0.f, nd = 0.f;
            // patch row / column of the lane's sample (cy, cx) and of its next
            // one (fy, fx), stepped by 64 samples without a division
            const int dq = 64 / n, dr = 64 - dq * n;
            auto adv = [&](int& ry, int& rx) {
                rx += dr;
                ry += dq;
                if (rx >= n) {
                    rx -= n;
                    ry++;
                }
            };
            float* sv = sval[wave];
            // IN: the whole patch lies inside the image, rows / columns 1 ..
            // H-2 / W-2 (most extrema; wave-uniform): no clamps, no per-sample
            // bounds test
            auto sample_loop = [&](auto in_tag) {
                constexpr bool IN = decltype(in_tag)::value;
                auto fetch_s = [&](int iy, int ix, float& l, float& r, float& u, float& d) {
                    if constexpr (IN) {
                        const int vo = ((y + iy - radius - rb) * pitch + (x + ix - radius)) * 4;
                        r = buffer_load_f32(rs, vo + 8, s1);
                        l = buffer_load_f32(rs, vo, s1);
                        u = buffer_load_f32(rs, vo + 4, 0);
                        d = buffer_load_f32(rs, vo + 4, s2);
                    } else {
                        fetch(iy, ix, l, r, u, d);
                    }
                };
                int cy = lane / n, cx = lane - (lane / n) * n;
                int fy = cy, fx = cx;
                adv(fy, fx);
                if (lane < N && (IN || (H > 2 && W > 2))) fetch_s(cy, cx, nl, nr, nu, nd);
                // one batch of 64 samples (the reference's row-major order) per
                // iteration: evaluate (lane = sample), then add the batch into
                // the per-bin sums (lane = bin)
                for (int t = 0; t < N; t += 64) {
                    const int idx = t + lane;
                    const float gl = nl, gr = nr, gu = nu, gd = nd;
                    if (idx + 64 < N && (IN || (H > 2 && W > 2))) fetch_s(fy, fx, nl, nr, nu, nd);
                    const int yp = cy - radius, xp = cx - radius;
                    cy = fy;
                    cx = fx;
                    adv(fy, fx);
                    const int yy = y + yp, xx = x + xp;
                    uint32_t bv = 0xffu;  // no bin: past N or outside the image
                    bool defer = false;
                    float val = 0.0f, dx = 0.0f, dy = 0.0f;
                    if (idx < N && (IN || (yy > 0 && yy < H - 1 && xx > 0 && xx < W - 1))) {
                        dx = gr - gl;
                        dy = gu - gd;
                        const float weight = swt[wave][abs(yp) * 17 + abs(xp)];
                        const float mag = sqrtf(dx * dx + dy * dy);
                        // The sample only needs its bin, round(bin_step * atan2f): a
                        // fast f32 atan2 (|error| <= 2.4e-7 rad -> the product moves
                        // by < 2e-6) decides it unless the product lies within 2e-5
                        // of a rounding boundary; those rare samples (~4e-5) take the
                        // correctly rounded f64 angle below.  Away from a tie,
                        // round(tf) = floor(tf) + (frac > 0.5); |tf| <= 18 (no
                        // saturation), and only a negative bin wraps.
                        const float ori = atan2_fast(dy, dx);
                        const float tf = bin_step * ori;
                        const float fl = floorf(tf), fr = tf - fl;
                        defer = fabsf(fr - 0.5f) < 2e-5f;
                        const int bi = (int)fl + (fr > 0.5f ? 1 : 0);
                        bv = (uint32_t)(bi < 0 ? bi + kOriBins : (bi >= kOriBins ? bi - kOriBins : bi));
                        val = weight * mag;
                    }
                    if (__ballot(defer)) {  // rare: the batch holds a near-tie sample
                        if (defer) {
                            int bi = sat_i32(roundf(bin_step * orient_angle_f64(dy, dx)));
                            bv = (uint32_t)(bi >= kOriBins ? bi - kOriBins : (bi < 0 ? bi + kOriBins : bi));
                        }
                    }
                    sv[lane] = val;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    // Lane b < 36 gets the mask of the batch's samples in bin b from
                    // six ballots of the bin bits, then adds exactly those samples
                    // in index order: the reference's per-bin order
                    // (`raw_hist[bin + 2] += w * mag`, bit-identical) at O(largest
                    // bin count per batch).  Samples with no bin match no lane.
                    uint64_t m = __ballot(bv < (uint32_t)kOriBins);
#pragma unroll
                    for (int i = 0; i < 6; i++) {
                        const uint64_t bi = __ballot((bv >> i) & 1u);
                        m &= ((lane >> i) & 1) ? bi : ~bi;
                    }
                    // SIFT_ORIENT_SUM_U samples per step: their LDS reads in flight
                    // together; a missing sample adds +0 (exact: acc >= +0)
                    auto run = [&](uint32_t mk, const float* vb) {
                        while (mk) {
                            int j[SIFT_ORIENT_SUM_U];
                            bool ok[SIFT_ORIENT_SUM_U];
                            j[0] = __builtin_ctz(mk);
                            ok[0] = true;
                            mk &= mk - 1u;
#pragma unroll
                            for (int u = 1; u < SIFT_ORIENT_SUM_U; u++) {
                                ok[u] = mk != 0u;
                                j[u] = ok[u] ? __builtin_ctz(mk) : j[0];
                                mk &= mk - 1u;
                            }
                            float v[SIFT_ORIENT_SUM_U];
#pragma unroll
                            for (int u = 0; u < SIFT_ORIENT_SUM_U; u++) v[u] = vb[j[u]];
#pragma unroll
                            for (int u = 0; u < SIFT_ORIENT_SUM_U; u++) acc += ok[u] ? v[u] : 0.0f;
                        }
                    };
                    run(lane < kOriBins ? (uint32_t)m : 0u, sv);
                    run(lane < kOriBins ? (uint32_t)(m >> 32) : 0u, sv + 32);
                    // the next batch's value store follows these reads in the
                    // wave's LDS order: no barrier needed before it
                }
            };
            if (y - radius >= 1 && y + radius <= H - 2 && x - radius >= 1 && x + radius <= W - 2)
                sample_loop(std::true_type{});
            else
                sample_loop(std::false_type{});
            if (L.samples) {  // measurement only
                const int y0 = max(y - radius, 1), y1 = min(y + radius, H - 2);
                const int x0 = max(x - radius, 1), x1 = min(x + radius, W - 2);
                nin = (y1 >= y0 && x1 >= x0) ? (uint32_t)((y1 - y0 + 1) * (x1 - x0 + 1)) : 0u;
            }
        }
        // circular [1,4,6,4,1]/16 smoothing (src/lib.rs:742-755)
        const int k = lane < kOriBins ? lane : 0;
        const float rm2 = __shfl(acc, (k + kOriBins - 2) % kOriBins);
        const float rm1 = __shfl(acc, (k + kOriBins - 1) % kOriBins);
        const float rp1 = __shfl(acc, (k + 1) % kOriBins);
        const float rp2 = __shfl(acc, (k + 2) % kOriBins);
        const float r0 = __shfl(acc, k);
        const float h = (rm2 + rp2) * (1.f / 16.f) + (rm1 + rp1) * (4.f / 16.f) + r0 * 6.f / 16.f;
        // max over the 36 bins
        float m = lane < kOriBins ? h : -1.0f;
    #pragma unroll
        for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        const float thr = m * kOriPeakRatio;
        const float hm = __shfl(h, (k + kOriBins - 1) % kOriBins);
        const float hp = __shfl(h, (k + 1) % kOriBins);
        const bool peak = lane < kOriBins && h > hm && h > hp && h >= thr;
        const uint64_t mask = __ballot(peak);
        const uint32_t npk = (uint32_t)__popcll(mask);
        // one global atomic per workgroup (4 waves)
        if (lane == 0) wcount[wave] = npk;
        if (L.samples && lane == 0) wsamp[wave] = nin;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t tot = wcount[0] + wcount[1] + wcount[2] + wcount[3];
            wbase = tot ? atomicAdd(L.counter, tot) : 0u;
            if (L.samples)
                atomicAdd(L.samples + (blockIdx.x & 7),
                          (unsigned long long)(wsamp[0] + wsamp[1] + wsamp[2] + wsamp[3]));
        }
        __syncthreads();
        uint32_t base = wbase;
        for (int w = 0; w < wave; w++) base += wcount[w];
        const uint32_t slot = base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
        if (!peak || slot >= L.cap) return;
        const float interp = (hm - hp) / (hm - 2.0f * h + hp);
        float bin = (float)k + 0.5f * interp;
        if (bin < 0.0f)
            bin = (float)kOriBins + bin;
        else if (bin >= (float)kOriBins)
            bin = bin - (float)kOriBins;
        KpRec kp;
        kp.key = e.key | (uint64_t)k;
        kp.img = e.img;
        kp.octave = e.octave;
        kp.scale = e.scale;

        kp.x = kp_x;
        kp.y = kp_y;
        kp.size = kp_scale * osf;
        kp.angle = 360.0f - (360.0f / (float)kOriBins) * bin;
        kp.response = e.response;
        desc_rotation(kp.angle, kp.sin_d, kp.cos_d);
        L.out[slot] = kp;
    }
}

void launch_orient(const OrientLaunch& L, hipStream_t st) {
    if (L.ext_cap == 0) return;
    dim3 grid((L.ext_cap + 3) / 4);
    klaunch(k_orient, grid, dim3(256), st, L);  // may carry a completion event (set_launch_done_event)
}

}  // namespace siftmi
