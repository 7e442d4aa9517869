// Gaussian scale space + DoG on MI355X (gfx950).
//
// Reference: precompute_images / create_seed_image / build_gaussian_scale_space
// / build_dog (src/lib.rs:131-279) with the OpenCVProcessing backend
// (src/opencv_processing.rs:38-74): cv::resize INTER_LINEAR for the 2x seed,
// cv::GaussianBlur (separable, BORDER_REFLECT_101) for every blur and
// cv::resize INTER_NEAREST for the octave step.
//
// HBM layout: octave o of frame f is a [6][H_o][pitch_o] f32 Gaussian stack
// followed (per octave arena) by the [5][H_o][pitch_o] DoG stack; pitch_o is
// W_o rounded up to 64 floats so every row starts 256-B aligned.
//
// Kernels (batched over frames with blockIdx.z):
//   k_seed<TH>    u8 frame -> f32 (LUT v/255) -> 2x bilinear (OpenCV half-pixel
//                 coefficients, separately rounded products) computed on the fly
//                 for the tile + halo, then the seed blur (R = 5) -> G_0 of
//                 octave 0.  The upsampled image never touches HBM.
//   k_blur<R,TH>  one separable blur G_{s-1} -> G_s: interior tiles load the
//                 tile + halo with 16-B global loads into LDS (reflect-101
//                 scalar path only on border tiles), the row pass is register-
//                 blocked (4 outputs/thread, ds_read_b128), the column pass 8
//                 outputs/thread; the epilogue writes G_s, D_{s-1} = G_s -
//                 G_{s-1} and, for s == 3, the next octave's base image
//                 (nearest 1/2 = pixel (2x, 2y)).
// The stage is HBM-bound: per octave pixel the reference materialises 6 G + 5 D
// images (44 B); see DESIGN.md for the roofline accounting.
#include "launch_ext.h"
#include "sift_common.h"
#include "sift_kernels.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace siftmi {

void set_launch_done_event(hipEvent_t e) { t_done = e; }
bool launch_done_pending() { return t_done != nullptr; }


// ---------------------------------------------------------------------------
// Tile geometry.  Input window columns [x0 - HWL, x0 + TW + HWL) with
// HWL = R rounded up to 4 so every row segment is float4-aligned.
// ---------------------------------------------------------------------------
template <int R, int TH_, int QW_ = 8>
struct BlurGeom {
    static constexpr int TW = 64;
    static constexpr int TH = TH_;
    static constexpr int QW = QW_;                       // row-pass outputs per item (4 or 8)
    static constexpr int HWL = (R + 3) & ~3;
    static constexpr int IH = TH + 2 * R;                // rows of the input window / row-pass output
    static constexpr int IWV = TW + 2 * HWL;             // loaded columns (multiple of 4)
    static constexpr int IWP = IWV + 4;                  // LDS pitch (breaks 2^k strides)
    static constexpr int OFF = HWL - R;                  // first used column inside a float4
    static constexpr int NV = (HWL + R + QW + 3) / 4;    // float4 reads per row-pass item
    static constexpr int THP = IWP;                      // row-pass output written in place (see below)
    static constexpr int LDS_FLOATS = IH * IWP;
    static constexpr int NLOAD4 = IH * (IWV / 4);        // float4 per interior tile
    static constexpr int LOADS_PER_THREAD = (NLOAD4 + 255) / 256;
    static_assert(4 * NV <= IWV - TW + QW, "row-pass reads stay inside the loaded window");
    static_assert(TH % 8 == 0, "TH: the column pass gives each thread TH/8 rows");
};

// Row pass + column pass + epilogue, shared by the seed and octave kernels.
// The row pass writes its output in place over the input window (`th` ==
// `tin`): every row is filtered by 8 lanes of one wave, which read the whole
// row window into registers before any of them stores (LDS executes a wave's
// instructions in order), so no lane overwrites a value another still needs.
// The DoG needs G_{s-1} at the tile centre: each thread copies its centre
// values to registers before the row pass.
// Both passes use packed f32 arithmetic (v_pk_fma_f32 / v_pk_add_f32: two
// independent, individually rounded lanes -- the same results as scalar fma /
// add): the row pass pairs adjacent outputs of a row, the column pass
// adjacent columns.
// volatile LDS view: keeps each row-window read one ds_read_b128 (the compiler
// otherwise narrows the unused edge lanes into ds_read2_b32 pairs)
typedef __attribute__((address_space(3))) volatile f4v lds_f4v;
// and each column-pass read one ds_read_b64 (256 B/clk; the compiler would
// pair them into ds_read2_b64, which runs at half that rate)
typedef __attribute__((address_space(3))) volatile f2v lds_f2v;

// P = kProfileOpenCV: OpenCV's RowFilter (fma chain) + SymmColumnFilter
// (centre product, fma of pair sums).  P = kProfileImageproc: imageproc's
// separable_filter -- acc = acc + p * k from the first tap (unfused) in both
// passes -- and the nearest 1/2 at pixel (2x + 1, 2y + 1) (image's Nearest).
template <int R, int TH, int P = kProfileOpenCV>
__device__ __forceinline__ void blur_tile_compute(const float* __restrict__ tin, float* __restrict__ th,
                                                  const BlurTaps& taps, int x0, int y0, int W, int H, int pitch,
                                                  float* __restrict__ dst, float* __restrict__ dog,
                                                  float* __restrict__ nxt, int pitch_n, int wn, int hn) {
    using G = BlurGeom<R, TH>;
    constexpr int VB2 = TH / 8;  // column pass: thread = (column pair, VB2 consecutive rows)
    const int tid = threadIdx.x;
    const int cp = tid & 31, band = tid >> 5;
    f2v centre[VB2];
    if (dog) {
#pragma unroll
        for (int o = 0; o < VB2; o++)
            centre[o] = *reinterpret_cast<const f2v*>(tin + (band * VB2 + o + R) * G::IWP + G::HWL + 2 * cp);
        __syncthreads();  // other waves overwrite these rows in place below
    }
    // row pass: item = (row, QW consecutive outputs); fma chain from the leftmost tap.
    // A wave filters 8 whole rows per iteration.  Lane -> (row, item) follows
    // the ds_read_b128 lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} per
    // 32-lane half): each group reads two adjacent rows, whose float4 slots are
    // the even / odd slots of a bank row (IWP/4 is odd) -> conflict-free.
    static_assert(G::QW == 8 && (G::IWP / 4) % 2 == 1, "row-pass lane map assumes 8 items per row, odd pitch");
    const int lane = tid & 63, wv = tid >> 6;
    int rq;  // (row in wave) * 8 + item
    {
        const int l = lane & 31;
        int g, k;
        if (l < 4) { g = 0; k = l; }
        else if (l < 12) { g = 1; k = l - 4; }
        else if (l < 16) { g = 0; k = l - 8; }
        else if (l < 20) { g = 1; k = l - 8; }
        else if (l < 28) { g = 0; k = l - 12; }
        else { g = 1; k = l - 16; }
        rq = ((lane >> 5) * 4 + g * 2) * 8 + k;
    }
    for (int i = wv * 64 + rq; i < G::IH * 8; i += 256) {
        const int ly = i >> 3, q = i & 7;
        const lds_f4v* rp = (const lds_f4v*)(tin + ly * G::IWP + G::QW * q);
        float v[4 * G::NV];
#pragma unroll
        for (int j = 0; j < G::NV; j++) {
            const f4v f = rp[j];
            v[4 * j + 0] = f.x;
            v[4 * j + 1] = f.y;
            v[4 * j + 2] = f.z;
            v[4 * j + 3] = f.w;
        }
        float acc[G::QW];
#pragma unroll
        for (int o = 0; o < G::QW; o++) acc[o] = v[G::OFF + o] * taps.k[R];
#pragma unroll
        for (int t = 1; t <= 2 * R; t++) {
            const float kt = taps.k[t > R ? t - R : R - t];
#pragma unroll
            for (int o = 0; o < G::QW; o++)
                acc[o] = P == kProfileOpenCV ? __builtin_fmaf(v[G::OFF + o + t], kt, acc[o])
                                             : acc[o] + v[G::OFF + o + t] * kt;
        }
        // all lanes of this row have their window in registers (in-order LDS)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int o = 0; o < G::QW; o += 4)
            *reinterpret_cast<float4*>(th + ly * G::THP + G::QW * q + o) =
                make_float4(acc[o], acc[o + 1], acc[o + 2], acc[o + 3]);
    }
    __syncthreads();
    // column pass: centre product then fma of the (below + above) pair sums outwards
    f2v v[VB2 + 2 * R];
#pragma unroll
    for (int j = 0; j < VB2 + 2 * R; j++)
        v[j] = *(const lds_f2v*)(th + (band * VB2 + j) * G::THP + 2 * cp);
    const int gx = x0 + 2 * cp;  // even
    if (gx >= W) return;
    const bool pair = gx + 1 < W;
    const bool full = y0 + TH <= H;
    const f2v k0 = {taps.k[0], taps.k[0]};
#pragma unroll
    for (int o = 0; o < VB2; o++) {
        const int gy = y0 + band * VB2 + o;
        if (!full && gy >= H) break;
        f2v acc;
        if constexpr (P == kProfileOpenCV) {
            acc = v[o + R] * k0;
#pragma unroll
            for (int t = 1; t <= R; t++) {
                const f2v kt = {taps.k[t], taps.k[t]};
                acc = __builtin_elementwise_fma(v[o + R + t] + v[o + R - t], kt, acc);
            }
        } else {
            const f2v kr = {taps.k[R], taps.k[R]};
            acc = v[o] * kr;
#pragma unroll
            for (int t = 1; t <= 2 * R; t++) {
                const float k = taps.k[t > R ? t - R : R - t];
                const f2v kt = {k, k};
                acc = acc + v[o + t] * kt;
            }
        }
        const size_t off = (size_t)gy * pitch + gx;
        // dst == nullptr: G_s is not materialised (the batch path's G_5, only
        // its DoG is used downstream)
        if (pair) {
            if (dst) *reinterpret_cast<f2v*>(dst + off) = acc;
            if (dog) *reinterpret_cast<f2v*>(dog + off) = acc - centre[o];
        } else {
            if (dst) dst[off] = acc.x;
            if (dog) dog[off] = acc.x - centre[o].x;
        }
        // nearest 1/2: pixel (2x, 2y) for cv::resize INTER_NEAREST, (2x + 1,
        // 2y + 1) for image's Nearest; gy parity == o parity
        if constexpr (P == kProfileOpenCV) {
            if ((o & 1) == 0 && nxt && (gx >> 1) < wn && (gy >> 1) < hn)
                nxt[(size_t)(gy >> 1) * pitch_n + (gx >> 1)] = acc.x;
        } else {
            if ((o & 1) == 1 && nxt && pair && (gx >> 1) < wn && (gy >> 1) < hn)
                nxt[(size_t)(gy >> 1) * pitch_n + (gx >> 1)] = ip_unit_clamp(acc.y);
        }
    }
}

// Border tiles: the window through reflect-101 (OpenCV) / clamp-to-edge
// (imageproc) indices, 8 independent loads in flight per thread per batch.
template <int R, int TH, int P>
__device__ __forceinline__ void load_window_border(float* __restrict__ tin, const float* __restrict__ sb, int x0,
                                                   int y0, int W, int H, int pitch) {
    using G = BlurGeom<R, TH>;
    constexpr int N = G::IH * G::IWV, KB = 8;
    for (int i0 = threadIdx.x; i0 < N; i0 += 256 * KB) {
        float v[KB];
#pragma unroll
        for (int k = 0; k < KB; k++) {
            const int i = min(i0 + 256 * k, N - 1);
            const int ly = i / G::IWV, lx = i - ly * G::IWV;
            const int gy = P == kProfileOpenCV ? reflect101(y0 - R + ly, H) : clamp_idx(y0 - R + ly, H);
            const int gx = P == kProfileOpenCV ? reflect101(x0 - G::HWL + lx, W) : clamp_idx(x0 - G::HWL + lx, W);
            v[k] = sb[(size_t)gy * pitch + gx];
        }
#pragma unroll
        for (int k = 0; k < KB; k++) {
            const int i = i0 + 256 * k;
            if (i < N) {
                const int ly = i / G::IWV, lx = i - ly * G::IWV;
                tin[ly * G::IWP + lx] = v[k];
            }
        }
    }
}

template <int R, int TH, int P>
__global__ __launch_bounds__(256) void k_blur(const float* __restrict__ src, size_t src_img_stride,
                                              float* __restrict__ dst, size_t dst_img_stride,
                                              float* __restrict__ dog, size_t dog_img_stride,
                                              float* __restrict__ nxt, size_t nxt_img_stride, int pitch_n, int wn,
                                              int hn, int W, int H, int pitch, const BlurTaps taps, int ty0) {
    using G = BlurGeom<R, TH>;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    float* tin = lds;  // [IH][IWP]  G_{s-1} window, then (in place) the row-pass output
    float* th = lds;
    const int tid = threadIdx.x;
    const TileId tile = xcd_tile();
    const int x0 = tile.x * G::TW, y0 = (tile.y + ty0) * G::TH;  // ty0: first tile row (row bands)
    const size_t b = tile.z;
    src += b * src_img_stride;
    const bool interior = x0 >= G::HWL && x0 + G::TW + G::HWL <= W && y0 >= R && y0 + G::TH + R <= H;
    if (interior) {
        // all loads in flight before the LDS stores (16 B per lane, coalesced rows)
        float4 tmp[G::LOADS_PER_THREAD];
        const float* base = src + (size_t)(y0 - R) * pitch + (x0 - G::HWL);
        // unconditional (index-clamped) loads: a guarded load makes hipcc wait
        // vmcnt(0) per element and spill the staging array to scratch
#pragma unroll
        for (int j = 0; j < G::LOADS_PER_THREAD; j++) {
            const int i = min(tid + 256 * j, G::NLOAD4 - 1);
            const int ly = i / (G::IWV / 4), c4 = i - ly * (G::IWV / 4);
            tmp[j] = *reinterpret_cast<const float4*>(base + (size_t)ly * pitch + 4 * c4);
        }
#pragma unroll
        for (int j = 0; j < G::LOADS_PER_THREAD; j++) {
            const int i = tid + 256 * j;
            if (i < G::NLOAD4) {
                const int ly = i / (G::IWV / 4), c4 = i - ly * (G::IWV / 4);
                *reinterpret_cast<float4*>(tin + ly * G::IWP + 4 * c4) = tmp[j];
            }
        }
    } else {
        load_window_border<R, TH, P>(tin, src, x0, y0, W, H, pitch);  // BORDER_REFLECT_101 / clamp to edge
    }
    __syncthreads();
    blur_tile_compute<R, TH, P>(tin, th, taps, x0, y0, W, H, pitch, dst ? dst + b * dst_img_stride : nullptr,
                             dog ? dog + b * dog_img_stride : nullptr, nxt ? nxt + b * nxt_img_stride : nullptr,
                             pitch_n, wn, hn);
}

// ---------------------------------------------------------------------------
// k_blur_strip: the same blur G_{s-1} -> G_s (same arithmetic as k_blur),
// streamed down a column strip instead of one tile per workgroup.
//
// A workgroup owns 128 output columns (64 lanes x a column pair) of a row
// segment [ys, ye) and walks down it in chunks of S = 32 rows.  Chunk c holds
// the row-pass output of window rows [ys - R + cS, ys - R + (c+1)S); the
// column pass for output rows [ys + kS, ys + (k+1)S) reads chunks k and k+1
// (S >= 2R), so every row-pass row is computed once per segment instead of
// (TH + 2R) / TH times per tile, and the global loads of chunk k+2 are in
// flight (registers) while chunk k+1 is row-filtered and chunk k column-
// filtered.  Two LDS slots of S x IWP floats hold the chunks; the row pass
// runs in place (each row's 16 items are one wave's lanes, which read their
// windows before any of them stores), so a slot is the loaded input and then
// the row-pass output.
//
// Per step (4096 outputs): [barrier] store prefetched chunk k+1 -> slot
// [(k+1)&1]; issue chunk k+2 loads; [barrier] row pass chunk k+1 in place;
// [barrier] column pass k.  The column pass code is instantiated per wave
// (rows w*8 .. w*8+7 of the step) so which slot each of its rows lives in is a
// compile-time choice and every LDS read is one ds_read_b64 with an immediate
// offset.
// ---------------------------------------------------------------------------
template <int R_, int S_ = 32, int HWL_ = -1>
struct StripGeom {
    static constexpr int R = R_;                      // blur radius
    static constexpr int TW = 128;                    // output columns per strip
    static constexpr int S = S_;                      // rows per chunk
    static constexpr int NW = 4;                      // waves per workgroup
    static constexpr int VB = S / NW;                 // column-pass rows per wave per step
    static constexpr int QW = 8;                      // row-pass outputs per item
    static constexpr int HWL = HWL_ < 0 ? (R + 3) & ~3 : HWL_;  // window halo (default: R rounded up to 4)
    static constexpr int IWV = TW + 2 * HWL;          // loaded columns per row (multiple of 8)
    static constexpr int IWP = IWV + 4;               // LDS row pitch: IWP / 4 odd
    static constexpr int OFF = HWL - R;
    static constexpr int NV = (HWL + R + QW + 3) / 4;  // float4 reads per row-pass item
    static constexpr int C4 = IWV / 4;                // float4 per loaded row
    static constexpr int NLOAD4 = S * C4;
    static constexpr int LPT = (NLOAD4 + 64 * NW - 1) / (64 * NW);
    static constexpr int SLOT = S * IWP;
    static constexpr int LDS_FLOATS = 2 * SLOT;
    // resident workgroups per CU that the LDS allows (<= 4): the register
    // budget follows.  R >= 10: at most 3 -- at 4 the R = 10 kernel spills
    // (128 VGPRs); at 3 it does not and runs 4% faster (octave 0 of 64
    // frames, tools/ubench_kernels.hip strip).  A second register buffer for
    // a prefetch depth of 2 chunks was slower at R = 8, 10 and no faster
    // elsewhere.
#ifndef SIFT_STRIP_MINB_CAP_R10
#define SIFT_STRIP_MINB_CAP_R10 3
#endif
    static constexpr int MINB0 = 163840 / (4 * LDS_FLOATS) < 4 ? 163840 / (4 * LDS_FLOATS) : 4;
    static constexpr int MINB = (R >= 10 && MINB0 > SIFT_STRIP_MINB_CAP_R10) ? SIFT_STRIP_MINB_CAP_R10 : MINB0;
    static constexpr int NCW = (2 * R + S - 1) / S + 1;  // chunks in a column-pass window (2, or 3 for S < 2R)
    static_assert(2 * R <= 2 * S, "a column-pass window spans at most three chunks");
    static_assert((IWP / 4) % 2 == 1, "row-pass lane groups: odd float4 pitch");
    static_assert(4 * NV <= IWV - TW + QW, "row-pass reads stay inside the loaded row");
    static_assert(S % 16 == 0 && TW / QW == 16, "row pass: a wave filters 4 rows x 16 items");
};
constexpr int kStripMaxR = 16;
// Cache policy of the Gaussian plane stores of the strip kernels: 2 = NT
// (streaming; the planes are far larger than the caches).  Measured on the
// whole bench: pyramid 14.7 -> 14.3 ms per 128 frames (SC0: no change).
#ifndef SIFT_STORE_CPOL
#define SIFT_STORE_CPOL 2
#endif

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// buffer offset past every plane (planes are < 2^31 bytes): a store there is
// dropped by the buffer's range check
constexpr uint32_t kStoreDrop = 0xfffffff0u;

// N stores the buffer drops.  A strip kernel's loop waits at its top for the
// chunk loads of the previous iteration, with the column pass's stores issued
// after them; the compiler counts those stores only if EVERY path into the
// loop top has as many -- so the prologue, which enters it after its loads
// and no column pass, issues the same number of dropped stores.
template <int N>
__device__ __forceinline__ void drop_stores(__amdgpu_buffer_rsrc_t r) {
#pragma unroll
    for (int i = 0; i < N; i++)  // distinct offsets: not merged as redundant stores
        __builtin_amdgcn_raw_buffer_store_b32(0u, r, kStoreDrop - 16u * (uint32_t)i, 0, 0);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Single reflection (the strip kernel runs only when W, H > R, so every index
// an output uses is in range after one reflection), then clamped: rows /
// columns loaded past what any output uses stay inside the image.
template <int P>
__device__ __forceinline__ int strip_index(int p, int n) {
    if (P == kProfileOpenCV) p = p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p);
    return p < 0 ? 0 : (p >= n ? n - 1 : p);
}

// Chunk rows [r0, r0 + S) of the source window into registers.  Interior
// chunks (all rows and the strip's whole window inside the image) are one
// 16-B buffer load per item with the row offset in soffset; border chunks
// load element-wise through strip_index.
template <int R, int P, class G = StripGeom<R>>
__device__ __forceinline__ void strip_load(float4 (&pre)[G::LPT], __amdgpu_buffer_rsrc_t rs, const int (&voff)[G::LPT],
                                           bool cols_in, int r0, int x0, int W, int H, int pitch) {
    if (cols_in && r0 >= 0 && r0 + G::S <= H) {
        const int so = r0 * pitch * 4;
#pragma unroll
        for (int j = 0; j < G::LPT; j++)
            pre[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[j], so, 0));
        return;
    }
#pragma unroll
    for (int j = 0; j < G::LPT; j++) {
        const int i = min((int)threadIdx.x + 64 * G::NW * j, G::NLOAD4 - 1);
        const int ly = i / G::C4, gx = x0 - G::HWL + 4 * (i - ly * G::C4);
        const int ro = strip_index<P>(r0 + ly, H) * pitch;
        float e[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            e[q] = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * (ro + strip_index<P>(gx + q, W)), 0, 0));
        pre[j] = make_float4(e[0], e[1], e[2], e[3]);
    }
}

template <class G>
__device__ __forceinline__ void strip_store(const float4 (&pre)[G::LPT], float* slot) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < G::LPT; j++) {
        const int i = tid + 64 * G::NW * j;
        if (G::NLOAD4 % (64 * G::NW) == 0 || i < G::NLOAD4) {
            const int ly = i / G::C4, c4 = i - ly * G::C4;
            *reinterpret_cast<float4*>(slot + ly * G::IWP + 4 * c4) = pre[j];
        }
    }
}

// Row-pass lane map: wave wv filters rows 4 wv .. 4 wv + 3 of each 16-row
// group, 16 items (8 outputs each) per row; lanes 0-31 rows 0, 1 (A, B),
// lanes 32-63 rows 2, 3.  An item's reads are float4 slots 2 pq + j of its
// row, its writes slots 2 pq and 2 pq + 1; the row pitch IWP / 4 is odd, so
// A's slots and B's have opposite parity.  Per 32 lanes, with k = lane & 3:
//     lanes   0-3  4-7  8-11  12-15  16-19  20-23  24-27  28-31
//     row      A    B    A     B      B      A      B      A
//     pq       k    k   8+k   8+k    4+k    4+k   12+k   12+k
// ds_read_b128 groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}; banks = slot
// mod 16) hold 8 A items with pq distinct mod 8 and 8 B items likewise;
// ds_write_b128 groups (8 contiguous lanes; banks = slot mod 8) hold 4 A and
// 4 B items with pq distinct mod 4 -> reads and writes conflict-free.
__device__ __forceinline__ void strip_rowpass_map(int lane, int wv, int& prow, int& pq) {
    const int idx = (lane >> 2) & 7, k = lane & 3;
    const int b = (idx & 1) ^ (idx >> 2);
    prow = wv * 4 + (lane >> 5) * 2 + b;
    pq = ((idx >> 1) & 1) * 8 + (idx >> 2) * 4 + k;
}

// Row pass of one chunk, in place: item = (row, 8 consecutive outputs), an FMA
// chain from the leftmost tap (OpenCV RowFilter) / unfused acc + p * k
// (imageproc).  Lane -> (row, item): strip_rowpass_map.
template <class G, int P>
__device__ __forceinline__ void strip_rowpass(float* slot, const BlurTaps& taps, int prow, int pq) {
    constexpr int R = G::R;
#pragma unroll
    for (int it = 0; it < G::S / 16; it++) {
        const int ly = it * 16 + prow;
        const lds_f4v* rp = (const lds_f4v*)(slot + ly * G::IWP + G::QW * pq);
        float v[4 * G::NV];
#pragma unroll
        for (int j = 0; j < G::NV; j++) {
            const f4v f = rp[j];
            v[4 * j + 0] = f.x;
            v[4 * j + 1] = f.y;
            v[4 * j + 2] = f.z;
            v[4 * j + 3] = f.w;
        }
        float acc[G::QW];
#pragma unroll
        for (int o = 0; o < G::QW; o++) acc[o] = v[G::OFF + o] * taps.k[R];
#pragma unroll
        for (int t = 1; t <= 2 * R; t++) {
            const float kt = taps.k[t > R ? t - R : R - t];
#pragma unroll
            for (int o = 0; o < G::QW; o++)
                acc[o] = P == kProfileOpenCV ? __builtin_fmaf(v[G::OFF + o + t], kt, acc[o])
                                             : acc[o] + v[G::OFF + o + t] * kt;
        }
        // every lane of this row has its window in registers (in-order LDS)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        float* wp = slot + ly * G::IWP + G::QW * pq;
        *reinterpret_cast<float4*>(wp) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(wp + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
}

// Column pass of wave WV for one step: output rows y0 = y + WV*VB .. + VB - 1
// of the column pair x0 + 2*lane.  Logical chunk row L (chunk k starts at
// output row y - R) is row L of slot a for L < S, row L - S of slot b
// otherwise -- a compile-time choice per row.  OpenCV's SymmColumnFilter
// (centre product, fma of pair sums) / imageproc's unfused chain.
// LOFF: the window starts LOFF rows into slot a (the seed pair's G_0 chunks
// start one row above their column-pass windows; k_seed_pair).
template <class G, int P, int WV, bool NXT, int LOFF = 0>
__device__ __forceinline__ void strip_colpass(const float* sa, const float* sb, const BlurTaps& taps, int lane,
                                              int y, int ye, int x0, int W, int pitch, __amdgpu_buffer_rsrc_t rd,
                                              __amdgpu_buffer_rsrc_t rn, int pitch_n, int wn, int hn) {
    constexpr int R = G::R;
    constexpr int NR = G::VB + 2 * R;
    static_assert(LOFF + G::NW * G::VB + 2 * R <= 2 * G::S, "the column-pass window lies in slots a and b");
    f2v v[NR];
#pragma unroll
    for (int j = 0; j < NR; j++) {
        const int L = LOFF + WV * G::VB + j;  // window row: slot a or b
        const float* rp = L < G::S ? sa + L * G::IWP : sb + (L - G::S) * G::IWP;
        v[j] = *(const lds_f2v*)(rp + 2 * lane);
    }
    f2v out[G::VB];
    const f2v k0 = {taps.k[0], taps.k[0]};
#pragma unroll
    for (int o = 0; o < G::VB; o++) {
        f2v acc;
        if constexpr (P == kProfileOpenCV) {
            acc = v[o + R] * k0;
#pragma unroll
            for (int t = 1; t <= R; t++) {
                const f2v kt = {taps.k[t], taps.k[t]};
                acc = __builtin_elementwise_fma(v[o + R + t] + v[o + R - t], kt, acc);
            }
        } else {
            const f2v kr = {taps.k[R], taps.k[R]};
            acc = v[o] * kr;
#pragma unroll
            for (int t = 1; t <= 2 * R; t++) {
                const float k = taps.k[t > R ? t - R : R - t];
                const f2v kt = {k, k};
                acc = acc + v[o + t] * kt;
            }
        }
        out[o] = acc;
    }
    const int y0 = y + WV * G::VB;
    // Every row issues one store (two with NXT) whatever the row / column
    // bounds: a store outside them gets its offset OR-ed with kStoreDrop (out
    // of range: the buffer drops it) instead of a branch, so the number of
    // stores after the next chunk's loads is static and the compiler's wait
    // for those loads does not also wait for these stores (loads and stores
    // share vmcnt on gfx9).  A pair whose second column is past the image
    // writes it into the row's padding (W odd: pitch > W), which nothing reads.
    const int nrow = min(G::VB, ye - y0);
    const int gx = x0 + 2 * lane;
    // offset = (row part, uniform) + (column part, per lane), OR-ed with
    // the row's and the lane's drop flags
    const uint32_t lane_col = (uint32_t)(gx * 4), lane_bad = gx < W ? 0u : kStoreDrop;
    const uint32_t lane_ncol = (uint32_t)((gx >> 1) * 4);
    const uint32_t lane_nbad = ((gx >> 1) < wn && (P == kProfileOpenCV || gx + 1 < W)) ? 0u : kStoreDrop;
#pragma unroll
    for (int o = 0; o < G::VB; o++) {
        const int gy = y0 + o;
        const uint32_t row_bad = o < nrow ? 0u : kStoreDrop;  // uniform
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, out[o]), rd,
                                              ((uint32_t)(gy * pitch * 4) + lane_col) | lane_bad | row_bad, 0,
                                              SIFT_STORE_CPOL);
        // nearest 1/2: pixel (2x, 2y) (cv::resize INTER_NEAREST) / (2x + 1, 2y + 1)
        // (image's Nearest); y0 is even (segments start at even rows,
        // strip_segment_rows), so those are the even / odd o
        if (NXT && (o & 1) == (P == kProfileOpenCV ? 0 : 1)) {  // o: unrolled constant
            const uint32_t nrow_bad = (gy >> 1) < hn ? row_bad : kStoreDrop;  // uniform
            // (the element's bits as u32x2(out[o]).y: see strip_colpass_clamped)
            const uint32_t odd = __builtin_bit_cast(u32x2, out[o]).y;
            const uint32_t val = P == kProfileOpenCV
                                     ? __builtin_bit_cast(u32x2, out[o]).x
                                     : __builtin_bit_cast(uint32_t, ip_unit_clamp(__builtin_bit_cast(float, odd)));
            __builtin_amdgcn_raw_buffer_store_b32(val, rn,
                                                  ((uint32_t)((gy >> 1) * pitch_n * 4) + lane_ncol) | lane_nbad |
                                                      nrow_bad,
                                                  0, 0);
        }
    }
}

// Column pass of wave WV with every row reference clamped to [0, H): the
// imageproc pair kernel's border chunks, whose G_s rows outside the image
// (computed from clamped input rows) are not copies of the edge rows as
// clamp-to-edge needs -- so they are never read: each tap reads the clamped
// row of the chunk window (window row 0 = G_s row y - R - LOFF) instead.
// Imageproc chain (acc = acc + v * k from the first tap), dynamic LDS offsets.
// NXT: image's Nearest 1/2 (pixel (2x + 1, 2y + 1): the odd rows' odd
// columns, as strip_colpass).
template <class G, bool NXT = false, int LOFF = 0>
__device__ __forceinline__ void strip_colpass_clamped(const float* sa, const float* sb, const BlurTaps& taps,
                                                      int lane, int wv, int y, int ye, int x0, int W, int H,
                                                      int pitch, __amdgpu_buffer_rsrc_t rd,
                                                      __amdgpu_buffer_rsrc_t rn, int pitch_n, int wn, int hn) {
    constexpr int R = G::R;
    const int y0 = y + wv * G::VB;
    const int nrow = min(G::VB, ye - y0);
    const int gx = x0 + 2 * lane;
    const uint32_t lane_col = (uint32_t)(gx * 4), lane_bad = gx < W ? 0u : kStoreDrop;
    const uint32_t lane_ncol = (uint32_t)((gx >> 1) * 4);
    const uint32_t lane_nbad = ((gx >> 1) < wn && gx + 1 < W) ? 0u : kStoreDrop;
    for (int o = 0; o < G::VB; o++) {
        const int gy = y0 + o;
        f2v acc = {0.0f, 0.0f};
#pragma unroll
        for (int t = 0; t <= 2 * R; t++) {
            const int L = min(max(gy - R + t, 0), H - 1) - (y - R - LOFF);
            const float* rp = L < G::S ? sa + L * G::IWP : sb + (L - G::S) * G::IWP;
            const f2v v = *(const lds_f2v*)(rp + 2 * lane);
            const float k = taps.k[t > R ? t - R : R - t];
            const f2v kt = {k, k};
            acc = t == 0 ? v * kt : acc + v * kt;
        }
        const uint32_t row_bad = o < nrow ? 0u : kStoreDrop;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, acc), rd,
                                              ((uint32_t)(gy * pitch * 4) + lane_col) | lane_bad | row_bad, 0,
                                              SIFT_STORE_CPOL);
        if (NXT && (gy & 1) == 1) {
            const uint32_t nrow_bad = (gy >> 1) < hn ? row_bad : kStoreDrop;
            // (the element as u32x2(acc).y: hipcc 7.2 stores element 0 for
            // bit_cast(uint32_t, acc.y) after the 64-bit store of acc here)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, ip_unit_clamp(__builtin_bit_cast(
                                                      float, __builtin_bit_cast(u32x2, acc).y))), rn,
                                                  ((uint32_t)((gy >> 1) * pitch_n * 4) + lane_ncol) | lane_nbad |
                                                      nrow_bad,
                                                  0, 0);
        }
    }
}

// grid: (strips, segments, frames); segment sg covers output rows
// [ya + sg * seg, min(yb, ya + (sg + 1) * seg)).  G_{s-1} / G_s planes are
// H * pitch floats (< 2^31 bytes: checked by the launcher).
// the next-octave stores of NXT (blur 3, R = 8) push it past 128 VGPRs:
// 3 workgroups per CU there instead of spilling (SIFT_STRIP_NXT_MINB)
#ifndef SIFT_STRIP_NXT_MINB
#define SIFT_STRIP_NXT_MINB 3
#endif
template <int R, bool NXT>
constexpr int strip_minb() {
    return (NXT && R >= 7 && StripGeom<R>::MINB > SIFT_STRIP_NXT_MINB) ? SIFT_STRIP_NXT_MINB : StripGeom<R>::MINB;
}

template <int R, int P, bool NXT>
__global__ __launch_bounds__(256, (strip_minb<R, NXT>())) void k_blur_strip(
    const float* __restrict__ src, size_t src_img_stride, float* __restrict__ dst, size_t dst_img_stride,
    float* __restrict__ nxt, size_t nxt_img_stride, int pitch_n, int wn, int hn, int W, int H, int pitch,
    const BlurTaps taps, int ya, int yb, int seg) {
    using G = StripGeom<R>;
    static_assert(G::NCW == 2, "two chunk slots");
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const TileId tile = xcd_tile();
    const int x0 = tile.x * G::TW;
    const int ys = ya + tile.y * seg, ye = min(yb, ys + seg);
    if (ys >= ye) return;
    const size_t b = tile.z;
    const uint32_t plane_bytes = (uint32_t)H * (uint32_t)pitch * 4u;
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(src + b * src_img_stride, plane_bytes);
    const __amdgpu_buffer_rsrc_t rd = uniform_rsrc(dst + b * dst_img_stride, plane_bytes);
    __amdgpu_buffer_rsrc_t rn = rd;
    if constexpr (NXT) rn = uniform_rsrc(nxt + b * nxt_img_stride, (uint32_t)hn * (uint32_t)pitch_n * 4u);
    // loads: item i = (row i / C4, float4 column i % C4) of the chunk
    const bool cols_in = x0 - G::HWL >= 0 && x0 + G::TW + G::HWL <= W;
    int voff[G::LPT];
#pragma unroll
    for (int j = 0; j < G::LPT; j++) {
        const int i = min(tid + 64 * G::NW * j, G::NLOAD4 - 1);
        const int ly = i / G::C4, c4 = i - ly * G::C4;
        voff[j] = (ly * pitch + x0 - G::HWL + 4 * c4) * 4;
    }
    int prow, pq;  // row-pass lane map
    strip_rowpass_map(lane, wv, prow, pq);
    const int nsteps = (ye - ys + G::S - 1) / G::S;
    float4 pre[G::LPT];
    strip_load<R, P>(pre, rs, voff, cols_in, ys - R, x0, W, H, pitch);
    strip_store<G>(pre, lds);
    strip_load<R, P>(pre, rs, voff, cols_in, ys - R + G::S, x0, W, H, pitch);
    drop_stores<G::VB * (NXT ? 2 : 1)>(rd);
    __syncthreads();
    strip_rowpass<G, P>(lds, taps, prow, pq);
    for (int k = 0; k < nsteps; k++) {
        float* sa = lds + (k & 1) * G::SLOT;
        float* sb = lds + ((k + 1) & 1) * G::SLOT;
        __syncthreads();  // column pass k - 1 is done with slot b
        strip_store<G>(pre, sb);
        if (k + 2 <= nsteps) strip_load<R, P>(pre, rs, voff, cols_in, ys - R + (k + 2) * G::S, x0, W, H, pitch);
        __syncthreads();
        strip_rowpass<G, P>(sb, taps, prow, pq);
        __syncthreads();
        const int y = ys + k * G::S;
        switch (wv) {
#define COLPASS(w)                                                                                      \
    case w:                                                                                             \
        strip_colpass<G, P, w, NXT>(sa, sb, taps, lane, y, ye, x0, W, pitch, rd, rn, pitch_n, wn, hn); \
        break;
            COLPASS(0) COLPASS(1) COLPASS(2) COLPASS(3)
            default:
                __builtin_unreachable();  // wv < 4: no store-free path (static vmcnt)
#undef COLPASS
        }
    }
}

// ---------------------------------------------------------------------------
// k_blur2_strip: two consecutive blurs of the chain, G_{s-1} -> G_s -> G_{s+1},
// in one streaming pass (OpenCV profile, both radii <= 8, 16-row chunks).
// G_s is written once and read zero times from HBM: 12 B per pixel of the
// pair instead of 16.
//
// A strip owns the 112 output columns [X, X + 112).  Blur A (radius Ra) is
// the strip scheme above with its 128 columns starting at X - 8: its column
// pass writes G_s rows into a ring of three LDS slots laid out as blur B's
// (radius Rb) input window [X - 8, X + 136), so B's row pass is the same
// 16-item lane map (its last 16 outputs read junk and are dropped) and B's
// column pass stores lanes 0..55.  Vertically B lags A by two chunks:
//   step k:  P1  store A-input chunk k + 1 (prefetched), prefetch k + 2
//            P2  row pass A on chunk k + 1 | row pass B on G_s chunk k - 1
//            P3  column pass A -> G_s chunk k (slot k % 3, HBM rows of this
//                segment) | column pass B -> G_{s+1} rows of chunk k - 2
// (one phase's two halves touch disjoint slots).
//
// Exactness at the image borders: G_s rows above / below the image come out
// of A's column pass as the reflect-101 images of real rows bit for bit (the
// pass is centre product + (below + above) pair sums, symmetric under
// reflection, and A's input rows are reflected), so only G_s COLUMNS outside
// the image -- A's row pass is an FMA chain from the leftmost tap, not
// symmetric -- are replaced by their reflect-101 sources before B's row pass.
// ---------------------------------------------------------------------------
template <int Ra, int Rb, int HA = -1>
struct PairGeom {
    using GA = StripGeom<Ra, 16, HA>;              // HA: A's window halo (8 for the seed loader's 144 columns)
    using GB = StripGeom<Rb, 16>;
    static constexpr int HB = GB::HWL;             // G_s halo columns of B's window
    static constexpr int TWO = GA::TW - 2 * HB;   // output columns per strip
    static constexpr int NBW = GB::NCW;           // G_s chunks in a column-pass window of B
    // B ring: the two-chunk window + the chunk being written (the two column
    // passes share a phase)
    static constexpr int NBR = NBW + 1;
    static constexpr int LDS_FLOATS = 2 * GA::SLOT + NBR * GB::SLOT;
    static constexpr int MINB = 163840 / (4 * LDS_FLOATS + 2048) < 4 ? 163840 / (4 * LDS_FLOATS + 2048) : 4;
    static_assert(GA::HWL <= 8 && GA::NCW == 2, "A: radius <= 8");
    static_assert(NBW == 2, "B: radius <= 8 (two-chunk column windows)");
    static_assert(GB::IWV >= GA::TW, "B's window holds A's 128 columns");
};

// A's column pass for wave WV: G_s rows y0 .. y0 + VB - 1 (y0 = first row of
// the chunk + WV*VB) of columns xa + 2*lane into B's slot, and into HBM for
// the rows [gys, gye) and columns [X, min(X + TWO, W)) this strip owns (NXT:
// with the next octave's base, nearest 1/2 = pixel (2x, 2y)).
template <class GA, int WV, bool NXT, int P = kProfileOpenCV>
__device__ __forceinline__ void pair_colpass_a(const float* sa, const float* sb, float* bslot, int bip,
                                               const BlurTaps& taps, int lane, int y, int gys, int gye, int xa,
                                               int hb, int W, int pitch, int two, __amdgpu_buffer_rsrc_t rd,
                                               __amdgpu_buffer_rsrc_t rn, int pitch_n, int wn, int hn) {
    constexpr int R = GA::R;
    constexpr int NR = GA::VB + 2 * R;
    f2v v[NR];
#pragma unroll
    for (int j = 0; j < NR; j++) {
        const int L = WV * GA::VB + j;
        const float* rp = L < GA::S ? sa + L * GA::IWP : sb + (L - GA::S) * GA::IWP;
        v[j] = *(const lds_f2v*)(rp + 2 * lane);
    }
    const f2v k0 = {taps.k[0], taps.k[0]};
    const int y0 = y + WV * GA::VB;
    const int gx = xa + 2 * lane;  // even
    const bool own = gx >= xa + hb && gx < xa + hb + two && gx < W;  // this strip's columns
    const uint32_t colbad = own ? 0u : kStoreDrop;

#pragma unroll
    for (int o = 0; o < GA::VB; o++) {
        f2v acc;
        if constexpr (P == kProfileOpenCV) {
            acc = v[o + R] * k0;
#pragma unroll
            for (int t = 1; t <= R; t++) {
                const f2v kt = {taps.k[t], taps.k[t]};
                acc = __builtin_elementwise_fma(v[o + R + t] + v[o + R - t], kt, acc);
            }
        } else {
            const f2v kr = {taps.k[R], taps.k[R]};
            acc = v[o] * kr;
#pragma unroll
            for (int t = 1; t <= 2 * R; t++) {
                const float k = taps.k[t > R ? t - R : R - t];
                const f2v kt = {k, k};
                acc = acc + v[o + t] * kt;
            }
        }
        *(f2v*)(bslot + (WV * GA::VB + o) * bip + 2 * lane) = acc;
        // predicated by out-of-range offsets, a static store count (see strip_colpass)
        const int gy = y0 + o;
        const uint32_t rowbad = gy >= gys && gy < gye ? 0u : kStoreDrop;  // uniform
        const uint32_t off = (uint32_t)((gy * pitch + gx) * 4);
        // (a pair past the image's last column writes into the row padding)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, acc), rd, off | colbad | rowbad, 0,
                                              SIFT_STORE_CPOL);
        if constexpr (NXT) {
            const uint32_t nbad = (gy & 1) == 0 && (gy >> 1) < hn ? rowbad : kStoreDrop;
            const uint32_t ncol = (gx >> 1) < wn ? colbad : kStoreDrop;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, acc.x), rn,
                                                  (uint32_t)(((gy >> 1) * pitch_n + (gx >> 1)) * 4) | ncol | nbad, 0,
                                                  0);
        }
    }
}

// A's input chunks from a G_{s-1} plane (k_blur2_strip): strip_load /
// strip_store of 16-row chunks of A's 144-column window.
template <int Ra, int P, class GA>
struct PlaneIn {
    float4 pre[GA::LPT];
    __amdgpu_buffer_rsrc_t rs;
    int voff[GA::LPT];
    bool cols_in;
    int xa, W, H, pitch;
    __device__ __forceinline__ void init(const float* src, int xa_, int W_, int H_, int pitch_) {
        xa = xa_, W = W_, H = H_, pitch = pitch_;
        rs = uniform_rsrc(src, (uint32_t)H * (uint32_t)pitch * 4u);
        cols_in = xa - GA::HWL >= 0 && xa + GA::TW + GA::HWL <= W;
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < GA::LPT; j++) {
            const int i = min(tid + 64 * GA::NW * j, GA::NLOAD4 - 1);
            const int ly = i / GA::C4, c4 = i - ly * GA::C4;
            voff[j] = (ly * pitch + xa - GA::HWL + 4 * c4) * 4;
        }
    }
    __device__ __forceinline__ void prefetch(int r0) { strip_load<Ra, P, GA>(pre, rs, voff, cols_in, r0, xa, W, H, pitch); }
    __device__ __forceinline__ void store(float* slot, int) { strip_store<GA>(pre, slot); }
};

// The two-blur streaming pass shared by k_blur2_strip and k_seed_pair (see
// above): A-input chunks from `ain`, G_s (A's output) and G_{s+1} (B's) to
// HBM through ra / rb; NXT / NXTB: the next octave's base from A's / B's
// column pass.  LOFF: G_s chunk k starts LOFF rows above B's window of
// output chunk k (A's input chunks start LOFF rows higher), so the seed
// loader's chunks start at odd window rows (its two-source-row fast path)
// while segments start at even rows.
template <int Ra, int Rb, bool NXT, int P, bool NXTB, int LOFF, int HA, class AIn>
__device__ __forceinline__ void blur2_body(AIn& ain, float* lds, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb,
                                           __amdgpu_buffer_rsrc_t rn, int pitch_n, int wn, int hn, int X, int ys,
                                           int ye, int W, int H, int pitch, const BlurTaps& taps_a,
                                           const BlurTaps& taps_b) {
    using Q = PairGeom<Ra, Rb, HA>;
    using GA = typename Q::GA;
    using GB = typename Q::GB;
    constexpr int S = GA::S;
    constexpr int NBW = Q::NBW, NBR = Q::NBR;
    static_assert(!(NXT && NXTB), "one next-octave output");
    float* aslot = lds;                   // 2 x GA::SLOT: A's input chunks (row-filtered in place)
    float* bslot = lds + 2 * GA::SLOT;    // NBR x GB::SLOT: G_s chunks (row-filtered in place)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int xa = X - Q::HB;             // A's 128 columns (= B's window) start here
    int prow, pq;  // row-pass lane map
    strip_rowpass_map(lane, wv, prow, pq);
    // G_s columns outside the image in a B slot row: replaced by their
    // reflect-101 sources (this wave's 4 rows, before its row pass B); only
    // strips at the left / right image border have any
    const bool fix_l = xa < 0, fix_r = xa + GA::TW > W;
    auto fixup = [&](float* slot) {
        if (!(fix_l || fix_r)) return;
        constexpr int NE = 4 * 2 * Q::HB, NIT = (NE + 63) / 64;
        float val[NIT];
        bool act[NIT];
        int dst[NIT];
#pragma unroll
        for (int it = 0; it < NIT; it++) {
            const int e = lane + 64 * it;
            const int r = wv * 4 + e / (2 * Q::HB), j = e % (2 * Q::HB);
            const int x = j < Q::HB ? xa + j : W + (j - Q::HB);  // left halo xa .. xa + HB - 1, right W .. W + HB - 1
            act[it] = e < NE && (j < Q::HB ? (fix_l && x < 0) : (fix_r && x - xa < GA::TW));
            dst[it] = r * GB::IWP + (x - xa);
            const int sx = P == kProfileOpenCV ? reflect101(x, W) : clamp_idx(x, W);
            val[it] = act[it] ? slot[r * GB::IWP + (sx - xa)] : 0.0f;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < NIT; it++)
            if (act[it]) slot[dst[it]] = val[it];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
    // chunks: G_{s+1} 0 .. nout-1; G_s 0 .. ng (B's windows reach NBW - 1
    // chunks past the last output chunk); A's input 0 .. ng + 1
    const int nout = (ye - ys + S - 1) / S;
    const int ng = nout + NBW - 2, na = ng + 1;
    const int ga = ys - Rb - Ra - LOFF;  // first A-input row (chunk 0)
    ain.prefetch(ga);
    ain.store(aslot, ga);
    ain.prefetch(ga + S);
    __syncthreads();
    strip_rowpass<GA, P>(aslot, taps_a, prow, pq);
    for (int k = 0; k <= nout + NBW - 1; k++) {
        __syncthreads();  // P1
        if (k + 1 <= na) {
            ain.store(aslot + ((k + 1) & 1) * GA::SLOT, ga + (k + 1) * S);
            if (k + 2 <= na) ain.prefetch(ga + (k + 2) * S);
        }
        __syncthreads();  // P2
        if (k + 1 <= na) strip_rowpass<GA, P>(aslot + ((k + 1) & 1) * GA::SLOT, taps_a, prow, pq);
        if (k >= 1 && k - 1 <= ng) {
            float* s1 = bslot + ((k - 1) % NBR) * GB::SLOT;
            fixup(s1);
            strip_rowpass<GB, P>(s1, taps_b, prow, pq);
        }
        // column pass B -> G_{s+1} rows of output chunk k - NBW (its G_s
        // chunks are row-filtered)
        auto colb = [&]() {
            if (!(k >= NBW && k - NBW < nout)) return;
            const int j = k - NBW;  // output chunk: G_s chunks j .. j + NBW - 1
            const float* s0 = bslot + (j % NBR) * GB::SLOT;
            const float* s1 = bslot + ((j + 1) % NBR) * GB::SLOT;
            const int y = ys + j * S;
            // imageproc: a wave whose taps reach rows outside the image reads
            // clamped rows instead (uniform branch; first / last chunks)
            if constexpr (P == kProfileImageproc) {
                const int y0 = y + wv * GB::VB;
                if (y0 - Rb < 0 || y0 + GB::VB - 1 + Rb > H - 1) {
                    if (lane < Q::TWO / 2)
                        strip_colpass_clamped<GB, NXTB, LOFF>(s0, s1, taps_b, lane, wv, y, ye, X, W, H, pitch, rb,
                                                              rn, pitch_n, wn, hn);
                    return;
                }
            }
            // after B's in-place row pass slot column c is output column X + c: lanes 0 .. TWO/2 - 1 are
            // this strip's columns (the rest read the junk past A's 128 columns)
            switch (wv) {
#define COLB(w)                                                                                                  \
    case w:                                                                                                      \
        if (lane < Q::TWO / 2)                                                                                   \
            strip_colpass<GB, P, w, NXTB, LOFF>(s0, s1, taps_b, lane, y, ye, X, W, pitch, rb, rn, pitch_n, wn, hn); \
        break;
                COLB(0) COLB(1) COLB(2) COLB(3)
                default:
                    __builtin_unreachable();
#undef COLB
            }
        };
        __syncthreads();  // P3
        if (k <= ng) {
            const float* s0 = aslot + (k & 1) * GA::SLOT;
            const float* s1 = aslot + ((k + 1) & 1) * GA::SLOT;
            float* dstb = bslot + (k % NBR) * GB::SLOT;
            const int y = ys - Rb - LOFF + k * S;  // first G_s row of chunk k
            switch (wv) {
#define COLA(w)                                                                                                       \
    case w:                                                                                                           \
        pair_colpass_a<GA, w, NXT, P>(s0, s1, dstb, GB::IWP, taps_a, lane, y, ys, ye, xa, Q::HB, W, pitch, Q::TWO, ra,\
                                   rn, pitch_n, wn, hn);                                                              \
        break;
                COLA(0) COLA(1) COLA(2) COLA(3)
                default:
                    __builtin_unreachable();
#undef COLA
            }
        }
        colb();
    }
}

template <int Ra, int Rb, bool NXT, int P = kProfileOpenCV, bool NXTB = false>
__global__ __launch_bounds__(256, (PairGeom<Ra, Rb>::MINB)) void k_blur2_strip(
    const float* __restrict__ src, size_t img_stride, float* __restrict__ dst_a, float* __restrict__ dst_b,
    float* __restrict__ nxt, size_t nxt_img_stride, int pitch_n, int wn, int hn, int W, int H, int pitch,
    const BlurTaps taps_a, const BlurTaps taps_b, int ya, int yb, int seg) {
    using Q = PairGeom<Ra, Rb>;
    static_assert(P == kProfileOpenCV || !NXT, "imageproc pairs: no next-octave output from A");
    __shared__ __attribute__((aligned(16))) float lds[Q::LDS_FLOATS];
    const TileId tile = xcd_tile();
    const int X = tile.x * Q::TWO;        // output columns [X, X + TWO)
    const int ys = ya + tile.y * seg, ye = min(yb, ys + seg);
    if (ys >= ye) return;
    const size_t b = tile.z;
    const uint32_t plane_bytes = (uint32_t)H * (uint32_t)pitch * 4u;
    const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(dst_a + b * img_stride, plane_bytes);
    const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(dst_b + b * img_stride, plane_bytes);
    __amdgpu_buffer_rsrc_t rn = ra;
    if constexpr (NXT || NXTB) rn = uniform_rsrc(nxt + b * nxt_img_stride, (uint32_t)hn * (uint32_t)pitch_n * 4u);
    PlaneIn<Ra, P, typename Q::GA> ain;
    ain.init(src + b * img_stride, X - Q::HB, W, H, pitch);
    blur2_body<Ra, Rb, NXT, P, NXTB, 0, -1>(ain, lds, ra, rb, rn, pitch_n, wn, hn, X, ys, ye, W, H, pitch, taps_a,
                                           taps_b);
}

// ---------------------------------------------------------------------------
// Seed: u8 -> f32 (v / 255, image::ConvertBuffer, src/lib.rs:198) -> 2x
// bilinear (cv::resize INTER_LINEAR, src/lib.rs:201-205) -> GaussianBlur
// (src/lib.rs:207-209), fused.  Coefficient tables are built on the host
// with OpenCV's formulas (resizeGeneric_).
// ---------------------------------------------------------------------------
// v / 255 (image::ConvertBuffer), correctly rounded, without a divide or an
// LDS table (data-dependent table reads bank-conflict): q = v * (1/255) is
// within an ulp, and one fma residual step rounds it correctly -- checked
// for all 256 inputs against IEEE division (tests/test_gpu_ops.py).
__device__ __forceinline__ float u8_unit(uint32_t v) {
    const float fv = (float)v, c = 1.0f / 255.0f;
    const float q = fv * c;
    return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, fv), c, q);
}

__device__ __forceinline__ float upsample_at(const uint8_t* __restrict__ src, size_t row_stride, int sh,
                                             const ResizeTab& tab, int dx, int dy) {
    const int sx = tab.xofs[dx];
    const bool two = dx < tab.xmax;
    const int sx1 = two ? sx + 1 : sx;
    const int sy0 = tab.yofs[dy];
    const int sy1 = sy0 + 1 < sh ? sy0 + 1 : sh - 1;
    const uint8_t* r0 = src + (size_t)sy0 * row_stride;
    const uint8_t* r1 = src + (size_t)sy1 * row_stride;
    const float p00 = u8_unit(r0[sx]), p01 = u8_unit(r0[sx1]);
    const float p10 = u8_unit(r1[sx]), p11 = u8_unit(r1[sx1]);
    const float a0 = tab.xa0[dx], a1 = tab.xa1[dx];
    // HResizeLinear: t = S[sx]*a0 + S[sx+1]*a1 (two roundings + add)
    const float h0 = two ? p00 * a0 + p01 * a1 : p00;
    const float h1 = two ? p10 * a0 + p11 * a1 : p10;
    // VResizeLinear: S0*b0 + S1*b1
    return h0 * tab.ya0[dy] + h1 * tab.ya1[dy];
}

// Index range [lo, hi] of the reflect-101 positions p0 .. p0 + n - 1 of an
// axis of length L (one reflection per side: n <= L).
__device__ __forceinline__ void reflect_range(int p0, int n, int L, int& lo, int& hi) {
    lo = max(p0, 0);
    hi = min(p0 + n - 1, L - 1);
    if (p0 < 0) hi = max(hi, min(-p0, L - 1));                    // left reflections 1 .. -p0
    if (p0 + n > L) lo = min(lo, max(2 * L - 1 - (p0 + n), 0));  // right ones down to 2L - 1 - (p0 + n)
}

template <int R, int TH>
__global__ __launch_bounds__(256) void k_seed(const uint8_t* __restrict__ frames, size_t frame_pitch,
                                              size_t row_stride, int sh, int sw, const ResizeTab tab,
                                              float* __restrict__ dst, size_t dst_img_stride, int W, int H,
                                              int pitch, const BlurTaps taps, int ty0) {
    using G = BlurGeom<R, TH>;
    // Source window of an exact 2x upsample: destination g reads source
    // floor(g / 2 - 0.25) and the next one, so the window's destination range
    // [glo, ghi] needs source [glo / 2 - 1, ghi / 2 + 1] (clamped): computed
    // here, no table reads before the source loads.
    constexpr int SR = G::IH / 2 + 4, SC = G::IWV / 2 + 4;
    constexpr int NW = (SC + 3) / 4 + 1;  // dwords per source row (unaligned start)
    constexpr int NLD = (SR * NW + 255) / 256;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    __shared__ float srcf[SR * SC];         // u8 -> f32 source window
    __shared__ __attribute__((aligned(16))) float hbuf[SR * G::IWV];  // HResizeLinear per source row
    // per window column / row: source index and coefficients (resize tables)
    __shared__ __attribute__((aligned(16))) int txo[G::IWV];
    __shared__ __attribute__((aligned(16))) float txa0[G::IWV], txa1[G::IWV];
    __shared__ int tyo[G::IH];
    __shared__ float tya0[G::IH], tya1[G::IH];
    static_assert(G::IWV % 4 == 0 && G::IWV <= 128 && G::IH <= 128, "table threads: columns 0..127, rows 128..255");
    float* tin = lds;
    float* th = lds;
    const int tid = threadIdx.x;
    const TileId tile = xcd_tile();
    const int x0 = tile.x * G::TW, y0 = (tile.y + ty0) * G::TH;  // ty0: first tile row (row bands)
    const size_t b = tile.z;
    const uint8_t* src = frames + b * frame_pitch;
    // the exact-2x window math needs single reflections and a 2x geometry
    const bool fast = W == 2 * sw && H == 2 * sh && W >= G::IWV && H >= G::IH;
    int sxa = 0, sya = 0, sxb = -1, syb = -1;
    if (fast) {
        int glo, ghi;
        reflect_range(x0 - G::HWL, G::IWV, W, glo, ghi);
        sxa = max(glo / 2 - 1, 0);
        sxb = min(ghi / 2 + 1, sw - 1);
        reflect_range(y0 - R, G::IH, H, glo, ghi);
        sya = max(glo / 2 - 1, 0);
        syb = min(ghi / 2 + 1, sh - 1);
    }
    // 1. in flight together: the window's source dwords and its resize table
    //    entries (threads 0..127: columns, 128..255: rows)
    const int a0 = sxa & ~3;  // first source dword (4-B aligned frame rows)
    const int nwr = (sxb - a0) / 4 + 1, nr = syb - sya + 1;
    // dword loads only when every row start is 4-byte aligned (odd strides /
    // unaligned frame bases take the byte path)
    const bool dw_ok = (((uintptr_t)src | (uintptr_t)row_stride) & 3u) == 0;
    uint32_t wv[NLD];
#pragma unroll
    for (int j = 0; j < NLD; j++) {
        const int i = tid + 256 * j;
        const int r = i / NW, w = i - r * NW;
        wv[j] = 0;
        if (fast && r < nr && w < nwr) {
            const int c = a0 + 4 * w;
            const uint8_t* p = src + (size_t)(sya + r) * row_stride + c;
            if (c + 3 < sw && dw_ok) {
                wv[j] = *reinterpret_cast<const uint32_t*>(p);
            } else {  // row end / unaligned rows: bytes only (the dword could run past the frame)
                for (int q = 0; q < 4 && c + q < sw; q++) wv[j] |= (uint32_t)p[q] << (8 * q);
            }
        }
    }
    {
        const int t = tid & 127;
        if (tid < 128 && t < G::IWV) {
            const int g = reflect101(x0 - G::HWL + t, W);
            const int s0 = tab.xofs[g];
            txo[t] = g < tab.xmax ? s0 : -1 - s0;  // < 0: single-tap right border
            txa0[t] = tab.xa0[g];
            txa1[t] = tab.xa1[g];
        } else if (tid >= 128 && t < G::IH) {
            const int g = reflect101(y0 - R + t, H);
            tyo[t] = tab.yofs[g];
            tya0[t] = tab.ya0[g];
            tya1[t] = tab.ya1[g];
        }
    }
    if (fast) {
        // 2. u8 -> f32 (v / 255) into the source window
#pragma unroll
        for (int j = 0; j < NLD; j++) {
            const int i = tid + 256 * j;
            const int r = i / NW, w = i - r * NW;
            if (r < nr && w < nwr) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int c = a0 + 4 * w + q - sxa;
                    if (c >= 0 && c < SC) srcf[r * SC + c] = u8_unit((wv[j] >> (8 * q)) & 0xff);
                }
            }
        }
        __syncthreads();
        // 3. HResizeLinear: t = S[sx]*a0 + S[sx+1]*a1 (two roundings + add); 4 columns per item
        constexpr int Q = G::IWV / 4;
        for (int i = tid; i < nr * Q; i += 256) {
            const int r = i / Q, c = (i - r * Q) * 4;
            const int4 xo = *reinterpret_cast<const int4*>(txo + c);
            const float4 w0 = *reinterpret_cast<const float4*>(txa0 + c);
            const float4 w1 = *reinterpret_cast<const float4*>(txa1 + c);
            const float* sr = srcf + r * SC - sxa;
            auto hres = [&](int o, float u0, float u1) {
                const bool two = o >= 0;
                const int sx = two ? o : -1 - o;
                const float p0 = sr[sx];
                return two ? p0 * u0 + sr[sx + 1] * u1 : p0;
            };
            *reinterpret_cast<float4*>(hbuf + r * G::IWV + c) =
                make_float4(hres(xo.x, w0.x, w1.x), hres(xo.y, w0.y, w1.y), hres(xo.z, w0.z, w1.z),
                            hres(xo.w, w0.w, w1.w));
        }
        __syncthreads();
        // 4. VResizeLinear: S0*b0 + S1*b1; 4 columns per item
        for (int i = tid; i < G::IH * Q; i += 256) {
            const int ly = i / Q, c = (i - ly * Q) * 4;
            const int s0 = tyo[ly];
            const int r0 = s0 - sya, r1 = min(s0 + 1, sh - 1) - sya;
            const float4 u = *reinterpret_cast<const float4*>(hbuf + r0 * G::IWV + c);
            const float4 v = *reinterpret_cast<const float4*>(hbuf + r1 * G::IWV + c);
            const float b0 = tya0[ly], b1 = tya1[ly];
            *reinterpret_cast<float4*>(tin + ly * G::IWP + c) =
                make_float4(u.x * b0 + v.x * b1, u.y * b0 + v.y * b1, u.z * b0 + v.z * b1, u.w * b0 + v.w * b1);
        }
    } else {  // small or non-2x frames: per pixel from the tables
        for (int i = tid; i < G::IH * G::IWV; i += 256) {
            const int ly = i / G::IWV, lx = i - ly * G::IWV;
            const int gy = reflect101(y0 - R + ly, H), gx = reflect101(x0 - G::HWL + lx, W);
            tin[ly * G::IWP + lx] = upsample_at(src, row_stride, sh, tab, gx, gy);
        }
    }
    __syncthreads();
    blur_tile_compute<R, TH>(tin, th, taps, x0, y0, W, H, pitch, dst + b * dst_img_stride, nullptr, nullptr, 0, 0,
                             0);
}

// ---------------------------------------------------------------------------
// k_seed_strip: the seed as a strip blur (StripGeom<5>: 128 columns, 32-row
// chunks, the same row / column passes and barriers as k_blur_strip) whose
// chunk loader computes the 2x bilinear upsample in registers instead of
// loading a plane.
//
// For an exact 2x upsample (W = 2 sw, H = 2 sh) cv_linear_coeffs has a closed
// form (src/lib.rs:201-205): destination index d = 0 takes
// source 0 with coefficients (1, 0); d = n - 1 the last source alone (rows:
// (1, 0) on a clamped second row); every other d takes sources (d - 1) >> 1
// and the next one with (0.75, 0.25) for odd d, (0.25, 0.75) for even d.  So
// no table is read.
//
// Loader item = 12 window columns x a pair of window rows (g, g + 1), g odd:
// in the interior both rows read source rows (g - 1) / 2 and the next, so
// HResizeLinear (two rounded products + add) runs once per source row for
// two output rows, and the 12 columns need 8 consecutive source bytes per
// source row -- fetched as the 4-byte-aligned dwords that hold them (no
// dword without a needed byte is read, so no access leaves the frame,
// whatever its stride or alignment).  Then v / 255 and VResizeLinear
// (S0 b0 + S1 b1), in packed f32 (two independently rounded lanes, the same
// bits as scalar).  Border items (a column outside [1, W - 2], a reflected
// or last row) take per-column tables and up to three source rows.  Wave w
// owns chunk rows 8w .. 8w + 7: lane l < 48 row pair 4w + (l & 3), column
// group l >> 2.  The items of chunk k + 2 are fetched while chunk k + 1 is
// row-filtered, as k_blur_strip prefetches its rows.  Chunks start at odd
// window rows when segments start at even rows (the launcher's choice);
// any start is exact, odd ones keep the interior pairs on two source rows.
// ---------------------------------------------------------------------------
// 2x bilinear source index and coefficients of destination d (0 <= d < n,
// n = 2 * ns): see above; `two` false: the single last source
__device__ __forceinline__ void seed_axis(int d, int n, int ns, int& s, float& a0, float& a1, bool& two) {
    two = true;
    if (d == 0) {
        s = 0;
        a0 = 1.0f;
        a1 = 0.0f;
    } else if (d == n - 1) {
        s = ns - 1;
        a0 = 1.0f;
        a1 = 0.0f;
        two = false;
    } else {
        s = (d - 1) >> 1;
        a0 = (d & 1) ? 0.75f : 0.25f;
        a1 = (d & 1) ? 0.25f : 0.75f;
    }
}

// v / 255 of two bytes (u8_unit, packed)
__device__ __forceinline__ f2v u8_unit2(float a, float b) {
    const f2v fv = {a, b}, c = {1.0f / 255.0f, 1.0f / 255.0f};
    const f2v q = fv * c;
    return __builtin_elementwise_fma(__builtin_elementwise_fma(-q, f2v{255.0f, 255.0f}, fv), c, q);
}

// 2x upsample chunk loader of the strip seeds (k_seed_strip):
// the closed-form coefficients and row-pair items described above, for a
// strip geometry G (S = 16 or 32 rows per chunk, 144 window columns) whose
// window starts at column xw0.  NOLOAD (timing ablation only): no loads, a
// constant chunk.
template <class G, int P, bool NOLOAD = false>
struct SeedLoader {
    // Every wave loads: 48 lanes per wave, NPW row pairs x NCG column groups.
    // S = 32 (k_seed_strip): items of 12 columns, 4 pairs per wave.  S = 16
    // (k_seed_pair): items of 6 columns, 2 pairs per wave -- with 12-column
    // items only waves 0, 1 had any, and the other two waited out the
    // loader's upsample at the next barrier.
    static constexpr int CW = G::S == 16 ? 6 : 12;  // window columns per item
    static constexpr int NCG = G::IWV / CW;         // column groups (24 / 12)
    static constexpr int NPW = G::S == 16 ? 2 : 4;  // row pairs per wave
    static constexpr int NLW = G::S / (2 * NPW);    // loading waves (4)
    static_assert(G::NW == 4 && G::IWV == 144 && NCG * NPW <= 64 && NLW * NPW * 2 == G::S && NLW == G::NW,
                  "loader item map");
    // border columns: per window column its source offset from the item's
    // first source byte (bits 0-3), single / two taps (bit 4), coefficients
    struct Tables {
        int info[G::IWV];
        float a0[G::IWV], a1[G::IWV];
        int smin[NCG];
    };
    __amdgpu_buffer_rsrc_t rs;
    uint32_t boff;
    size_t row_stride;
    int sh, sw, W, H;
    const Tables* tb;
    bool act, wxin;
    int pr, cg, c0, smin;
    // prefetched chunk: per source row (up to 3) the <= 3 dwords holding the
    // item's bytes, raw (the byte alignment waits until the chunk is stored,
    // so the loads stay in flight across a row and a column pass)
    uint32_t pw[3][3];
    uint32_t psh;  // byte offset of each source row (2 bits each)
    int pbase;     // first source row

    // threads 0 .. NCG-1 fill the border-column tables; the caller then
    // synchronises the workgroup before init()
    static __device__ __forceinline__ void tables(Tables& t, int xw0, int W, int sw) {
        const int tid = threadIdx.x;
        if (tid < NCG) {
            const int cb = xw0 + CW * tid;
            int lo = 1 << 30;
            int sx[CW];
            bool two[CW];
#pragma unroll
            for (int k = 0; k < CW; k++) {
                seed_axis(strip_index<P>(cb + k, W), W, sw, sx[k], t.a0[CW * tid + k], t.a1[CW * tid + k], two[k]);
                lo = min(lo, sx[k]);
            }
#pragma unroll
            for (int k = 0; k < CW; k++) t.info[CW * tid + k] = (sx[k] - lo) | (two[k] ? 16 : 0);
            t.smin[tid] = lo;  // CW (<= 12) columns span <= 8 sources
        }
    }
    __device__ __forceinline__ void init(const uint8_t* src, size_t row_stride_, int sh_, int sw_, int W_, int H_,
                                         int xw0, const Tables& t, int lane, int wv) {
        // the frame as a buffer from its 4-byte-aligned base (boff bytes before
        // it), sized to whole dwords: a dword holding a frame byte never faults
        row_stride = row_stride_;
        sh = sh_, sw = sw_, W = W_, H = H_;
        tb = &t;
        boff = (uint32_t)(uintptr_t)src & 3u;
        const uint32_t nbytes = (boff + (uint32_t)(sh - 1) * (uint32_t)row_stride + (uint32_t)sw + 3u) & ~3u;
        rs = uniform_rsrc(src - boff, nbytes);
        // this lane's item: row pair pr of the wave, column group cg
        act = wv < NLW && lane < NCG * NPW;
        pr = wv * NPW + (lane & (NPW - 1));
        cg = lane / NPW;
        c0 = xw0 + CW * cg;  // first window column (even)
        const bool xin = c0 >= 1 && c0 + CW - 1 <= W - 2;
        // wave-uniform path choice: a wave takes the table path when any of its
        // items needs it (only the first / last strip of a row)
        wxin = __builtin_amdgcn_ballot_w64(act && !xin) == 0;
        smin = wxin ? c0 / 2 - 1 : t.smin[cg];
        psh = 0;
        pbase = 0;
    }
    __device__ __forceinline__ void rows_of(int g, int& sy0, int& sy1, float& b0, float& b1) const {
        bool two;
        seed_axis(strip_index<P>(g, H), H, sh, sy0, b0, b1, two);
        sy1 = min(sy0 + 1, sh - 1);
    }
    // interior chunk (uniform): window rows g0 .. g0 + S - 1 in [1, H - 2] and
    // g0 odd -- every pair (g, g + 1) reads source rows (g - 1) / 2 and the
    // next with coefficients (0.75, 0.25) / (0.25, 0.75), no table path
    __device__ __forceinline__ bool rows_in(int g0) const { return g0 >= 1 && g0 + G::S <= H - 1 && (g0 & 1) != 0; }
    __device__ __forceinline__ void prefetch(int g0) {
        if constexpr (NOLOAD) return;
        if (!act) return;
        const int g = g0 + 2 * pr;
        int nrows = 2;
        if (rows_in(g0)) {
            pbase = (g - 1) >> 1;
        } else {
            int a0, a1, c0_, c1_;
            float f0, f1;
            rows_of(g, a0, a1, f0, f1);
            rows_of(g + 1, c0_, c1_, f0, f1);
            pbase = min(a0, c0_);
            nrows = max(a1, c1_) - pbase + 1;  // <= 3
        }
        psh = 0;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            if (r < 2 || r < nrows) {
                // the three dwords from the one holding the first byte: the
                // buffer returns 0 for any past the frame's end
                const uint32_t off = boff + (uint32_t)(pbase + r) * (uint32_t)row_stride + (uint32_t)smin;
                const uint32_t o4 = off & ~3u;
                pw[r][0] = __builtin_amdgcn_raw_buffer_load_b32(rs, o4, 0, 0);
                pw[r][1] = __builtin_amdgcn_raw_buffer_load_b32(rs, o4 + 4u, 0, 0);
                pw[r][2] = __builtin_amdgcn_raw_buffer_load_b32(rs, o4 + 8u, 0, 0);
                psh |= (off & 3u) << (2 * r);
            }
        }
    }
    // the 8 source bytes of one source row as v / 255 (u8_unit)
    __device__ __forceinline__ void units(const uint32_t (&w)[3], uint32_t sh3, float (&p)[8]) const {
        const uint32_t lo = __builtin_amdgcn_alignbyte(w[1], w[0], sh3);
        const uint32_t hi = __builtin_amdgcn_alignbyte(w[2], w[1], sh3);
        // (float)(byte k): v_cvt_f32_ubyte{0..3}
        auto by = [](uint32_t w, int k) { return (float)((w >> (8 * k)) & 0xffu); };
        const f2v p01 = u8_unit2(by(lo, 0), by(lo, 1));
        const f2v p23 = u8_unit2(by(lo, 2), by(lo, 3));
        const f2v p45 = u8_unit2(by(hi, 0), by(hi, 1));
        const f2v p67 = u8_unit2(by(hi, 2), by(hi, 3));
        p[0] = p01.x, p[1] = p01.y, p[2] = p23.x, p[3] = p23.y;
        p[4] = p45.x, p[5] = p45.y, p[6] = p67.x, p[7] = p67.y;
    }
    // horizontal 2x step of one row's 12 window columns from its 8 source
    // values (OpenCV HResizeLinear: t = S[sx]*a0 + S[sx+1]*a1; imageproc's
    // Triangle horizontal_sample has the same two nonzero taps in the same
    // order -- its third, zero-weight tap adds +0)
    __device__ __forceinline__ void hmix(const float (&p)[8], float (&h)[CW]) const {
        if (wxin) {
            // column c0 + 2i: S[i] * 0.25 + S[i + 1] * 0.75; c0 + 2i + 1:
            // S[i + 1] * 0.75 + S[i + 2] * 0.25
            const f2v ka = {0.25f, 0.75f}, kb = {0.75f, 0.25f};
#pragma unroll
            for (int i = 0; i < CW / 2; i++) {
                const f2v v = f2v{p[i], p[i + 1]} * ka + f2v{p[i + 1], p[i + 2]} * kb;
                h[2 * i] = v.x;
                h[2 * i + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < CW; k++) {
                const int info = tb->info[CW * cg + k], d = info & 15;
                float v0 = p[0], v1 = p[1];
#pragma unroll
                for (int e = 1; e < 7; e++) {
                    v0 = d == e ? p[e] : v0;
                    v1 = d == e ? p[e + 1] : v1;
                }
                h[k] = (info & 16) ? v0 * tb->a0[CW * cg + k] + v1 * tb->a1[CW * cg + k] : v0;
            }
        }
    }
    // one item row of CW floats into the slot (16-B stores for 12 columns, 8-B
    // for 6: an item's first column is even, so 8-B aligned)
    __device__ __forceinline__ static void put_row(float* o, const float (&v)[CW]) {
        if constexpr (CW % 4 == 0) {
#pragma unroll
            for (int k = 0; k < CW; k += 4) *reinterpret_cast<float4*>(o + k) = make_float4(v[k], v[k + 1], v[k + 2], v[k + 3]);
        } else {
#pragma unroll
            for (int k = 0; k < CW; k += 2) *reinterpret_cast<float2*>(o + k) = make_float2(v[k], v[k + 1]);
        }
    }
    // HResizeLinear of one source row's CW columns from its (up to) 8 bytes
    __device__ __forceinline__ void hres(const uint32_t (&w)[3], uint32_t sh3, float (&h)[CW]) const {
        float p[8];
        units(w, sh3, p);
        hmix(p, h);
    }
    // the prefetched chunk (window rows from g0) -> upsampled rows of the
    // slot (row pitch G::IWP), rows 2 pr, 2 pr + 1
    __device__ __forceinline__ void store(float* slot, int g0) const {
        if (!act) return;
        const int g = g0 + 2 * pr;
        float* out = slot + (2 * pr) * G::IWP + CW * cg;
        int sy[2][2];
        float b[2][2];
        const bool rin = rows_in(g0);
        if (rin) {
            sy[0][0] = sy[1][0] = pbase;
            sy[0][1] = sy[1][1] = pbase + 1;
            b[0][0] = 0.75f;  // g odd
            b[0][1] = 0.25f;
            b[1][0] = 0.25f;  // g + 1 even
            b[1][1] = 0.75f;
        } else {
            rows_of(g, sy[0][0], sy[0][1], b[0][0], b[0][1]);
            rows_of(g + 1, sy[1][0], sy[1][1], b[1][0], b[1][1]);
        }
        // wave-uniform: every pair of the wave on two source rows (all but the
        // first / last chunks of a frame)
        const bool two_rows =
            rin || __builtin_amdgcn_ballot_w64(act && !(sy[0][0] == pbase && sy[1][0] == pbase &&
                                                       sy[0][1] == pbase + 1 && sy[1][1] == pbase + 1)) == 0;
        if constexpr (P == kProfileOpenCV) {
            // cv::resize: HResizeLinear per source row, then VResizeLinear
            float h0[CW], h1[CW];
            hres(pw[0], psh & 3u, h0);
            hres(pw[1], (psh >> 2) & 3u, h1);
#pragma unroll
            for (int r = 0; r < 2; r++) {
                float v[CW];
                if (two_rows) {
                    // VResizeLinear: S0*b0 + S1*b1
                    const f2v b0 = {b[r][0], b[r][0]}, b1 = {b[r][1], b[r][1]};
#pragma unroll
                    for (int k = 0; k < CW; k += 2) {
                        const f2v o = f2v{h0[k], h0[k + 1]} * b0 + f2v{h1[k], h1[k + 1]} * b1;
                        v[k] = o.x;
                        v[k + 1] = o.y;
                    }
                } else {  // border rows: any two of the three source rows
                    float h2[CW];
                    hres(pw[2], (psh >> 4) & 3u, h2);
                    const int i0 = sy[r][0] - pbase, i1 = sy[r][1] - pbase;
#pragma unroll
                    for (int k = 0; k < CW; k++) {
                        const float s0 = i0 == 0 ? h0[k] : (i0 == 1 ? h1[k] : h2[k]);
                        const float s1 = i1 == 0 ? h0[k] : (i1 == 1 ? h1[k] : h2[k]);
                        v[k] = s0 * b[r][0] + s1 * b[r][1];
                    }
                }
                put_row(out + r * G::IWP, v);
            }
        } else {
            // image::imageops::resize Triangle 2x: vertical_sample over the
            // item's 8 source columns, then horizontal_sample, clamped to
            // [0, 1].  Per destination index the nonzero taps and their order
            // are seed_axis' (the zero-weight third tap adds +0).
            float p0[8], p1[8];
            units(pw[0], psh & 3u, p0);
            units(pw[1], (psh >> 2) & 3u, p1);
            float p2[8];
            if (!two_rows) units(pw[2], (psh >> 4) & 3u, p2);
#pragma unroll
            for (int r = 0; r < 2; r++) {
                float vs[8];
                if (two_rows) {
                    const f2v b0 = {b[r][0], b[r][0]}, b1 = {b[r][1], b[r][1]};
#pragma unroll
                    for (int k = 0; k < 8; k += 2) {
                        const f2v o = f2v{p0[k], p0[k + 1]} * b0 + f2v{p1[k], p1[k + 1]} * b1;
                        vs[k] = o.x;
                        vs[k + 1] = o.y;
                    }
                } else {
                    const int i0 = sy[r][0] - pbase, i1 = sy[r][1] - pbase;
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        const float s0 = i0 == 0 ? p0[k] : (i0 == 1 ? p1[k] : p2[k]);
                        const float s1 = i1 == 0 ? p0[k] : (i1 == 1 ? p1[k] : p2[k]);
                        vs[k] = s0 * b[r][0] + s1 * b[r][1];
                    }
                }
                float v[CW];
                hmix(vs, v);
#pragma unroll
                for (int k = 0; k < CW; k++) v[k] = fminf(fmaxf(v[k], 0.0f), 1.0f);
                put_row(out + r * G::IWP, v);
            }
        }
    }
};

// A's input chunks computed from the u8 frame (k_seed_pair): the strip
// seed's 2x upsample loader (SeedLoader), 144 window columns from xa - 8.
template <class GA, int P>
struct SeedIn {
    SeedLoader<GA, P> ld;
    __device__ __forceinline__ void prefetch(int r0) { ld.prefetch(r0); }
    __device__ __forceinline__ void store(float* slot, int r0) { ld.store(slot, r0); }
};

// k_seed_pair: the seed blur and blur 1 of octave 0 in one pass -- A is the
// strip seed (u8 -> 2x upsample in registers -> R_seed blur, k_seed_strip's
// loader and arithmetic) writing G_0, B is blur 1 writing G_1: G_0 is written
// once and never read back (blur 2 then starts from G_1).
template <int Ra, int Rb, int P>
__global__ __launch_bounds__(256, (PairGeom<Ra, Rb, 8>::MINB)) void k_seed_pair(
    const uint8_t* __restrict__ frames, size_t frame_pitch, size_t row_stride, int sh, int sw,
    float* __restrict__ dst_a, float* __restrict__ dst_b, size_t img_stride, int W, int H, int pitch,
    const BlurTaps taps_a, const BlurTaps taps_b, int ya, int yb, int seg, uint32_t* __restrict__ init_cnt,
    int init_m, int init_words) {
    using Q = PairGeom<Ra, Rb, 8>;
    using GA = typename Q::GA;
    using L = SeedLoader<GA, P>;
    __shared__ __attribute__((aligned(16))) float lds[Q::LDS_FLOATS];
    __shared__ typename L::Tables tabs;
    const int tid = threadIdx.x, lane = tid & 63;
    if (init_cnt && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {  // the chunk's counters (k_chunk_init)
        for (int i = tid; i < 4 + init_m + init_words; i += 256)
            init_cnt[i < 4 + init_m ? i : i + init_m] = (i >= 4 && i < 4 + init_m) ? 0xffffffffu : 0u;
    }
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const TileId tile = xcd_tile();
    const int X = tile.x * Q::TWO;
    const int ys = ya + tile.y * seg, ye = min(yb, ys + seg);
    if (ys >= ye) return;
    const size_t b = tile.z;
    const uint32_t plane_bytes = (uint32_t)H * (uint32_t)pitch * 4u;
    const __amdgpu_buffer_rsrc_t ra = uniform_rsrc(dst_a + b * img_stride, plane_bytes);
    const __amdgpu_buffer_rsrc_t rb = uniform_rsrc(dst_b + b * img_stride, plane_bytes);
    const int xw0 = X - Q::HB - GA::HWL;  // A's window: 144 columns
    L::tables(tabs, xw0, W, sw);
    __syncthreads();
    SeedIn<GA, P> ain;
    ain.ld.init(frames + b * frame_pitch, row_stride, sh, sw, W, H, xw0, tabs, lane, wv);
    blur2_body<Ra, Rb, false, P, false, 1, 8>(ain, lds, ra, rb, ra, 0, 0, 0, X, ys, ye, W, H, pitch, taps_a, taps_b);
}

// ABL: timing ablations for tools/ubench_kernels.hip only (the product
// launches ABL = 0): 1 drops the plane stores (zero-size buffer), 2 the
// loader's loads and upsample, 4 the row pass
template <int R, int P = kProfileOpenCV, int ABL = 0>
__global__ __launch_bounds__(256, (StripGeom<R, 32, 8>::MINB)) void k_seed_strip(const uint8_t* __restrict__ frames,
                                                                        size_t frame_pitch, size_t row_stride, int sh,
                                                                        int sw, float* __restrict__ dst,
                                                                        size_t dst_img_stride, int W, int H, int pitch,
                                                                        const BlurTaps taps, int ya, int yb, int seg) {
    using G = StripGeom<R, 32, 8>;  // 8-column halo for any R <= 8: 144 = 12 x 12 window columns
    using L = SeedLoader<G, P, (ABL & 2) != 0>;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    __shared__ typename L::Tables tabs;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const TileId tile = xcd_tile();
    const int x0 = tile.x * G::TW;
    const int ys = ya + tile.y * seg, ye = min(yb, ys + seg);
    if (ys >= ye) return;
    const __amdgpu_buffer_rsrc_t rd =
        uniform_rsrc(dst + (size_t)tile.z * dst_img_stride, (ABL & 1) ? 0u : (uint32_t)H * (uint32_t)pitch * 4u);
    L::tables(tabs, x0 - G::HWL, W, sw);
    __syncthreads();
    L ld;
    ld.init(frames + (size_t)tile.z * frame_pitch, row_stride, sh, sw, W, H, x0 - G::HWL, tabs, lane, wv);
    int prow, pq;  // row-pass lane map
    strip_rowpass_map(lane, wv, prow, pq);
    const int nsteps = (ye - ys + G::S - 1) / G::S;
    const int gb = ys - R;  // window row of chunk 0
    ld.prefetch(gb);
    ld.store(lds, gb);
    ld.prefetch(gb + G::S);
    drop_stores<G::VB>(rd);
    __syncthreads();
    if constexpr ((ABL & 4) == 0) strip_rowpass<G, P>(lds, taps, prow, pq);
    for (int k = 0; k < nsteps; k++) {
        float* sa = lds + (k & 1) * G::SLOT;
        float* sb = lds + ((k + 1) & 1) * G::SLOT;
        __syncthreads();  // column pass k - 1 is done with slot b
        ld.store(sb, gb + (k + 1) * G::S);
        if (k + 2 <= nsteps) ld.prefetch(gb + (k + 2) * G::S);
        __syncthreads();
        if constexpr ((ABL & 4) == 0) strip_rowpass<G, P>(sb, taps, prow, pq);
        __syncthreads();
        const int y = ys + k * G::S;
        switch (wv) {
#define COLPASS(w)                                                                                    \
    case w:                                                                                           \
        strip_colpass<G, P, w, false>(sa, sb, taps, lane, y, ye, x0, W, pitch, rd, rd, 0, 0, 0);     \
        break;
            COLPASS(0) COLPASS(1) COLPASS(2) COLPASS(3)
            default:
                __builtin_unreachable();  // wv < 4: no store-free path (static vmcnt)
#undef COLPASS
        }
    }
}

// ---------------------------------------------------------------------------
// Seed, Imageproc profile: u8 -> f32 (v / 255) -> image::imageops::resize
// Triangle 2x (vertical_sample into an f32 intermediate, then
// horizontal_sample; t = t + p * w from the first tap, result clamped to
// [0, 1]) -> imageproc gaussian_blur_f32 (clamp-to-edge), fused like k_seed.
// ---------------------------------------------------------------------------
template <int R, int TH>
__global__ __launch_bounds__(256) void k_seed_ip(const uint8_t* __restrict__ frames, size_t frame_pitch,
                                                 size_t row_stride, int sh, int sw, const IpResizeTab tab,
                                                 float* __restrict__ dst, size_t dst_img_stride, int W, int H,
                                                 int pitch, const BlurTaps taps) {
    using G = BlurGeom<R, TH>;
    constexpr int SR = G::IH / 2 + kIpTaps + 2, SC = G::IWV / 2 + kIpTaps + 2;
    static_assert(G::IH <= 128 && G::IWV <= 128, "span reduction covers 128 positions per axis");
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    __shared__ float srcf[SR * SC];     // u8 -> f32 source window
    __shared__ float vbuf[G::IH * SC];  // vertical_sample rows of the window
    __shared__ int span[4][2];
    __shared__ int txl[G::IWV], tyl[G::IH];
    __shared__ float txw[G::IWV][kIpTaps], tyw[G::IH][kIpTaps];
    float* tin = lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const TileId tile = xcd_tile();
    const int x0 = tile.x * G::TW, y0 = tile.y * G::TH;
    const size_t b = tile.z;
    const uint8_t* src = frames + b * frame_pitch;
    {
        // window column (threads 0..127) / row (128..255): clamp-to-edge
        // position, its sampling taps, and the source span they cover
        const int t = tid & 127;
        const bool isx = tid < 128;
        const bool act = isx ? t < G::IWV : t < G::IH;
        const int g = act ? (isx ? clamp_idx(x0 - G::HWL + t, W) : clamp_idx(y0 - R + t, H)) : 0;
        int s0 = 0, s1 = 0;
        if (act) {
            const int* lp = isx ? tab.xl : tab.yl;
            const float* wp = isx ? tab.xw : tab.yw;
            s0 = lp[g];
            s1 = min(s0 + kIpTaps - 1, (isx ? sw : sh) - 1);
#pragma unroll
            for (int k = 0; k < kIpTaps; k++) {
                if (isx)
                    txw[t][k] = wp[g * kIpTaps + k];
                else
                    tyw[t][k] = wp[g * kIpTaps + k];
            }
            if (isx)
                txl[t] = s0;
            else
                tyl[t] = s0;
        }
        int mn = act ? s0 : INT_MAX, mx = act ? s1 : INT_MIN;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            mn = min(mn, __shfl_xor(mn, o));
            mx = max(mx, __shfl_xor(mx, o));
        }
        if (lane == 0) {
            span[wv][0] = mn;
            span[wv][1] = mx;
        }
    }
    __syncthreads();
    const int sxa = min(span[0][0], span[1][0]), sxb = max(span[0][1], span[1][1]);
    const int sya = min(span[2][0], span[3][0]), syb = max(span[2][1], span[3][1]);
    const int nc = sxb - sxa + 1, nr = syb - sya + 1;
    if (nc <= SC && nr <= SR) {
        for (int r = wv; r < nr; r += 4)
            for (int c = lane; c < nc; c += 64) srcf[r * SC + c] = u8_unit(src[(size_t)(sya + r) * row_stride + sxa + c]);
        __syncthreads();
        // vertical_sample: window row ly over the source columns
        for (int i = tid; i < G::IH * nc; i += 256) {
            const int ly = i / nc, c = i - ly * nc;
            const int l = tyl[ly] - sya;
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < kIpTaps; k++) acc = acc + srcf[min(l + k, nr - 1) * SC + c] * tyw[ly][k];
            vbuf[ly * SC + c] = acc;
        }
        __syncthreads();
        // horizontal_sample, clamped to [0, 1]
        for (int i = tid; i < G::IH * G::IWV; i += 256) {
            const int ly = i / G::IWV, lx = i - ly * G::IWV;
            const int l = txl[lx] - sxa;
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < kIpTaps; k++) acc = acc + vbuf[ly * SC + min(l + k, nc - 1)] * txw[lx][k];
            tin[ly * G::IWP + lx] = fminf(fmaxf(acc, 0.0f), 1.0f);
        }
    } else {  // degenerate shapes: direct gathers
        for (int i = tid; i < G::IH * G::IWV; i += 256) {
            const int ly = i / G::IWV, lx = i - ly * G::IWV;
            float acc = 0.0f;
#pragma unroll
            for (int kx = 0; kx < kIpTaps; kx++) {
                const int cx = min(txl[lx] + kx, sw - 1);
                float v = 0.0f;
#pragma unroll
                for (int ky = 0; ky < kIpTaps; ky++)
                    v = v + u8_unit(src[(size_t)min(tyl[ly] + ky, sh - 1) * row_stride + cx]) * tyw[ly][ky];
                acc = acc + v * txw[lx][kx];
            }
            tin[ly * G::IWP + lx] = fminf(fmaxf(acc, 0.0f), 1.0f);
        }
    }
    __syncthreads();
    blur_tile_compute<R, TH, kProfileImageproc>(tin, lds, taps, x0, y0, W, H, pitch, dst + b * dst_img_stride, nullptr,
                                                nullptr, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int R>
static void launch_blur_r(const BlurLaunch& L, hipStream_t st) {
    constexpr int TH = R >= 10 ? 64 : 32;  // measured: tools/ubench_kernels.hip blur
    using G = BlurGeom<R, TH>;
    const int tiles_y = (L.H + G::TH - 1) / G::TH;
    // optional row range (row bands): tile rows covering [L.y0, L.y1)
    const int ty0 = L.y1 > L.y0 ? L.y0 / G::TH : 0;
    const int ty1 = L.y1 > L.y0 ? std::min(tiles_y, (L.y1 + G::TH - 1) / G::TH) : tiles_y;
    if (ty1 <= ty0) return;
    dim3 grid((L.W + G::TW - 1) / G::TW, ty1 - ty0, L.n_img);
    if (L.profile == kProfileImageproc)
        klaunch((k_blur<R, TH, kProfileImageproc>), grid, dim3(256), st, L.src, L.src_img_stride, L.dst,
                           L.dst_img_stride, L.dog, L.dog_img_stride, L.nxt, L.nxt_img_stride, L.pitch_n, L.wn, L.hn,
                           L.W, L.H, L.pitch, L.taps, ty0);
    else
        klaunch((k_blur<R, TH, kProfileOpenCV>), grid, dim3(256), st, L.src, L.src_img_stride, L.dst,
                           L.dst_img_stride, L.dog, L.dog_img_stride, L.nxt, L.nxt_img_stride, L.pitch_n, L.wn, L.hn,
                           L.W, L.H, L.pitch, L.taps, ty0);
}

template <int R, int P>
static void launch_blur_strip_rp(const BlurLaunch& L, dim3 grid, int ya, int yb, int seg, hipStream_t st) {
    using G = StripGeom<R>;
    if (L.nxt)
        klaunch((k_blur_strip<R, P, true>), grid, dim3(64 * G::NW), st, L.src, L.src_img_stride, L.dst,
                           L.dst_img_stride, L.nxt, L.nxt_img_stride, L.pitch_n, L.wn, L.hn, L.W, L.H, L.pitch,
                           L.taps, ya, yb, seg);
    else
        klaunch((k_blur_strip<R, P, false>), grid, dim3(64 * G::NW), st, L.src, L.src_img_stride,
                           L.dst, L.dst_img_stride, L.nxt, L.nxt_img_stride, L.pitch_n, L.wn, L.hn, L.W, L.H,
                           L.pitch, L.taps, ya, yb, seg);
}

// Row segments of a strip launch over `rows` rows with `per` strips x frames:
// ~strip_wg_target() workgroups, but no segment shorter than ~320 rows unless
// the launch would then have fewer than ~2048 workgroups (then down to ~40
// rows) -- a segment re-filters its halo rows and fills / drains its chunk
// pipeline, so short segments cost more than the extra parallelism buys
// (measured, tools/ubench_kernels.hip segs: octave 1 of 64 1080p frames,
// R = 13, 319 us at 13 segments of 84 rows vs 254 us at 3 of 360), while the
// small octaves need the segments to fill the chip.  Returns the segment length.
static int strip_segment_rows(int rows, long per, long target = 6144) {
    const long few = std::min<long>((2048 + per - 1) / per, rows / 40);
    long nseg = std::min<long>((target + per - 1) / per, std::max<long>(rows / 320, few));
    nseg = std::max(1L, nseg);
    // even: with an even first row every segment starts at an even row (the
    // strip kernels' next-octave rows are then the even / odd rows of each
    // column pass statically; the seed's row pairs share source rows)
    return (int)(((rows + nseg - 1) / nseg + 1) & ~1);
}

template <int R>
static void launch_blur_strip_r(const BlurLaunch& L, hipStream_t st) {
    using G = StripGeom<R>;
    // an even first row (one extra row above a band is exact): see strip_segment_rows
    const int ya = L.y1 > L.y0 ? std::max(L.y0, 0) & ~1 : 0;
    const int yb = L.y1 > L.y0 ? std::min(L.y1, L.H) : L.H;
    if (yb <= ya) return;
    const int strips = (L.W + G::TW - 1) / G::TW;
    // segments: ~6 k workgroups per launch (a few dozen per CU: the last
    // round of equal-sized workgroups is a small fraction; round 3: 6 k beat
    // 12 k by 1-2% of pyramid time, octave 0 of 1080p in 4 segments instead
    // of 7; 3 k, 4 k, 8 k within noise of 6 k), none shorter than two chunks
    // (each segment re-filters its 2R halo rows)
    const int rows = yb - ya;
    const int seg = strip_segment_rows(rows, (long)strips * L.n_img);
    const int nseg = (rows + seg - 1) / seg;
    const dim3 grid(strips, nseg, L.n_img);
    if (L.profile == kProfileImageproc)
        launch_blur_strip_rp<R, kProfileImageproc>(L, grid, ya, yb, seg, st);
    else
        launch_blur_strip_rp<R, kProfileOpenCV>(L, grid, ya, yb, seg, st);
}

template <int Ra, int Rb, int P = kProfileOpenCV>
static void launch_blur2_rr(const BlurLaunch& A, const BlurLaunch& B, hipStream_t st) {
    using Q = PairGeom<Ra, Rb>;
    const int strips = (A.W + Q::TWO - 1) / Q::TWO;
    // the octave-0 (2, 3) pair (B.nxt) at ~8 k workgroups: measured against
    // 3 k / 4 k / 6 k / 12 k on 64 1080p frames (tools/head_ab.sh)
    const int seg = strip_segment_rows(A.H, (long)strips * A.n_img, B.nxt ? 8192 : 6144);
    const int nseg = (A.H + seg - 1) / seg;
    const dim3 grid(strips, nseg, A.n_img);
    if (B.nxt) {  // blurs 2, 3 of octave 0: B writes the next octave's base
        klaunch((k_blur2_strip<Ra, Rb, false, P, true>), grid, dim3(256), st, A.src, A.src_img_stride,
                           A.dst, B.dst, B.nxt, B.nxt_img_stride, B.pitch_n, B.wn, B.hn, A.W, A.H, A.pitch, A.taps,
                           B.taps, 0, A.H, seg);
    } else if constexpr (P == kProfileImageproc) {
        klaunch((k_blur2_strip<Ra, Rb, false, P>), grid, dim3(256), st, A.src, A.src_img_stride, A.dst,
                           B.dst, A.nxt, A.nxt_img_stride, A.pitch_n, A.wn, A.hn, A.W, A.H, A.pitch, A.taps, B.taps,
                           0, A.H, seg);
    } else if (A.nxt) {
        klaunch((k_blur2_strip<Ra, Rb, true>), grid, dim3(256), st, A.src, A.src_img_stride, A.dst,
                           B.dst, A.nxt, A.nxt_img_stride, A.pitch_n, A.wn, A.hn, A.W, A.H, A.pitch, A.taps, B.taps,
                           0, A.H, seg);
    } else {
        klaunch((k_blur2_strip<Ra, Rb, false>), grid, dim3(256), st, A.src, A.src_img_stride, A.dst,
                           B.dst, A.nxt, A.nxt_img_stride, A.pitch_n, A.wn, A.hn, A.W, A.H, A.pitch, A.taps, B.taps,
                           0, A.H, seg);
    }
}

int launch_blur_pair(int ra, int rb, const BlurLaunch& A, const BlurLaunch& B, hipStream_t st, const PathOpts& o) {
    // A: G_{s-1} -> G_s, B: G_s -> G_{s+1} of one octave arena (same geometry
    // and image stride); whole planes, no DoG; at most one of them writes the
    // next octave's base (B: blurs 2, 3 of octave 0 after k_seed_pair)
    const bool ok = A.profile == B.profile && !A.dog && !B.dog && !(A.nxt && B.nxt) && A.y1 <= A.y0 &&
                    B.y1 <= B.y0 && A.dst && B.dst && B.src == A.dst && A.W == B.W && A.H == B.H &&
                    A.pitch == B.pitch && A.src_img_stride == A.dst_img_stride &&
                    B.src_img_stride == A.src_img_stride && B.dst_img_stride == A.src_img_stride && A.W >= 64 &&
                    A.H >= 64 && (uint64_t)A.H * (uint64_t)A.pitch * 4 < (1ull << 31) && !o.tile_blur && o.pair;
    if (!ok) return -1;
    // (5, 6): blurs 1, 2; (6, 8) with B.nxt: blurs 2, 3 of octave 0 (G_1 from
    // k_seed_pair).  A (8, 10) pair for blurs 3, 4 (three-chunk column
    // windows at 16-row chunks) was built, exact and slower than the two
    // single launches (1.75 vs 1.62 ms per 64 frames of 3840x2160, round 2;
    // DESIGN.md 3.10), and was removed.
    if (A.profile == kProfileImageproc) {
        // imageproc's clamp-to-edge chain: rows outside the image are read
        // clamped (strip_colpass_clamped); blurs 1, 2 are radii 3, 4; blurs
        // 2, 3 radii 4, 4
        if (ra == 3 && rb == 4 && !A.nxt && !B.nxt) { launch_blur2_rr<3, 4, kProfileImageproc>(A, B, st); return 0; }
        if (ra == 4 && rb == 4 && !A.nxt && B.nxt) { launch_blur2_rr<4, 4, kProfileImageproc>(A, B, st); return 0; }
        return -1;
    }
    if (ra == 5 && rb == 6 && !B.nxt) { launch_blur2_rr<5, 6>(A, B, st); return 0; }
    if (ra == 6 && rb == 8 && !A.nxt && B.nxt) { launch_blur2_rr<6, 8>(A, B, st); return 0; }
    return -1;
}

int launch_blur(int R, const BlurLaunch& L, hipStream_t st, const PathOpts& o) {
    // the strip kernel: materialised G_s, no DoG plane (the batch path), one
    // reflection per border (W, H > R), planes addressable by 32-bit offsets
    if (L.dst && !L.dog && R <= kStripMaxR && L.W > R && L.H > R &&
        (uint64_t)L.H * (uint64_t)L.pitch * 4 < (1ull << 31) && !o.tile_blur) {
        switch (R) {
#define CASE(r) \
    case r:     \
        launch_blur_strip_r<r>(L, st); return 0;
            CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10) CASE(11) CASE(12)
            CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
            default:
                break;
        }
    }
    switch (R) {
#define CASE(r) \
    case r:     \
        launch_blur_r<r>(L, st); return 0;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10) CASE(11) CASE(12)
        CASE(13) CASE(14) CASE(15) CASE(16) CASE(17) CASE(18) CASE(19) CASE(20) CASE(21) CASE(22) CASE(23) CASE(24)
#undef CASE
        default:
            return -1;
    }
}

template <int R>
static void launch_seed_r(const SeedLaunch& L, hipStream_t st) {
#ifndef SIFT_SEED_TH
#define SIFT_SEED_TH 32
#endif
    constexpr int TH = SIFT_SEED_TH;
    using G = BlurGeom<R, TH>;
    const int tiles_y = (L.H + G::TH - 1) / G::TH;
    const int ty0 = L.y1 > L.y0 ? L.y0 / G::TH : 0;
    const int ty1 = L.y1 > L.y0 ? std::min(tiles_y, (L.y1 + G::TH - 1) / G::TH) : tiles_y;
    if (ty1 <= ty0) return;
    dim3 grid((L.W + G::TW - 1) / G::TW, ty1 - ty0, L.n_img);
    klaunch((k_seed<R, TH>), grid, dim3(256), st, L.frames, L.frame_pitch, L.row_stride, L.sh, L.sw, L.tab,
                       L.dst, L.dst_img_stride, L.W, L.H, L.pitch, L.taps, ty0);
}

template <int R>
static void launch_seed_ip_r(const SeedLaunch& L, hipStream_t st) {
    constexpr int TH = 32;
    using G = BlurGeom<R, TH>;
    dim3 grid((L.W + G::TW - 1) / G::TW, (L.H + G::TH - 1) / G::TH, L.n_img);
    klaunch((k_seed_ip<R, TH>), grid, dim3(256), st, L.frames, L.frame_pitch, L.row_stride, L.sh, L.sw,
                       L.iptab, L.dst, L.dst_img_stride, L.W, L.H, L.pitch, L.taps);
}

int launch_seed(int R, const SeedLaunch& L, hipStream_t st, const PathOpts& o) {
    // the seed sigma is a constant: OpenCV cvRound(1.249 * 8 + 1) | 1 = 11
    // taps (R = 5); imageproc ceil(2 * 1.249) = 3
    const bool ip = L.profile == kProfileImageproc;
    if (R != (ip ? 3 : 5)) return -1;
    // the strip seed: exact 2x geometry, frames wide / tall enough for one
    // reflection of every window (else the tile kernels)
    if (L.W == 2 * L.sw && L.H == 2 * L.sh && L.W >= 160 && L.H >= 64 &&
        (uint64_t)L.H * (uint64_t)L.pitch * 4 < (1ull << 31) && !o.tile_blur) {
        using G = StripGeom<5>;
        // segments start at even rows: the loader's row pairs then share their
        // two source rows (k_seed_strip); an extra row above a band is exact
        const int ya = L.y1 > L.y0 ? std::max(L.y0, 0) & ~1 : 0;
        const int yb = L.y1 > L.y0 ? std::min(L.y1, L.H) : L.H;
        if (yb <= ya) return 0;
        const int strips = (L.W + G::TW - 1) / G::TW;
        const int rows = yb - ya;
        const int seg = strip_segment_rows(rows, (long)strips * L.n_img);
        const int nseg = (rows + seg - 1) / seg;
        const dim3 grid(strips, nseg, L.n_img);
        if (ip)
            klaunch((k_seed_strip<3, kProfileImageproc>), grid, dim3(256), st, L.frames, L.frame_pitch,
                               L.row_stride, L.sh, L.sw, L.dst, L.dst_img_stride, L.W, L.H, L.pitch, L.taps, ya, yb,
                               seg);
        else
            klaunch((k_seed_strip<5, kProfileOpenCV>), grid, dim3(256), st, L.frames, L.frame_pitch,
                               L.row_stride, L.sh, L.sw, L.dst, L.dst_img_stride, L.W, L.H, L.pitch, L.taps, ya, yb,
                               seg);
        return 0;
    }
    if (ip)
        launch_seed_ip_r<3>(L, st);
    else
        launch_seed_r<5>(L, st);
    return 0;
}

template <int Ra, int Rb, int P>
static void launch_seed_pair_rr(const SeedLaunch& S, const BlurLaunch& B, hipStream_t st) {
    using Q = PairGeom<Ra, Rb, 8>;
    const int strips = (S.W + Q::TWO - 1) / Q::TWO;
    const int seg = strip_segment_rows(S.H, (long)strips * S.n_img, 8192);  // as the (2, 3) pair
    const int nseg = (S.H + seg - 1) / seg;
    klaunch((k_seed_pair<Ra, Rb, P>), dim3(strips, nseg, S.n_img), dim3(256), st, S.frames,
                       S.frame_pitch, S.row_stride, S.sh, S.sw, S.dst, B.dst, S.dst_img_stride, S.W, S.H, S.pitch,
                       S.taps, B.taps, 0, S.H, seg, S.init_cnt, S.init_m, S.init_words);
}

int launch_seed_pair(int rs, int rb, const SeedLaunch& S, const BlurLaunch& B, hipStream_t st, const PathOpts& o) {
    // the strip seed's geometry (exact 2x, one reflection per window) and the
    // pair's (whole planes, B = blur 1 of the seed's plane, same arena)
    const bool ok = S.W == 2 * S.sw && S.H == 2 * S.sh && S.W >= 160 && S.H >= 64 &&
                    (uint64_t)S.H * (uint64_t)S.pitch * 4 < (1ull << 31) && S.y1 <= S.y0 && B.y1 <= B.y0 &&
                    B.profile == S.profile && B.src == S.dst && B.dst && !B.dog && !B.nxt && B.W == S.W &&
                    B.H == S.H && B.pitch == S.pitch && B.src_img_stride == S.dst_img_stride &&
                    B.dst_img_stride == S.dst_img_stride && !o.tile_blur && o.pair && o.seed_pair;
    if (!ok) return -1;
    if (S.profile == kProfileImageproc) {
        if (rs == 3 && rb == 3) { launch_seed_pair_rr<3, 3, kProfileImageproc>(S, B, st); return 0; }
        return -1;
    }
    if (rs == 5 && rb == 5) { launch_seed_pair_rr<5, 5, kProfileOpenCV>(S, B, st); return 0; }
    return -1;
}

// ---------------------------------------------------------------------------
// k_octave_tail: every small octave of a frame in ONE launch.  From octave o0
// on (the first octave whose planes fit the LDS layout below) a workgroup
// owns one frame: it reads G_0 of octave o0 into LDS, runs the five
// incremental blurs of the octave LDS to LDS, stores every G_s, forms the
// next octave's G_0 (nearest 1/2 of G_3) in LDS while G_3 is written, and
// carries on to the last octave.  The arithmetic is exactly k_blur's (OpenCV:
// fma chain from the leftmost tap, then centre product + fma of the (below +
// above) pair sums; imageproc: unfused chains from the first tap).  This
// replaces 5 launches per tail octave (a few tiles per frame each, bound by
// launch and pipeline-fill latency) with one.
//
// A tail octave is a few thousand pixels per workgroup, so the passes are
// bound by LDS latency along each output's tap chain: the borders are
// materialised instead of evaluated per tap (reflect-101 / clamp-to-edge halo
// columns of the blur input, halo rows of the row-pass output, filled by a
// pass of their own where a halo row / column mirrors more than one image
// row / column, else by the passes that compute the mirrored values), so every
// tap read is a plain offset, and each thread
// carries four independent chains (four outputs of a row / of a column).
// LDS layout (floats), with Rm the largest radius of the octave's blurs:
//   A, B  G_{s-1} / G_s:     H rows of pitch PA = (W + 2 Rm) | 1 (column halos), x at + Rm
//   T     row-pass output:   H + 2 Rm rows of pitch TP = W | 1 (row halos), y at + Rm
//   N     next octave G_0:   (H / 2) x (W / 2), dense
// Odd pitches: the row pass maps consecutive lanes to consecutive rows (same
// columns), so its reads of A and writes of T hit distinct banks; the column
// pass maps lanes along a row.
// ---------------------------------------------------------------------------
// Phase timestamps of workgroup 0's thread 0 (s_memrealtime / s_memtime)
// for tools/ubench_kernels built with -DSIFT_TAIL_PROF (tools/ubench_tailprof);
// the product build does not define it and the marks compile to nothing
#ifdef SIFT_TAIL_PROF
__device__ unsigned long long g_tail_prof[2048];
__shared__ int tail_prof_n;
#define TAIL_MARK(tag)                                                                                  \
    do {                                                                                                \
        if (threadIdx.x == 0 && blockIdx.x == 0 && tail_prof_n < 1024) {                                \
            g_tail_prof[2 * tail_prof_n] = wall_clock64();                                              \
            g_tail_prof[2 * tail_prof_n + 1] = (unsigned long long)(tag) | ((unsigned long long)clock64() << 8); \
            tail_prof_n++;                                                                              \
        }                                                                                               \
    } while (0)
#else
#define TAIL_MARK(tag) \
    do {               \
    } while (0)
#endif
template <int P>
__device__ __forceinline__ int tail_index(int p, int n) {
    return P == kProfileOpenCV ? reflect101(p, n) : clamp_idx(p, n);
}

__host__ __device__ inline int tail_pa(int W, int rm) { return (W + 2 * rm) | 1; }
__host__ __device__ inline int tail_tp(int W) { return W | 1; }
__host__ __device__ inline int tail_lds_floats(int W, int H, int rm) {
    return 2 * tail_pa(W, rm) * H + tail_tp(W) * (H + 2 * rm) + (W / 2) * (H / 2);
}

// halo columns [-R, 0) and [W, W + R) of every row of X (pitch W + 2 Rm)
template <int P>
__device__ __forceinline__ void tail_fill_cols(float* X, int W, int H, int Rm, int R) {
    const int PA = tail_pa(W, Rm);
    for (int i = threadIdx.x; i < H * 2 * R; i += 1024) {
        const int y = i / (2 * R), j = i - y * (2 * R);
        const int p = j < R ? j - R : W + j - R;
        float* row = X + y * PA + Rm;
        row[p] = row[tail_index<P>(p, W)];
    }
}

// One blur of a tail octave (radius R a compile-time constant: every output's
// window is read from LDS once into registers and the tap chain runs on
// registers; the taps come from the kernel argument, i.e. scalar registers).
template <int P, int R>
__device__ __forceinline__ void tail_blur_r(float* __restrict__ A, float* __restrict__ T, float* __restrict__ B,
                                            const BlurTaps& taps, int Rn, int Rm, int W, int H,
                                            float* __restrict__ g, int pitch, bool nxt, float* __restrict__ N,
                                            float* __restrict__ gn, int wn, int hn, int pn) {
    constexpr int Q = 4;
    const int PA = tail_pa(W, Rm), TP = tail_tp(W);
    // halos written by the passes themselves where one mirror image suffices
    const bool rows_direct = P != kProfileOpenCV || H > R;
    const bool cols_direct = Rn > 0 && (P != kProfileOpenCV || W > Rn);
    // row pass (A's halo columns are in place): fma chain from the leftmost
    // tap (OpenCV) / unfused chain (imageproc); item = (row, 4 columns),
    // consecutive items down a column of items (lanes on distinct banks).
    // The last item of a row may read past its halo (into the next row /
    // buffer: still LDS) for columns >= W, which are not stored.
    const int qw = (W + Q - 1) / Q;
    for (int i = threadIdx.x; i < H * qw; i += 1024) {
        const int xq = i / H, y = i - xq * H, x0 = xq * Q;
        const float* p = A + y * PA + Rm + x0 - R;
        float v[Q + 2 * R];
#pragma unroll
        for (int j = 0; j < Q + 2 * R; j++) v[j] = p[j];
        float acc[Q];
#pragma unroll
        for (int q = 0; q < Q; q++) acc[q] = v[q] * taps.k[R];
#pragma unroll
        for (int t = 1; t <= 2 * R; t++) {
            const float kt = taps.k[t > R ? t - R : R - t];
#pragma unroll
            for (int q = 0; q < Q; q++)
                acc[q] = P == kProfileOpenCV ? __builtin_fmaf(v[q + t], kt, acc[q]) : acc[q] + v[q + t] * kt;
        }
        float* o = T + (y + Rm) * TP + x0;
#pragma unroll
        for (int q = 0; q < Q; q++)
            if (x0 + q < W) o[q] = acc[q];
        // T's halo rows [-R, 0) and [H, H + R) that mirror row y, written
        // here instead of by a pass of their own (one barrier less): one
        // reflection (OpenCV, H > R) / the edge rows (imageproc)
        if (rows_direct) {
            auto mirror = [&](int p) {
                float* h = T + (p + Rm) * TP + x0;
#pragma unroll
                for (int q = 0; q < Q; q++)
                    if (x0 + q < W) h[q] = acc[q];
            };
            if constexpr (P == kProfileOpenCV) {
                if (y >= 1 && y <= R) mirror(-y);
                if (y >= H - 1 - R && y <= H - 2) mirror(2 * H - 2 - y);
            } else {
                if (y == 0)
                    for (int p = -R; p < 0; p++) mirror(p);
                if (y == H - 1)
                    for (int p = H; p < H + R; p++) mirror(p);
            }
        }
    }
    __syncthreads();
    TAIL_MARK(1);
    if (!rows_direct) {  // T's halo rows [-R, 0) and [H, H + R)
        for (int i = threadIdx.x; i < 2 * R * W; i += 1024) {
            const int j = i / W, x = i - j * W;
            const int p = j < R ? j - R : H + j - R;
            T[(p + Rm) * TP + x] = T[(tail_index<P>(p, H) + Rm) * TP + x];
        }
        __syncthreads();
        TAIL_MARK(2);
    }
    // column pass: centre product + fma of the (below + above) pair sums
    // (OpenCV) / the unfused chain from the first tap (imageproc); item =
    // (column, 4 consecutive rows), lanes along the row (coalesced stores)
    const int qh = (H + Q - 1) / Q;
    constexpr int par = P == kProfileOpenCV ? 0 : 1;  // nearest 1/2: (2x, 2y) / (2x + 1, 2y + 1)
    for (int i = threadIdx.x; i < W * qh; i += 1024) {
        const int yq = i / W, x = i - yq * W, y0 = yq * Q;
        const float* p = T + (y0 - R + Rm) * TP + x;  // window row 0 = image row y0 - R
        float v[Q + 2 * R];
#pragma unroll
        for (int j = 0; j < Q + 2 * R; j++) v[j] = p[j * TP];
        float acc[Q];
        if constexpr (P == kProfileOpenCV) {
#pragma unroll
            for (int q = 0; q < Q; q++) acc[q] = v[q + R] * taps.k[0];
#pragma unroll
            for (int t = 1; t <= R; t++) {
                const float kt = taps.k[t];
#pragma unroll
                for (int q = 0; q < Q; q++) acc[q] = __builtin_fmaf(v[q + R + t] + v[q + R - t], kt, acc[q]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < Q; q++) acc[q] = v[q] * taps.k[R];
#pragma unroll
            for (int t = 1; t <= 2 * R; t++) {
                const float kt = taps.k[t > R ? t - R : R - t];
#pragma unroll
                for (int q = 0; q < Q; q++) acc[q] = acc[q] + v[q + t] * kt;
            }
        }
#pragma unroll
        for (int q = 0; q < Q; q++) {
            const int y = y0 + q;
            if (y >= H) break;
            float* brow = B + y * PA + Rm;
            brow[x] = acc[q];
            // B's halo columns for the next blur (radius Rn) that mirror
            // column x (one reflection: OpenCV, W > Rn / imageproc's edges)
            if (cols_direct) {
                if constexpr (P == kProfileOpenCV) {
                    if (x >= 1 && x <= Rn) brow[-x] = acc[q];
                    if (x >= W - 1 - Rn && x <= W - 2) brow[2 * W - 2 - x] = acc[q];
                } else {
                    if (x == 0)
                        for (int p = -Rn; p < 0; p++) brow[p] = acc[q];
                    if (x == W - 1)
                        for (int p = W; p < W + Rn; p++) brow[p] = acc[q];
                }
            }
            g[(size_t)y * pitch + x] = acc[q];
            if (nxt && (x & 1) == par && (y & 1) == par && (x >> 1) < wn && (y >> 1) < hn) {
                const float nv = P == kProfileOpenCV ? acc[q] : ip_unit_clamp(acc[q]);
                N[(y >> 1) * wn + (x >> 1)] = nv;
                gn[(size_t)(y >> 1) * pn + (x >> 1)] = nv;
            }
        }
    }
    __syncthreads();
    TAIL_MARK(3);
    if (Rn > 0 && !cols_direct) {  // B's halo columns for the next blur
        tail_fill_cols<P>(B, W, H, Rm, Rn);
        __syncthreads();
        TAIL_MARK(4);
    }
}

// radii of the two profiles' octave blurs (OpenCV 5, 6, 8, 10, 13; imageproc
// 3, 4, 4, 5, 7) get their own instantiations; others return false (the
// caller then runs the octave per blur: tail_octave_start checks this)
__host__ __device__ constexpr bool tail_radius_ok(int R) {
    return R == 3 || R == 4 || R == 5 || R == 6 || R == 7 || R == 8 || R == 10 || R == 13;
}

template <int P>
__device__ __forceinline__ void tail_blur(float* __restrict__ A, float* __restrict__ T, float* __restrict__ B,
                                          const BlurTaps& taps, int R, int Rn, int Rm, int W, int H,
                                          float* __restrict__ g, int pitch, bool nxt, float* __restrict__ N,
                                          float* __restrict__ gn, int wn, int hn, int pn) {
    switch (R) {
#define TB(r)                                                                                     \
    case r:                                                                                       \
        tail_blur_r<P, r>(A, T, B, taps, Rn, Rm, W, H, g, pitch, nxt, N, gn, wn, hn, pn); \
        break;
        TB(3) TB(4) TB(5) TB(6) TB(7) TB(8) TB(10) TB(13)
#undef TB
        default:
            break;
    }
}

template <int P>
__global__ __launch_bounds__(1024) void k_octave_tail(const TailLaunch L) {
    __shared__ float lds[kTailLdsFloats];
    const int tid = threadIdx.x;
    const int b = (int)blockIdx.x;
    int Rm = 0;
    for (int s = 1; s < kImagesPerOctave; s++) Rm = max(Rm, L.r[s]);
#ifdef SIFT_TAIL_PROF
    if (tid == 0) tail_prof_n = 0;
    TAIL_MARK(0);
#endif
    for (int o = L.o0; o < L.n_oct; o++) {
        TAIL_MARK(10 + o);
        const int W = L.ow[o], H = L.oh[o], pitch = L.pitch[o], PA = tail_pa(W, Rm);
        float* A = lds;                         // G_{s-1}
        float* B = A + PA * H;                  // G_s
        float* T = B + PA * H;                  // row-pass output
        float* N = T + tail_tp(W) * (H + 2 * Rm);  // next octave's G_0
        float* g = L.gauss[o] + (size_t)b * L.gstride[o];
        const size_t plane = (size_t)pitch * H;
        const bool has_next = o + 1 < L.n_oct;
        const int wn = has_next ? L.ow[o + 1] : 0, hn = has_next ? L.oh[o + 1] : 0;
        float* gn = has_next ? L.gauss[o + 1] + (size_t)b * L.gstride[o + 1] : nullptr;
        const int pn = has_next ? L.pitch[o + 1] : 0;
        // G_0: from HBM (first tail octave) or from the previous octave's N
        // (which overlaps this octave's A / B: copy through registers)
        if (o == L.o0) {
            for (int y = tid >> 6; y < H; y += 16)
                for (int x = tid & 63; x < W; x += 64) A[y * PA + Rm + x] = g[(size_t)y * pitch + x];
        } else {
            const int Wp = L.ow[o - 1], Hp = L.oh[o - 1];
            const float* Np = lds + 2 * tail_pa(Wp, Rm) * Hp + tail_tp(Wp) * (Hp + 2 * Rm);
            float v[4];  // W * H <= 4096 here (checked by tail_octave_start)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int i = tid + 1024 * k;
                v[k] = i < W * H ? Np[i] : 0.0f;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int i = tid + 1024 * k;
                if (i < W * H) {
                    const int y = i / W, x = i - y * W;
                    A[y * PA + Rm + x] = v[k];
                }
            }
        }
        __syncthreads();
        TAIL_MARK(5);
        tail_fill_cols<P>(A, W, H, Rm, L.r[1]);
        __syncthreads();
        TAIL_MARK(6);
#pragma unroll 1
        for (int s = 1; s < kImagesPerOctave; s++) {
            tail_blur<P>(A, T, B, L.taps[s], L.r[s], s + 1 < kImagesPerOctave ? L.r[s + 1] : 0, Rm, W, H,
                         g + s * plane, pitch, s == 3 && has_next, N, gn, wn, hn, pn);
            float* t = A;
            A = B;
            B = t;
        }
    }
    TAIL_MARK(99);
}

int tail_octave_start(const int* ow, const int* oh, int n_oct, const int* radii) {
    int rmax = 0;
    for (int s = 1; s < kImagesPerOctave; s++) {
        if (!tail_radius_ok(radii[s])) return n_oct;  // no instantiation: per-blur launches
        rmax = std::max(rmax, radii[s]);
    }
    for (int o = 0; o < n_oct; o++) {
        // the G_0 hand-over copies <= 4 values per thread: the octave after
        // the first tail octave must have at most 4096 pixels
        const bool next_ok = o + 1 >= n_oct || ow[o + 1] * oh[o + 1] <= 4096;
        // (+ slack: the last row / column items read up to 3 rows / columns past their halo)
        if (tail_lds_floats(ow[o], oh[o], rmax) + 4 * ow[o] + 64 <= kTailLdsFloats && next_ok) return o;
    }
    return n_oct;
}

void launch_octave_tail(const TailLaunch& L, hipStream_t st) {
    if (L.o0 >= L.n_oct || L.n_img <= 0) return;
    if (L.profile == kProfileImageproc)
        klaunch(k_octave_tail<kProfileImageproc>, dim3(L.n_img), dim3(1024), st, L);
    else
        klaunch(k_octave_tail<kProfileOpenCV>, dim3(L.n_img), dim3(1024), st, L);
}

// ---------------------------------------------------------------------------
// DoG planes of precompute_images (build_dog, src/lib.rs:271-279): D_s =
// G_{s+1} - G_s over whole pitched planes (4 floats per thread; the padding
// columns are never read back).
// ---------------------------------------------------------------------------
__global__ void k_dog(const float* __restrict__ gauss, size_t plane, size_t g_img_stride, float* __restrict__ dog,
                      size_t dog_img_stride, size_t n4) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const float* g = gauss + (size_t)blockIdx.z * g_img_stride + (size_t)blockIdx.y * plane;
    float* d = dog + (size_t)blockIdx.z * dog_img_stride + (size_t)blockIdx.y * plane;
    const float4 a = reinterpret_cast<const float4*>(g)[i];
    const float4 b = reinterpret_cast<const float4*>(g + plane)[i];
    reinterpret_cast<float4*>(d)[i] = make_float4(b.x - a.x, b.y - a.y, b.z - a.z, b.w - a.w);
}

void launch_dog(const float* gauss, size_t plane, size_t g_img_stride, float* dog, size_t dog_img_stride, int W, int H,
                int pitch, int n_img, hipStream_t st) {
    (void)W;
    const size_t n4 = (size_t)pitch * H / 4;  // pitch: a multiple of 64 floats
    klaunch(k_dog, dim3((unsigned)((n4 + 255) / 256), kDogPerOctave, n_img), dim3(256), st, gauss,
                       plane, g_img_stride, dog, dog_img_stride, n4);
}

// ---------------------------------------------------------------------------
// Processing-trait op kernels on a single f32 image (src/lib.rs:86-90):
// generic bilinear / nearest resize used by sift_mi_resize_* (op parity only).
// ---------------------------------------------------------------------------
__global__ void k_resize_linear_f32(const float* __restrict__ src, int sw, int sh, const ResizeTab tab,
                                    float* __restrict__ dst, int dw, int dh) {
    const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (dx >= dw || dy >= dh) return;
    const int sx = tab.xofs[dx];
    const bool two = dx < tab.xmax;
    const int sx1 = two ? sx + 1 : sx;
    const int sy0 = tab.yofs[dy];
    const int sy1 = sy0 + 1 < sh ? sy0 + 1 : sh - 1;
    const float* r0 = src + (size_t)sy0 * sw;
    const float* r1 = src + (size_t)sy1 * sw;
    const float h0 = two ? r0[sx] * tab.xa0[dx] + r0[sx1] * tab.xa1[dx] : r0[sx];
    const float h1 = two ? r1[sx] * tab.xa0[dx] + r1[sx1] * tab.xa1[dx] : r1[sx];
    dst[(size_t)dy * dw + dx] = h0 * tab.ya0[dy] + h1 * tab.ya1[dy];
}

__global__ void k_resize_nearest_f32(const float* __restrict__ src, int sw, const int* __restrict__ xofs,
                                     const int* __restrict__ yofs, float* __restrict__ dst, int dw, int dh) {
    const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (dx >= dw || dy >= dh) return;
    dst[(size_t)dy * dw + dx] = src[(size_t)yofs[dy] * sw + xofs[dx]];
}

void launch_resize_linear_f32(const float* src, int sw, int sh, const ResizeTab& tab, float* dst, int dw, int dh,
                              hipStream_t st) {
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, 1);
    klaunch(k_resize_linear_f32, grid, dim3(256), st, src, sw, sh, tab, dst, dw, dh);
}

void launch_resize_nearest_f32(const float* src, int sw, const int* xofs, const int* yofs, float* dst, int dw, int dh,
                               hipStream_t st) {
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, 1);
    klaunch(k_resize_nearest_f32, grid, dim3(256), st, src, sw, xofs, yofs, dst, dw, dh);
}

// image::imageops::resize (Imageproc profile): vertical_sample into tmp
// (sw x dh), then horizontal_sample with the final [0, 1] clamp.
__global__ void k_ip_vsample(const float* __restrict__ src, int sw, int sh, const int* __restrict__ yl,
                             const float* __restrict__ yw, int ytaps, float* __restrict__ tmp, int dh) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= sw || y >= dh) return;
    const int l = yl[y];
    float acc = 0.0f;
    // zero-padded taps (weight 0) may run past the image: clamp the index
    for (int k = 0; k < ytaps; k++) acc = acc + src[(size_t)min(l + k, sh - 1) * sw + x] * yw[y * ytaps + k];
    tmp[(size_t)y * sw + x] = acc;
}

__global__ void k_ip_hsample(const float* __restrict__ tmp, int sw, const int* __restrict__ xl,
                             const float* __restrict__ xw, int xtaps, float* __restrict__ dst, int dw, int dh) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= dw || y >= dh) return;
    const int l = xl[x];
    float acc = 0.0f;
    for (int k = 0; k < xtaps; k++) acc = acc + tmp[(size_t)y * sw + min(l + k, sw - 1)] * xw[x * xtaps + k];
    dst[(size_t)y * dw + x] = fminf(fmaxf(acc, 0.0f), 1.0f);
}

void launch_ip_resize_f32(const float* src, int sw, int sh, const int* xl, const float* xw, int xtaps, const int* yl,
                          const float* yw, int ytaps, float* tmp, float* dst, int dw, int dh, hipStream_t st) {
    klaunch(k_ip_vsample, dim3((sw + 63) / 64, (dh + 3) / 4, 1), dim3(256), st, src, sw, sh, yl, yw,
                       ytaps, tmp, dh);
    klaunch(k_ip_hsample, dim3((dw + 63) / 64, (dh + 3) / 4, 1), dim3(256), st, tmp, sw, xl, xw, xtaps,
                       dst, dw, dh);
}

}  // namespace siftmi
