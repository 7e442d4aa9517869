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

// On success n holds the neighbourhood of the converged point (scale, y, x),
// which extremum_contrast / extremum_is_on_edge read next.
__device__ __forceinline__ bool interpolate(const gfloat* g0, size_t P, int W, int H, int pitch, int& scale, int& x,
                                            int& y, float& os, float& ox, float& oy, Nbhd& n, uint32_t* band_flag,
                                            int vlo, int vhi) {
    for (int it = 0; it < kMaxInterpSteps; it++) {
        // row bands with a restricted pyramid (host.cpp run_pyramid): the
        // rows read here must be computed ones, else the host recomputes the
        // band on the whole-frame pyramid
        if (band_flag && (y - 1 < vlo || y + 1 >= vhi)) atomicOr(band_flag, 1u);
        load_nbhd(g0, P, pitch, scale, y, x, n);
        // AT(plane, dy, dx): plane 0 / 1 / 2 = prev / curr / next
#define AT(a, dy, dx) n.d[a][(dy) + 1][(dx) + 1]
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
#undef AT
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
        if (fabsf(s_) < 0.5f && fabsf(x_) < 0.5f && fabsf(y_) < 0.5f) {
            os = s_;
            ox = x_;
            oy = y_;
            return true;
        }
        // `x as isize + offset.round() as isize` (saturating), then bounds
        const int64_t LIM = (int64_t)1 << 40;
        const int64_t rx = sat_i64(roundf(x_)), ry = sat_i64(roundf(y_)), rs = sat_i64(roundf(s_));
        if (rx > LIM || rx < -LIM || ry > LIM || ry < -LIM || rs > LIM || rs < -LIM) return false;
        const int64_t nx = x + rx, ny = y + ry, ns = scale + rs;
        if (!(ns >= 1 && ns <= kScalesPerOctave) || nx < kImageBorder || nx >= W - kImageBorder ||
            ny < kImageBorder || ny >= H - kImageBorder)
            return false;
        x = (int)nx;
        y = (int)ny;
        scale = (int)ns;
    }
    return false;
}

// ---------------------------------------------------------------------------
// k_detect_rows: point_is_local_extremum (src/lib.rs:437-506) over all three
// scale triples of an octave, with no LDS staging.  A wave owns a strip of 64
// columns (62 outputs: lanes 1..62, the edge lanes are halo) and DR_SH rows;
// it walks down the strip, loading one row of the 5 DoG planes per step (one
// coalesced 256-B load per plane), forming the 3-wide row max / min with DPP
// wave shifts and keeping the last 3 rows in registers.  Every DoG byte is
// read ~1.1x, there are no barriers, and the loads of the next row are in
// flight while a row is tested.  (A 64x16-tile kernel staging the 5 planes
// in LDS ran 1.8x longer: latency-bound, 62% of wave cycles waiting.)
// Extrema are appended as packed emission keys for k_refine.
// ---------------------------------------------------------------------------
constexpr int DR_SH = 32;       // rows per strip
constexpr int DR_COLS = 62;     // output columns per wave
constexpr int DR_LCAP = 256;    // per-block LDS candidate list

__device__ __forceinline__ float dpp_from_left(float v) {  // lane i <- lane i - 1 (wave_shr:1)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane i <- lane i + 1 (wave_shl:1)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
}

// 73 VGPRs, 6 waves per SIMD; forcing 7 spills in the row loop (+30% time)
#ifndef SIFT_DETECT_WPE
#define SIFT_DETECT_WPE 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_DETECT_WPE))) void k_detect_rows(const DetectLaunch ML) {
    __shared__ uint64_t lcand[DR_LCAP];
    __shared__ uint32_t lcount, gbase;
    // this block's octave (block-uniform: a scan of <= 16 block offsets)
    int oi = 0;
    while (oi + 1 < ML.n_oct && blockIdx.x >= ML.block0[oi + 1]) oi++;
    const DetectOctave& L = ML.oct[oi];
    const int W = L.W, H = L.H, pitch = L.pitch;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nsx = (W + DR_COLS - 1) / DR_COLS, nsy = (L.y_hi - L.y_lo + DR_SH - 1) / DR_SH;
    const uint32_t g = (blockIdx.x - ML.block0[oi]) * 4 + wave;  // strip index: frame-major, then row band, then column
    const uint32_t per = (uint32_t)(nsx * nsy);
    const int b = (int)(g / per);
    const uint32_t rem = g - (uint32_t)b * per;
    const int sy = (int)(rem / nsx), sx = (int)(rem % nsx);
    if (tid == 0) lcount = 0;
    __syncthreads();
    if (b < ML.n_img) {
        const float* gb = L.gauss + (size_t)b * L.img_stride;
        const size_t P = (size_t)pitch * H;
        const int x = sx * DR_COLS - 1 + lane;  // this lane's column
        const int xc = min(max(x, 0), W - 1);
        const bool xout = lane >= 1 && lane <= DR_COLS && x >= kImageBorder && x < W - kImageBorder;
        const int y0 = L.y_lo + sy * DR_SH, y1 = min(y0 + DR_SH, L.y_hi);
        // rolling state per plane: row max / min of rows y - 1, y, y + 1
        float hmx[kDogPerOctave][3], hmn[kDogPerOctave][3];
        float lrx[kDogPerOctave], lrn[kDogPerOctave], ctr[kDogPerOctave];  // row y (middle planes used)
        float nv[kImagesPerOctave], nlx[kDogPerOctave], nln[kDogPerOctave];
        // one row of G_0..G_5; the loads of row y + 2 stay in flight as raw
        // Gaussians and become D values (to_dog) when the row is consumed
        auto load_row = [&](int yy, float (&g)[kImagesPerOctave]) {
            const gfloat* rp = as_global(gb) + (size_t)min(max(yy, 0), H - 1) * pitch + xc;
#pragma unroll
            for (int p = 0; p < kImagesPerOctave; p++) g[p] = rp[(size_t)p * P];
        };
        auto to_dog = [&](const float (&g)[kImagesPerOctave], float (&v)[kDogPerOctave]) {
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) v[p] = g[p + 1] - g[p];
        };
        auto row_stats = [&](const float (&v)[kDogPerOctave], float (&mx)[kDogPerOctave], float (&mn)[kDogPerOctave],
                             float (&lx)[kDogPerOctave], float (&ln)[kDogPerOctave]) {
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                const float l = dpp_from_left(v[p]), r = dpp_from_right(v[p]);
                lx[p] = fmaxf(l, r);
                ln[p] = fminf(l, r);
                mx[p] = fmaxf(lx[p], v[p]);
                mn[p] = fminf(ln[p], v[p]);
            }
        };
        float v[kDogPerOctave], m0[kDogPerOctave], n0[kDogPerOctave];
        // rows y0 - 1 and y0
        load_row(y0 - 1, nv);
        to_dog(nv, v);
        row_stats(v, m0, n0, nlx, nln);
#pragma unroll
        for (int p = 0; p < kDogPerOctave; p++) {
            hmx[p][0] = m0[p];
            hmn[p][0] = n0[p];
        }
        load_row(y0, nv);
        to_dog(nv, v);
        row_stats(v, m0, n0, lrx, lrn);
#pragma unroll
        for (int p = 0; p < kDogPerOctave; p++) {
            hmx[p][1] = m0[p];
            hmn[p][1] = n0[p];
            ctr[p] = v[p];
        }
        const float threshold = floorf(0.5f * kContrastThreshold / (float)kScalesPerOctave);
        // Two rows in flight (rows y + 1 and y + 2 while row y is tested) in
        // two alternating buffers -- the loop is unrolled by two so neither
        // buffer is copied while its loads are outstanding.
        float nv2[kImagesPerOctave];
        load_row(y0 + 1, nv);
        load_row(y0 + 2, nv2);
        auto step = [&](int y, float (&buf)[kImagesPerOctave]) {
            // row y + 1 arrived in buf; row y + 3 goes in flight into it
            float cur[kDogPerOctave];
            to_dog(buf, cur);
            if (y + 2 < y1) load_row(y + 3, buf);
            row_stats(cur, m0, n0, nlx, nln);
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                hmx[p][2] = m0[p];
                hmn[p][2] = n0[p];
            }
            // point_is_local_extremum for row y, scales 1..3
            const bool yin = xout && y >= kImageBorder && y < H - kImageBorder;
            float pmx[kDogPerOctave], pmn[kDogPerOctave];
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                pmx[p] = fmaxf(fmaxf(hmx[p][0], hmx[p][1]), hmx[p][2]);
                pmn[p] = fminf(fminf(hmn[p][0], hmn[p][1]), hmn[p][2]);
            }
            uint32_t ok3 = 0;
#pragma unroll
            for (int s_in = 1; s_in <= kScalesPerOctave; s_in++) {
                const float val = ctr[s_in];
                const float m8 = fmaxf(fmaxf(hmx[s_in][0], hmx[s_in][2]), lrx[s_in]);
                const float n8 = fminf(fminf(hmn[s_in][0], hmn[s_in][2]), lrn[s_in]);
                const float mx = fmaxf(fmaxf(pmx[s_in - 1], pmx[s_in + 1]), m8);
                const float mn = fminf(fminf(pmn[s_in - 1], pmn[s_in + 1]), n8);
                const bool ok = yin && fabsf(val) > threshold && (val > 0.0f ? val >= mx : val <= mn);
                ok3 |= (uint32_t)ok << (s_in - 1);
            }
            if (__ballot(ok3 != 0)) {  // wave-uniform: rare
                while (ok3) {
                    const int bit = __builtin_ctz(ok3);
                    ok3 &= ok3 - 1;
                    const uint64_t key = make_key((uint32_t)(ML.img_base + b), (uint32_t)L.octave,
                                                  (uint32_t)(bit + 1), (uint32_t)y, (uint32_t)x);
                    const uint32_t li = atomicAdd(&lcount, 1u);
                    if (li < DR_LCAP) {
                        lcand[li] = key;
                    } else {
                        const uint32_t slot = atomicAdd(ML.counter, 1u);
                        if (slot < ML.cap) ML.cand[slot] = key;
                    }
                }
            }
            // shift rows: y + 1 becomes the centre row
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                hmx[p][0] = hmx[p][1];
                hmn[p][0] = hmn[p][1];
                hmx[p][1] = hmx[p][2];
                hmn[p][1] = hmn[p][2];
                lrx[p] = nlx[p];
                lrn[p] = nln[p];
                ctr[p] = cur[p];
            }
        };
        for (int y = y0; y < y1; y += 2) {
            step(y, nv);
            if (y + 1 < y1) step(y + 1, nv2);
        }
    }
    // one global atomic per block, then a coalesced copy of the block's list
    __syncthreads();
    const uint32_t nl = lcount < DR_LCAP ? lcount : DR_LCAP;
    if (nl == 0) return;
    if (tid == 0) gbase = atomicAdd(ML.counter, nl);
    __syncthreads();
    for (uint32_t i = tid; i < nl; i += 256)
        if (gbase + i < ML.cap) ML.cand[gbase + i] = lcand[i];
}

void launch_detect(DetectLaunch& L, hipStream_t st) {
    // drop empty octaves, then lay the octaves' blocks end to end
    int k = 0;
    for (int i = 0; i < L.n_oct; i++) {
        const DetectOctave& d = L.oct[i];
        if (d.y_lo < 0 || d.y_hi > d.H || d.y_hi <= d.y_lo) continue;
        L.oct[k++] = d;
    }
    L.n_oct = k;
    uint32_t nb = 0;
    for (int i = 0; i < k; i++) {
        const DetectOctave& d = L.oct[i];
        L.block0[i] = nb;
        const uint32_t strips =
            (uint32_t)((d.W + DR_COLS - 1) / DR_COLS) * ((d.y_hi - d.y_lo + DR_SH - 1) / DR_SH) * L.n_img;
        nb += (strips + 3) / 4;
    }
    L.block0[k] = nb;
    if (nb == 0) return;
    hipLaunchKernelGGL(k_detect_rows, dim3(nb), dim3(256), 0, st, L);
}

// ---------------------------------------------------------------------------
// k_blur_detect: the octave's last blur (G_4 -> G_5, radius R) and the
// extremum scan of its three scales (point_is_local_extremum,
// src/lib.rs:437-506) in one pass.  G_5 is produced on chip, so the scan
// reads G_0..G_4 (G_4 from the blur's own LDS rows) and never reads G_4 /
// G_5 back from HBM: ~26 B per octave pixel for blur 5 and detection
// together instead of ~35 (blur 5: 8 + halo, k_detect_rows: 24 + halo).
//
// A wave owns k_detect_rows' strip geometry: 64 columns x = xb - 1 + lane
// (62 outputs, the edge lanes are halo) by a segment of rows [ya, yb), and
// walks down it one row of G_4 at a time:
//   * the G_4 row's 64 + 2R columns [xb - 1 - R, xb + 63 + R) go to an LDS
//     ring (BD_RING rows per wave; loaded two rows ahead), and each lane's
//     row-filter output at its column is the FMA chain from the leftmost tap
//     of OpenCV's RowFilter (imageproc: the unfused chain) over 2R + 1 ring
//     values -- the same operations as the strip kernels (pyramid.hip);
//   * the last 2R + 1 row-filter outputs are a register window, whose column
//     filter (centre product + fma of the pair sums / imageproc's unfused
//     chain) is G_5 at row r = q - R: stored (rows [ya, yb), lanes 1..62);
//   * row r's D_0..D_4 are formed from G_0..G_3 (loaded two rows ahead),
//     G_4 (its ring row, still resident) and G_5, and the 3x3x3 test of row
//     r - 1 runs on the rolling row max / min exactly as k_detect_rows.
// Rows and columns outside the image are reflect-101 (clamp-to-edge) like the
// strip blur; only rows inside the image are stored or tested, so G_5 and the
// candidates are those of launch_blur + k_detect_rows bit for bit.
// ---------------------------------------------------------------------------
constexpr int BD_RING = 16;  // raw G_4 rows per wave (the rows r .. r + R and the next)
constexpr int BD_RP = 100;   // ring row pitch (floats): 64 + 2R columns, R <= 18

template <int P>
__device__ __forceinline__ int bd_index(int p, int n) {
    if (P == kProfileOpenCV) p = p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p);
    return p < 0 ? 0 : (p >= n ? n - 1 : p);
}

// 1-D block id remapped so each XCD walks a contiguous range (neighbouring
// strips of one row segment share their G_4 halo columns in that XCD's L2)
__device__ __forceinline__ uint32_t xcd_block_1d() {
    const uint32_t nwg = gridDim.x, orig = blockIdx.x;
    const uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <int R, int P>
__global__ __launch_bounds__(256) void k_blur_detect(const BlurDetectLaunch L) {
    static_assert(64 + 2 * R <= BD_RP && R + 3 <= BD_RING, "ring geometry");
    __shared__ float ring[4][BD_RING * BD_RP];
    __shared__ uint64_t lcand[DR_LCAP];
    __shared__ uint32_t lcount, gbase;
    // the wave index through readfirstlane: everything derived from it (the
    // strip, its rows, the buffer row offsets) is then known to be uniform
    // and lives in SGPRs -- a soffset the compiler cannot prove uniform turns
    // every buffer access into a readfirstlane waterfall loop
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W = L.W, H = L.H, pitch = L.pitch;
    const uint32_t g = xcd_block_1d() * 4 + wave;  // strip index: frame-major, then row segment, then column
    const uint32_t per = (uint32_t)(L.nsx * L.nsy);
    const int b = (int)(g / per);
    const uint32_t rem = g - (uint32_t)b * per;
    const int sy = (int)(rem / (uint32_t)L.nsx), sx = (int)(rem % (uint32_t)L.nsx);
    if (tid == 0) lcount = 0;
    __syncthreads();
    if (b < L.n_img) {
        const size_t P_ = (size_t)pitch * H;
        const uint32_t pb = (uint32_t)P_ * 4u;  // plane bytes (< 2^31: launch_blur_detect)
        const float* gb = L.gauss + (size_t)b * L.img_stride;
        const __amdgpu_buffer_rsrc_t rg0 = uniform_rsrc(gb, pb), rg1 = uniform_rsrc(gb + P_, pb),
                                     rg2 = uniform_rsrc(gb + 2 * P_, pb), rg3 = uniform_rsrc(gb + 3 * P_, pb),
                                     rg4 = uniform_rsrc(gb + 4 * P_, pb), rg5 = uniform_rsrc(gb + 5 * P_, pb);
        const int xb = sx * DR_COLS;
        const int x = xb - 1 + lane;  // this lane's column
        const int xc = min(max(x, 0), W - 1);
        const bool xout = lane >= 1 && lane <= DR_COLS && x >= kImageBorder && x < W - kImageBorder;
        const bool xst = lane >= 1 && lane <= DR_COLS && x < W;
        const int ya = sy * L.seg, yb = min(ya + L.seg, H);
        // G_4 ring columns [xb - 1 - R, xb + 63 + R): lane -> column ca, and
        // lanes < 2R also ca + 64
        const int ca = xb - 1 - R + lane;
        const int va = bd_index<P>(ca, W) * 4, vb = bd_index<P>(ca + 64, W) * 4, vx = xc * 4;
        float* rg = ring[wave];
        auto ld4 = [&](int q, float& a, float& c) {  // G_4 row q (reflected) into registers
            const int so = bd_index<P>(q, H) * pitch * 4;
            // both loads on every lane (vb is clamped into the row): an
            // exec-masked load sits behind a skip branch, which makes the
            // compiler's load-counter waits conservative
            a = buffer_load_f32(rg4, va, so);
            c = buffer_load_f32(rg4, vb, so);
        };
        auto ld03 = [&](int r, float (&d)[4]) {  // G_0..G_3 at (row r clamped, column xc)
            const int so = min(max(r, 0), H - 1) * pitch * 4;
            d[0] = buffer_load_f32(rg0, vx, so);
            d[1] = buffer_load_f32(rg1, vx, so);
            d[2] = buffer_load_f32(rg2, vx, so);
            d[3] = buffer_load_f32(rg3, vx, so);
        };
        // row filter of G_4 row q at this lane's column (q's ring row)
        auto rowpass = [&](int q) -> float {
            const float* p = rg + (q & (BD_RING - 1)) * BD_RP + lane;
            float v[2 * R + 1];
#pragma unroll
            for (int t = 0; t <= 2 * R; t++) v[t] = p[t];
            float acc = v[0] * L.taps.k[R];
#pragma unroll
            for (int t = 1; t <= 2 * R; t++) {
                const float kt = L.taps.k[t > R ? t - R : R - t];
                acc = P == kProfileOpenCV ? __builtin_fmaf(v[t], kt, acc) : acc + v[t] * kt;
            }
            return acc;
        };
        float win[2 * R + 1];  // row-filter outputs of rows r - R .. r + R
        // rolling detection state (k_detect_rows): row max / min of rows r - 2,
        // r - 1, r per DoG plane, the left / right max / min and centre of row r - 1
        float hmx[kDogPerOctave][3], hmn[kDogPerOctave][3];
        float lrx[kDogPerOctave], lrn[kDogPerOctave], ctr[kDogPerOctave];
        const float threshold = floorf(0.5f * kContrastThreshold / (float)kScalesPerOctave);
        const int q0 = ya - 1 - R, q1 = yb + R;  // G_4 rows filtered: [q0, q1]
        // Row data of one G_4 row q: its ring columns (a, c) and G_0..G_3 of
        // row r = q - R at this lane's column (the window-filling rows r <
        // ya - 1 load rows ya - 1 / ya instead; rows past the end re-load
        // the last one).  Four buffers: the two rows of a half-iteration are
        // processed from one pair while the next two rows' loads, issued at the
        // top of the half, are in flight into the other pair.  Every half
        // issues the same memory operations (a G_5 row outside the segment is
        // stored to an offset the buffer drops), so the compiler's load-counter
        // waits are static: each waits for loads issued a half-iteration
        // earlier, never for the ones just issued.
        struct RowBuf {
            float a, c, d[4];
        };
        auto load = [&](int q, RowBuf& B, int par) {
            const int qq = min(q, q1), r = qq - R;
            ld4(qq, B.a, B.c);
            ld03(r >= ya - 1 ? min(r, yb) : ya - 1 + par, B.d);
        };
        auto shift = [&]() {
#pragma unroll
            for (int j = 0; j < 2 * R; j++) win[j] = win[j + 1];
        };
        // G_4 row q from B into the ring, row-filtered into win[2R]; once the
        // window holds rows r - R .. r + R (r = q - R >= ya - 1): G_5 of row r,
        // row r's DoG values, the test of row r - 1.  Steps past q1 only
        // issue their (dropped) store.
        auto step = [&](int q, const RowBuf& B) {
            const bool on = q <= q1;  // uniform
            const int r = q - R;
            float g5 = 0.0f;
            if (on) {
                float* wp = rg + (q & (BD_RING - 1)) * BD_RP;
                wp[lane] = B.a;
                if (lane < 2 * R) wp[64 + lane] = B.c;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                win[2 * R] = rowpass(q);
                if constexpr (P == kProfileOpenCV) {
                    g5 = win[R] * L.taps.k[0];
#pragma unroll
                    for (int t = 1; t <= R; t++) g5 = __builtin_fmaf(win[R + t] + win[R - t], L.taps.k[t], g5);
                } else {
                    g5 = win[0] * L.taps.k[R];
#pragma unroll
                    for (int t = 1; t <= 2 * R; t++) g5 = g5 + win[t] * L.taps.k[t > R ? t - R : R - t];
                }
            }
            const uint32_t bad = (on && xst && r >= ya && r < yb) ? 0u : 0xfffffff0u;  // past every plane: dropped
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, g5), rg5,
                                                  ((uint32_t)(r * pitch * 4) + (uint32_t)vx) | bad, 0, 2 /* nt */);
            if (!(on && r >= ya - 1)) {  // uniform
                shift();
                return;
            }
            // row r's DoG values (G_4 from the ring: row r is resident)
            const float g4 = rg[(r & (BD_RING - 1)) * BD_RP + lane + R];
            float cur[kDogPerOctave];
            cur[0] = B.d[1] - B.d[0];
            cur[1] = B.d[2] - B.d[1];
            cur[2] = B.d[3] - B.d[2];
            cur[3] = g4 - B.d[3];
            cur[4] = g5 - g4;
            float nlx[kDogPerOctave], nln[kDogPerOctave];
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                const float l = dpp_from_left(cur[p]), rr = dpp_from_right(cur[p]);
                nlx[p] = fmaxf(l, rr);
                nln[p] = fminf(l, rr);
                hmx[p][2] = fmaxf(nlx[p], cur[p]);
                hmn[p][2] = fminf(nln[p], cur[p]);
            }
            const int y = r - 1;  // tested row: rows r - 2, r - 1, r are in
            if (y >= ya) {        // uniform
                const bool yin = xout && y >= kImageBorder && y < H - kImageBorder;
                float pmx[kDogPerOctave], pmn[kDogPerOctave];
#pragma unroll
                for (int p = 0; p < kDogPerOctave; p++) {
                    pmx[p] = fmaxf(fmaxf(hmx[p][0], hmx[p][1]), hmx[p][2]);
                    pmn[p] = fminf(fminf(hmn[p][0], hmn[p][1]), hmn[p][2]);
                }
                uint32_t ok3 = 0;
#pragma unroll
                for (int s_in = 1; s_in <= kScalesPerOctave; s_in++) {
                    const float val = ctr[s_in];
                    const float m8 = fmaxf(fmaxf(hmx[s_in][0], hmx[s_in][2]), lrx[s_in]);
                    const float n8 = fminf(fminf(hmn[s_in][0], hmn[s_in][2]), lrn[s_in]);
                    const float mx = fmaxf(fmaxf(pmx[s_in - 1], pmx[s_in + 1]), m8);
                    const float mn = fminf(fminf(pmn[s_in - 1], pmn[s_in + 1]), n8);
                    const bool ok = yin && fabsf(val) > threshold && (val > 0.0f ? val >= mx : val <= mn);
                    ok3 |= (uint32_t)ok << (s_in - 1);
                }
                if (__ballot(ok3 != 0)) {  // wave-uniform: rare
                    while (ok3) {
                        const int bit = __builtin_ctz(ok3);
                        ok3 &= ok3 - 1;
                        const uint64_t key = make_key((uint32_t)(L.img_base + b), (uint32_t)L.octave,
                                                      (uint32_t)(bit + 1), (uint32_t)y, (uint32_t)x);
                        const uint32_t li = atomicAdd(&lcount, 1u);
                        if (li < DR_LCAP) {
                            lcand[li] = key;
                        } else {
                            const uint32_t slot = atomicAdd(L.counter, 1u);
                            if (slot < L.cap) L.cand[slot] = key;
                        }
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                hmx[p][0] = hmx[p][1];
                hmn[p][0] = hmn[p][1];
                hmx[p][1] = hmx[p][2];
                hmn[p][1] = hmn[p][2];
                lrx[p] = nlx[p];
                lrn[p] = nln[p];
                ctr[p] = cur[p];
            }
            shift();
        };
        // rows q, q + 1 from (A0, A1) while q + 2, q + 3 load into (B0, B1),
        // then the other way round (even / odd rows: par 0 / 1)
        RowBuf A0, A1, B0, B1;
        load(q0, A0, 0);
        load(q0 + 1, A1, 1);
        for (int q = q0; q <= q1; q += 4) {
            load(q + 2, B0, 0);
            load(q + 3, B1, 1);
            __builtin_amdgcn_sched_barrier(0);
            step(q, A0);
            step(q + 1, A1);
            __builtin_amdgcn_sched_barrier(0);
            load(q + 4, A0, 0);
            load(q + 5, A1, 1);
            __builtin_amdgcn_sched_barrier(0);
            step(q + 2, B0);
            step(q + 3, B1);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // one global atomic per block, then a coalesced copy of the block's list
    __syncthreads();
    const uint32_t nl = lcount < DR_LCAP ? lcount : DR_LCAP;
    if (nl == 0) return;
    if (tid == 0) gbase = atomicAdd(L.counter, nl);
    __syncthreads();
    for (uint32_t i = tid; i < nl; i += 256)
        if (gbase + i < L.cap) L.cand[gbase + i] = lcand[i];
}

// PathOpts::fused_detect: 0 keeps blur 5 and detection apart, 2 fuses every
// octave it can at 32-row segments (test paths)
int launch_blur_detect(int R, BlurDetectLaunch& L, hipStream_t st, const PathOpts& o) {
    if (o.fused_detect == 0) return -1;
    const bool force = o.fused_detect == 2;
    const bool ok = L.W > R + 1 && L.H > R + 1 && L.W >= 2 * kImageBorder && L.H >= 2 * kImageBorder &&
                    (uint64_t)L.H * (uint64_t)L.pitch * 4 < (1ull << 31) && L.n_img > 0;
    if (!ok) return -1;
    const bool ocv = L.profile == kProfileOpenCV;
    if (!((ocv && R == 13) || (!ocv && R == 7))) return -1;
    L.nsx = (L.W + DR_COLS - 1) / DR_COLS;
    // row segments: a segment re-filters 2R + 2 halo rows, so long ones, but
    // enough waves to fill the chip (>= ~16 k).  A wave walks its segment row
    // after row, so an octave too small for that at >= 64-row segments (one
    // 1080p frame's octaves, a batch's small octaves) is left to launch_blur +
    // k_detect_rows: there the fused pass is a chain of latency-bound row
    // steps (one frame's octave 4: 54 us against 10 us for its blur 5)
    int seg = 0;
    for (int s : {256, 128, 64}) {
        if ((long)L.nsx * ((L.H + s - 1) / s) * L.n_img >= 16384) {
            seg = s;
            break;
        }
    }
    if (force) seg = 32;  // many segment boundaries on test-sized frames
    if (!seg) return -1;
    L.seg = seg;
    L.nsy = (L.H + seg - 1) / seg;
    const long waves = (long)L.nsx * L.nsy * L.n_img;
    const dim3 grid((uint32_t)((waves + 3) / 4));
    if (ocv)
        hipLaunchKernelGGL((k_blur_detect<13, kProfileOpenCV>), grid, dim3(256), 0, st, L);
    else
        hipLaunchKernelGGL((k_blur_detect<7, kProfileImageproc>), grid, dim3(256), 0, st, L);
    return 0;
}

// ---------------------------------------------------------------------------
// k_refine: one thread per candidate extremum -- interpolate_extremum,
// extremum_contrast, extremum_is_on_edge (src/lib.rs:334-367); accepted
// extrema are appended with one atomic per wave.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool refine_one(const RefineLaunch& L, uint64_t key, ExtRec& e) {
    const int b = (int)(key >> kKeyImgShift);
    const int o = (int)((key >> kKeyOctShift) & 15);
    const int s_in = (int)((key >> kKeyScaleShift) & 3);
    const int y = (int)((key >> kKeyYShift) & kKeyCoordMask);
    const int x = (int)((key >> kKeyXShift) & kKeyCoordMask);
    const int W = L.ow[o], H = L.oh[o], pitch = L.opitch[o];
    const gfloat* g0 = as_global(L.gauss[o]) + (size_t)(b - L.img_base) * L.g_img_stride[o];
    const size_t P = (size_t)pitch * H;
    int sc = s_in, xi = x, yi = y;
    float os, ox, oy;
    Nbhd n;
    int vlo = 0, vhi = H;  // rows of this octave's Gaussians that are exact
    if (L.band_flag) {
        vlo = max(0, (int)((uint64_t)H * L.band_r / L.band_n) - 1 - L.band_margin);
        vhi = min(H, (int)((uint64_t)H * (L.band_r + 1) / L.band_n) + 1 + L.band_margin);
    }
    if (!interpolate(g0, P, W, H, pitch, sc, xi, yi, os, ox, oy, n, L.band_flag, vlo, vhi)) return false;
    // the converged point's neighbourhood is n (the last step did not move)
#define PREV(dy, dx) n.d[0][(dy) + 1][(dx) + 1]
#define CURR(dy, dx) n.d[1][(dy) + 1][(dx) + 1]
#define NEXT(dy, dx) n.d[2][(dy) + 1][(dx) + 1]
    // extremum_contrast (src/lib.rs:606-626)
    const float g1 = (NEXT(0, 0) - PREV(0, 0)) / 2.f;
    const float g2 = (CURR(1, 0) - CURR(-1, 0)) / 2.f;
    const float g3 = (CURR(0, 1) - CURR(0, -1)) / 2.f;
    const float interp = os * g1 + oy * g2 + ox * g3;
    const float contrast = fabsf(CURR(0, 0) + interp / 2.f);
    if (contrast * (float)kScalesPerOctave <= kContrastThreshold) return false;
    // extremum_is_on_edge (src/lib.rs:630-653)
    const float v2 = CURR(0, 0) * 2.0f;
    const float h11 = CURR(1, 0) + CURR(-1, 0) - v2;
    const float d22 = CURR(0, 1) + CURR(0, -1) - v2;
    const float h12 = (CURR(1, 1) - CURR(1, -1) - CURR(-1, 1) + CURR(-1, -1)) / 4.f;
#undef PREV
#undef CURR
#undef NEXT
    const float tr = d22 + h11;
    const float det = d22 * h11 - h12 * h12;
    if (det <= 0.f) return false;
    if ((tr * tr * kEdgeThreshold) > (kEdgeThreshold + 1.0f) * (kEdgeThreshold + 1.0f) * det) return false;
    // an accepted keypoint's orientation / descriptor patch must be exact too
    // (at the image's own top / bottom rows the patch reads clamp, so no limit)
    if (L.band_flag && ((vlo > 0 && yi - L.band_patch < vlo) || (vhi < H && yi + L.band_patch >= vhi)))
        atomicOr(L.band_flag, 1u);
    e.key = key;
    e.img = b;
    e.octave = o;
    e.scale = sc;
    e.x = xi;
    e.y = yi;
    e.off_s = os;
    e.off_x = ox;
    e.off_y = oy;
    e.response = contrast;
    e.pad = 0;
    return true;
}

#ifndef SIFT_REFINE_WPE
#define SIFT_REFINE_WPE 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_REFINE_WPE))) void k_refine(const RefineLaunch L) {
    const uint32_t n = min(*L.n_cand, L.cand_cap);
    const int lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x * 256; base < n; base += gridDim.x * 256) {
        const uint32_t i = base + threadIdx.x;
        ExtRec e;
        const bool keep = i < n && refine_one(L, L.cand[i], e);
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
    const uint32_t n_ext = min(*L.n_ext, L.ext_cap);
    // one group of 4 extrema per workgroup; the grid covers the bound, the
    // device count ends it early (block-uniform)
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
            e = L.ext[r];
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
        kp.pad = 0;
        kp.x = kp_x;
        kp.y = kp_y;
        kp.size = kp_scale * osf;
        kp.angle = 360.0f - (360.0f / (float)kOriBins) * bin;
        kp.response = e.response;
        kp.pad2 = 0.f;
        L.out[slot] = kp;
    }
}

void launch_orient(const OrientLaunch& L, hipStream_t st) {
    if (L.ext_cap == 0) return;
    dim3 grid((L.ext_cap + 3) / 4);
    hipLaunchKernelGGL(k_orient, grid, dim3(256), 0, st, L);
}

}  // namespace siftmi
