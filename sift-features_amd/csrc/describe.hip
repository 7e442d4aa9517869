// 4x4x8 SIFT descriptors on MI355X: one wave (one workgroup) per keypoint,
// no atomics.  Two accumulation strategies over the same per-sample math:
//   describe_wave_fast  (default) lane-private LDS histograms, summed per bin;
//                       u8 components within +-1 of the reference;
//   describe_wave_exact bin-owner lanes adding in the reference's sequential
//                       sample order -- bit-identical bins and bytes (up to
//                       1-ulp differences of the f64-evaluated exp / atan2 /
//                       sin / cos vs glibc), ~7x slower.
//
// Reference: compute_descriptors / compute_descriptor (src/lib.rs:759-990).
// Every expression keeps the reference's operand order (-ffp-contract=off);
// the L2 norms use the reference's chunk-of-4 order (src/lib.rs:957-976).
#include <float.h>

#include <algorithm>
#include <type_traits>

#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {


// Per-wave LDS scratch: the row table of the sample enumeration (first
// column, prefix count; up to 2*39+1 rows) and one band of per-sample records.
constexpr int ROWS_MAX = 80;
constexpr int REC_CAP = 1664;  // records per band; a window (<= 3223 samples) needs at most 2 bands

struct DescScratch {
    float2 rec[REC_CAP];  // (mag * weight, obin) per compacted sample; mag < 0 marks a rejected sample
    int rowlo[ROWS_MAX];
    int rowpre[ROWS_MAX + 1];
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Footprint of a cell on one axis: a*xi + k*yi in [c - 3.5, c - 1.5).  For
// |a| > 1e-6 the xi bounds are lo(yi) = lo0 + kk*yi, hi(yi) = hi0 + kk*yi
// (widened by 2 columns; the exact f32 floor test decides membership).
// Otherwise the constraint does not depend on xi: the whole row is in or out.
__device__ __forceinline__ void lin_bounds(float a, float k, float c, float& lo0, float& hi0, float& kk,
                                           bool& row_only) {
    row_only = !(fabsf(a) > 1e-6f);
    const float inv = row_only ? 0.0f : 1.0f / a;
    const float u = (c - 3.5f) * inv, v = (c - 1.5f) * inv;
    lo0 = fminf(u, v) - 2.0f;
    hi0 = fmaxf(u, v) + 2.0f;
    kk = -k * inv;
}
__device__ __forceinline__ bool row_in(float fy, float k, float c) {
    const float b = fy * k;
    return b >= c - 3.5f - 1e-3f && b < c - 1.5f + 1e-3f;
}
__device__ __forceinline__ float row_lo(float lo0, float kk, bool row_only, float fy, float k, float c) {
    return row_only ? (row_in(fy, k, c) ? -1e9f : 1e9f) : lo0 + kk * fy;
}
__device__ __forceinline__ float row_hi(float hi0, float kk, bool row_only, float fy, float k, float c) {
    return row_only ? (row_in(fy, k, c) ? 1e9f : -1e9f) : hi0 + kk * fy;
}

// Inclusive wave prefix sum with DPP row shifts and row broadcasts (no LDS
// permutes): within each 16-lane row, then across rows.
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// Per-row column intervals of the rotated 4x4 region (window rows
// -radius..radius, n <= 79: lanes own rows lane and lane + 64), widened by one
// column on each side -- the reference's f32 predicate decides membership per
// sample -- and their exclusive prefix sums (the compacted sample index of
// each row's first sample), built with wave scans.
// Optional clip window [xmin, xmax] x [ymin, ymax] (window coordinates): the
// fast path drops samples outside the image here instead of testing each one.
// SHRINK (fast path): the up to 3 end columns of each row that fail the fast
// path's own f32 region test are dropped here rather than enumerated (the
// per-sample test stays, so this only removes samples it would reject).
template <bool SHRINK = false, class T = int>
__device__ __forceinline__ void build_row_table(T* rowlo, T* rowpre, int radius, float cos_s, float sin_s,
                                                int lane, int xmin = INT_MIN, int xmax = INT_MAX,
                                                int ymin = INT_MIN, int ymax = INT_MAX) {
    const int n = 2 * radius + 1;
    const double c = cos_s, s = sin_s;
    const bool cz = !(fabs(c) > 1e-30), sz = !(fabs(s) > 1e-30);
    const double rc = cz ? 0.0 : 1.0 / c, rs = sz ? 0.0 : 1.0 / s;
    int cnt[2] = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int row = lane + 64 * h;
        if (row < n) {
            const double yi = (double)(row - radius);
            double lo = fmax(-radius, (double)xmin), hi = fmin(radius, (double)xmax);
            bool empty = row - radius < ymin || row - radius > ymax;
            if (!cz) {
                const double a = (yi * s - 2.5) * rc, b = (yi * s + 2.5) * rc;
                lo = fmax(lo, fmin(a, b) - 1.0);
                hi = fmin(hi, fmax(a, b) + 1.0);
            } else {
                empty = !(fabs(yi * s) < 2.5 + 1e-3);
            }
            if (!sz) {
                const double a = (-yi * c - 2.5) * rs, b = (-yi * c + 2.5) * rs;
                lo = fmax(lo, fmin(a, b) - 1.0);
                hi = fmin(hi, fmax(a, b) + 1.0);
            } else {
                empty = empty || !(fabs(yi * c) < 2.5 + 1e-3);
            }
            int ilo = (int)floor(lo), ihi = (int)ceil(hi);
            if (SHRINK && !empty) {
                const float fy = (float)(row - radius);
                auto inside = [&](int xi) {  // describe_wave_fast's test, same f32 operations
                    const float fx = (float)xi;
                    const float col_bin = (fx * cos_s - fy * sin_s) + (float)(kDescHist / 2);
                    const float row_bin = (fx * sin_s + fy * cos_s) + (float)(kDescHist / 2);
                    return row_bin > -0.5f && row_bin < (float)kDescHist + 0.5f && col_bin > -0.5f &&
                           col_bin < (float)kDescHist + 0.5f;
                };
#pragma unroll
                for (int k = 0; k < 3; k++) ilo += (ilo <= ihi && !inside(ilo)) ? 1 : 0;
#pragma unroll
                for (int k = 0; k < 3; k++) ihi -= (ihi >= ilo && !inside(ihi)) ? 1 : 0;
            }
            rowlo[row] = (T)ilo;
            cnt[h] = (empty || ihi < ilo) ? 0 : ihi - ilo + 1;
        }
    }
    const int s0 = wave_incl_scan(cnt[0]), s1 = wave_incl_scan(cnt[1]);
    const int t0 = __builtin_amdgcn_readlane(s0, 63);
    if (lane < n) rowpre[lane + 1] = (T)s0;
    if (lane + 64 < n) rowpre[lane + 65] = (T)(s1 + t0);
    if (lane == 0) rowpre[0] = 0;
    wave_sync();
}

// Sequential sum s[0] + s[2] + ... + s[62] over the even lanes (the
// reference's chunk order) with v_readlane: the 32 reads are independent and
// the adds take scalar operands, instead of a chain of 31 LDS permutes.
__device__ __forceinline__ float chunk_sum(float s) {
    const int si = __float_as_int(s);
    float t = __int_as_float(__builtin_amdgcn_readlane(si, 0));
#pragma unroll
    for (int j = 1; j < 32; j++) t = t + __int_as_float(__builtin_amdgcn_readlane(si, 2 * j));
    return t;
}

// Normalisation (src/lib.rs:951-989) of the 128 interior bins held two per
// lane (lane l: flat[2l], flat[2l+1]); chunk j = flat[4j..4j+4) = lanes 2j,
// 2j+1, summed in the reference's exact chunk-of-4 order.
// Wave sum in DPP tree order (fast path: its bins already differ from the
// reference's by summation order, and so may the norms)
__device__ __forceinline__ float wave_tree_sum(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, false));  // row_shr:1
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xf, 0xf, false));  // row_shr:2
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xf, 0xf, false));  // row_shr:4
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xf, 0xf, false));  // row_shr:8
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false));  // row_bcast:15
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false));  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// FAST: the L2 sums in DPP tree order (describe_wave_fast); otherwise the
// reference's chunk-of-4 order (describe_wave_exact)
template <bool FAST = false>
__device__ __forceinline__ void describe_normalize(float acc0, float acc1, uint8_t* __restrict__ out, int lane) {
    float l2, l2c, v0, v1;
    if constexpr (FAST) {
        l2 = sqrtf(wave_tree_sum(acc0 * acc0 + acc1 * acc1));
        const float cap = l2 * 0.2f;
        v0 = fminf(acc0, cap);
        v1 = fminf(acc1, cap);
        l2c = wave_tree_sum(v0 * v0 + v1 * v1);
    } else {
    const float c_hi0 = __shfl(acc0, (lane + 1) & 63), c_hi1 = __shfl(acc1, (lane + 1) & 63);
    float s = 0.0f;
    s += acc0 * acc0;
    s += acc1 * acc1;
    s += c_hi0 * c_hi0;
    s += c_hi1 * c_hi1;
    l2 = chunk_sum(s);
    l2 = sqrtf(l2);
    const float cap = l2 * 0.2f;
    v0 = fminf(acc0, cap), v1 = fminf(acc1, cap);
    const float d_hi0 = __shfl(v0, (lane + 1) & 63), d_hi1 = __shfl(v1, (lane + 1) & 63);
    s = 0.0f;
    s += v0 * v0;
    s += v1 * v1;
    s += d_hi0 * d_hi0;
    s += d_hi1 * d_hi1;
    l2c = chunk_sum(s);
    }
    l2c = sqrtf(l2c);
    const float norm = 512.0f / fmaxf(l2c, FLT_EPSILON);
    const int32_t q0 = sat_i32(roundf(v0 * norm)), q1v = sat_i32(roundf(v1 * norm));
    const uint32_t u0 = q0 > 255 ? 255u : (uint32_t)(uint8_t)q0;
    const uint32_t u1 = q1v > 255 ? 255u : (uint32_t)(uint8_t)q1v;
    reinterpret_cast<uint16_t*>(out)[lane] = (uint16_t)(u0 | (u1 << 8));
}

// Wave-cooperative compute_descriptor (src/lib.rs:785-990), bit-exact.
//
// The reference adds every sample's 8 trilinear contributions into a 6x6x8
// histogram in row-major sample order; only the 4x4 interior (128 bins) is
// kept.  Here lane l owns the 2 interior bins (cell 1 + l/16 ... , orientation
// pair l%4): phase A evaluates the per-sample values once (gradient, Gaussian
// weight, f64 atan2) into LDS records, phase B walks, in row-major order,
// only the samples whose 2x2-cell footprint covers the lane's cell and adds
// them to its two bins -- the reference's exact per-bin summation order, with
// no atomics.  Only samples inside the rotated 4x4 region are enumerated
// (per-row column intervals computed in float and widened; the reference's f32
// predicate decides), the window is split into bands of <= REC_CAP samples.
//
// kAblate (performance experiments only, tools/ubench_kernels.hip; 0 in the
// product): bit 0 skip phase B, bit 1 replace atan2, bit 2 replace exp,
// bit 3 replace the gradient loads.
template <int kAblate = 0>
__device__ __forceinline__ void describe_wave_exact(const float* __restrict__ img, int pitch, int width, int height,
                                                    float xf, float yf, float scale, float orientation,
                                                    float sin_ori, float cos_ori, DescScratch& sc,
                                                    uint8_t* __restrict__ out, int lane) {
    const int32_t x = (int32_t)sat_u32(roundf(xf));
    const int32_t y = (int32_t)sat_u32(roundf(yf));
    const float BIN_ANGLE_STEP = (float)kDescBins / 360.0f;
    const float hist_width = kLambdaDescr * scale;
    int radius = sat_i32(roundf(kLambdaDescr * scale * 1.41421356237309504880f * (float)(kDescHist + 1) * 0.5f));
    radius = radius < 0 ? 0 : (radius > (ROWS_MAX - 2) / 2 ? (ROWS_MAX - 2) / 2 : radius);
    // (sin_ori, cos_ori): orientation_rotation(orientation), src/lib.rs:800-801
    const float sin_s = sin_ori / hist_width, cos_s = cos_ori / hist_width;
    const int n = 2 * radius + 1;
    // 1. per-row candidate column interval of the whole 4x4 region
    build_row_table(sc.rowlo, sc.rowpre, radius, cos_s, sin_s, lane);
    // lane role: interior cell (cr, cc) in 1..4, orientation bins b0, b0 + 1
    const int ci = lane >> 2;
    const int cr = 1 + (ci >> 2), cc = 1 + (ci & 3);
    const int b0 = 2 * (lane & 3), b1 = b0 + 1;
    float acc0 = 0.0f, acc1 = 0.0f;
    // footprint bounds per row as linear functions of yi (widened by 2 columns):
    //   r1 in {cr-1, cr}  <=>  row_rot = xi*sin_s + yi*cos_s in [cr - 3.5, cr - 1.5)
    //   q1 in {cc-1, cc}  <=>  col_rot = xi*cos_s - yi*sin_s in [cc - 3.5, cc - 1.5)
    // (a ~ 0 coefficient makes the constraint row-only; see lin_bounds)
    float aLo, aHi, aK, bLo, bHi, bK;
    bool aRow, bRow;
    lin_bounds(sin_s, cos_s, (float)cr, aLo, aHi, aK, aRow);
    lin_bounds(cos_s, -sin_s, (float)cc, bLo, bHi, bK, bRow);
    for (int row0 = 0; row0 < n;) {
        // band [row0, row1): as many rows as fit in REC_CAP records
        int row1 = row0 + 1;
        while (row1 < n && sc.rowpre[row1 + 1] - sc.rowpre[row0] <= REC_CAP) row1++;
        const int kbase = sc.rowpre[row0], kend = sc.rowpre[row1];
        // phase A: per-sample values, lane-strided over the band
        int row = row0;
        for (int k = kbase + lane; k < kend; k += 64) {
            while (sc.rowpre[row + 1] <= k) row++;
            const int yi = row - radius;
            const int xi = sc.rowlo[row] + (k - sc.rowpre[row]);
            const float col_rot = (float)xi * cos_s - (float)yi * sin_s;
            const float row_rot = (float)xi * sin_s + (float)yi * cos_s;
            const float row_bin = row_rot + (float)(kDescHist / 2);
            const float col_bin = col_rot + (float)(kDescHist / 2);
            const int32_t ay = y + yi, ax = x + xi;
            float2 rc = make_float2(-1.0f, 0.0f);
            if (row_bin > -0.5f && row_bin < (float)kDescHist + 0.5f && col_bin > -0.5f &&
                col_bin < (float)kDescHist + 0.5f && ay > 0 && ay < height - 1 && ax > 0 && ax < width - 1) {
                float dx, dy;
                if (kAblate & 8) {
                    dx = (float)xi * 0.01f + 0.001f;
                    dy = (float)yi * 0.01f - 0.002f;
                } else {
                    const gfloat* rw = as_global(img) + (size_t)ay * pitch;
                    dx = rw[ax + 1] - rw[ax - 1];
                    dy = rw[ax - pitch] - rw[ax + pitch];
                }
                const float wsq = col_rot * col_rot + row_rot * row_rot;
                const float weight =
                    (kAblate & 4) ? 1.0f + wsq * (-0.125f) : exp_f32(wsq * (-2.f / (float)(kDescHist * kDescHist)));
                // ((atan2(dy, dx).to_degrees() + 360) % 360) as f32 - orientation;
                // the f64 remainder of v in [180, 540] by 360 is exactly v or v - 360
                double deg = ((kAblate & 2) ? (double)(dy * 50.0f + dx)
                                            : atan2((double)dy, (double)dx) * (180.0 / 3.14159265358979323846)) +
                             360.0;
                deg = deg >= 360.0 ? deg - 360.0 : deg;
                const float ori = (float)deg - orientation;
                const float mag = sqrtf(dx * dx + dy * dy);
                rc = make_float2(mag * weight, ori * BIN_ANGLE_STEP);
            }
            sc.rec[k - kbase] = rc;
        }
        wave_sync();
        // phase B: this lane's 2x2-cell footprint, row-major.  Each lane walks
        // its own flattened (row, column) cursor so the wave iterates
        // max-over-lanes(footprint) times instead of sum-over-rows(max).
        if (!(kAblate & 1)) {
            int rw = row0 - 1, xi = 1, xb = 0, kr = 0, yi = 0;
            for (;;) {
                if (xi > xb) {  // advance to the next row with a non-empty interval
                    if (++rw >= row1) break;
                    yi = rw - radius;
                    const int pre = sc.rowpre[rw];
                    const int cnt = sc.rowpre[rw + 1] - pre;
                    const int rlo = sc.rowlo[rw];
                    const float fy = (float)yi;
                    float xlo = fmaxf(row_lo(aLo, aK, aRow, fy, cos_s, (float)cr),
                                      row_lo(bLo, bK, bRow, fy, -sin_s, (float)cc));
                    float xhi = fminf(row_hi(aHi, aK, aRow, fy, cos_s, (float)cr),
                                      row_hi(bHi, bK, bRow, fy, -sin_s, (float)cc));
                    xi = max(rlo, (int)ceilf(xlo));
                    xb = min(rlo + cnt - 1, (int)floorf(xhi));
                    kr = pre - rlo - kbase;
                    continue;
                }
                const float2 rc = sc.rec[kr + xi];
                const float col_rot = (float)xi * cos_s - (float)yi * sin_s;
                const float row_rot = (float)xi * sin_s + (float)yi * cos_s;
                xi++;
                if (rc.x < 0.0f) continue;
                const float rb = (row_rot + (float)(kDescHist / 2)) - 0.5f;
                const float cb = (col_rot + (float)(kDescHist / 2)) - 0.5f;
                const float rf = floorf(rb), cf = floorf(cb);
                const int r1 = (int)rf + 1, q1 = (int)cf + 1;
                if ((r1 != cr && r1 + 1 != cr) || (q1 != cc && q1 + 1 != cc)) continue;
                const float mag = rc.x, obin = rc.y;
                const float of = floorf(obin);
                const float ori_frac = obin - of;
                int o0 = (int)of;
                o0 = o0 < 0 ? o0 + kDescBins : (o0 >= kDescBins ? o0 - kDescBins : o0);
                const int o1 = o0 + 1 >= kDescBins ? 0 : o0 + 1;
                const float c1 = mag * (rb - rf), c0 = mag - c1;
                const float crow = cr == r1 ? c0 : c1;
                const float t = crow * (cb - cf);
                const float ccol = cc == q1 ? crow - t : t;
                const float hi = ccol * ori_frac, lo = ccol - hi;
                acc0 += o0 == b0 ? lo : (o1 == b0 ? hi : 0.0f);
                acc1 += o0 == b1 ? lo : (o1 == b1 ? hi : 0.0f);
            }
        } else {
            acc0 += sc.rec[lane].x;
        }
        wave_sync();
        row0 = row1;
    }
    describe_normalize(acc0, acc1, out, lane);
}

// Fast path (the default): lane-private 4x4x8 histograms.
//
// Lanes walk the compacted samples with stride 64 and add each sample's
// interior contributions (cells 1..4 x 1..4; the reference discards the
// border ring, src/lib.rs:951) into a private 128-bin slice of LDS (bin-major,
// lane-minor layout: conflict-free) with plain read-add-write (LDS float atomics cost ~3 cycles per lane on gfx950,
// tools/ubench_lds.hip); the 64 slices are then summed per bin.  Per-sample
// arithmetic is the reference's; only the order of the bin additions differs,
// so bins agree to f32 rounding and the u8 components to +-1 (the tolerance
// tests/test_gpu_parity.py states).  describe_wave_exact is the bit-exact
// alternative (sift_mi_set_exact_descriptors).
//
// kShare lanes share one slice (64 / kShare slices per wave): their updates
// are issued group by group (lanes [g*S, (g+1)*S) in step g), so no two lanes
// of a slice write in the same instruction.  Sharing trades LDS instructions
// for LDS footprint -- 38.9 KB per wave at kShare = 1 (one wave per SIMD),
// 19.5 KB at 2, 9.7 KB at 4 -- i.e. for occupancy.
//
// Slice layout: 9 slots per interior cell (slot 8 aliases orientation 0 and is
// folded into it at the end), so a sample's two orientation bins o0, o0 + 1 of
// a cell are always adjacent slots -- one ds_read2_b32 / ds_write2_b32 and one
// v_pk_add_f32 per cell -- plus one dummy pair per footprint corner that takes
// the border-ring contributions (the reference discards that ring): a
// sample's 4 slot pairs never alias, so all reads issue before the writes.
constexpr int PRIV_STRIDE = 16 * 9 + 4 * 2;

// The row table in 16-bit entries (|column| <= 40, prefix counts <= 3223):
// 10052 B per wave at kShare 4, so 16 waves fit in a CU's 160 KB of LDS (32-bit
// entries: 10372 B, 15 waves).
template <int kShare>
struct DescScratchFast {
    float h[64 / kShare * PRIV_STRIDE];
    int16_t rowlo[ROWS_MAX];
    int16_t rowpre[ROWS_MAX + 1];
};

// atan2(dy, dx) in degrees for a pair of samples: |t| = min/max in [0, 1]
// (v_rcp_f32), atan(t) = t + t s P(s) (s = t^2, degree-7 minimax, |error| <
// 6e-8 on [0, 1] in f32), then the octant / quadrant reflections.  atan2(+0,
// +0) = 0 and atan2(+0, x < 0) = 180 as the reference's; the gradient
// differences are never -0.
__device__ __forceinline__ f2v atan2_deg2(f2v dy, f2v dx) {
    const f2v ax = __builtin_elementwise_abs(dx), ay = __builtin_elementwise_abs(dy);
    const f2v mx = __builtin_elementwise_max(ax, ay), mn = __builtin_elementwise_min(ax, ay);
    f2v t = mn * f2v{__builtin_amdgcn_rcpf(mx.x), __builtin_amdgcn_rcpf(mx.y)};
    t.x = mx.x > 0.0f ? t.x : 0.0f;
    t.y = mx.y > 0.0f ? t.y : 0.0f;
    const f2v sq = t * t;
    f2v p = f2v{0.0025999427f, 0.0025999427f};
    p = __builtin_elementwise_fma(p, sq, f2v{-0.015042510f, -0.015042510f});
    p = __builtin_elementwise_fma(p, sq, f2v{0.040974170f, 0.040974170f});
    p = __builtin_elementwise_fma(p, sq, f2v{-0.073540933f, -0.073540933f});
    p = __builtin_elementwise_fma(p, sq, f2v{0.10567977f, 0.10567977f});
    p = __builtin_elementwise_fma(p, sq, f2v{-0.14184459f, -0.14184459f});
    p = __builtin_elementwise_fma(p, sq, f2v{0.19990212f, 0.19990212f});
    p = __builtin_elementwise_fma(p, sq, f2v{-0.33332980f, -0.33332980f});
    f2v a = __builtin_elementwise_fma(t * sq, p, t);
    constexpr float kHalfPi = 1.57079632679489662f, kPi = 3.14159265358979324f;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        float v = ay[j] > ax[j] ? kHalfPi - a[j] : a[j];
        v = dx[j] < 0.0f ? kPi - v : v;
        a[j] = dy[j] < 0.0f ? -v : v;
    }
    return a * (180.0f / kPi);
}

// Fast path per-sample math: the reference's expressions (same operand order,
// -ffp-contract=off) in packed f32 on two samples at a time, with hardware
// transcendentals -- v_sqrt_f32 / v_exp_f32 (1 ulp) and atan2_deg2 -- in place
// of the correctly rounded ones: the sample angle moves by < 1e-5 degree and
// the weights by ~1e-7 relative, inside the fast path's +-1 u8 tolerance.
struct NoHook {
    __device__ void operator()() const {}
};

// `mid` runs between the sample loop and the final reduction (the caller
// issues its next keypoint's loads there, hidden behind the reduction).
template <int kShare, int kAblate = 0, class Mid = NoHook>
__device__ __forceinline__ void describe_wave_fast(const float* __restrict__ img, int pitch, int width, int height,
                                                   float xf, float yf, float scale, float orientation,
                                                   float sin_ori, float cos_ori, DescScratchFast<kShare>& sc,
                                                   uint8_t* __restrict__ out, int lane, Mid mid = Mid(),
                                                   uint32_t* n_samples = nullptr) {
    constexpr int NS = 64 / kShare;  // slices
    const int32_t x = (int32_t)sat_u32(roundf(xf));
    const int32_t y = (int32_t)sat_u32(roundf(yf));
    const float BIN_ANGLE_STEP = (float)kDescBins / 360.0f;
    const float hist_width = kLambdaDescr * scale;
    int radius = sat_i32(roundf(kLambdaDescr * scale * 1.41421356237309504880f * (float)(kDescHist + 1) * 0.5f));
    radius = radius < 0 ? 0 : (radius > (ROWS_MAX - 2) / 2 ? (ROWS_MAX - 2) / 2 : radius);
    // (sin_ori, cos_ori): orientation_rotation(orientation), src/lib.rs:800-801
    const float sin_s = sin_ori / hist_width, cos_s = cos_ori / hist_width;
    const int n = 2 * radius + 1;
    // bin b of lane l's slice lives at h[b * 64 + l]: every lane's read-add-write
    // of any bin hits its own bank (l mod 32) -> conflict-free scatter
    float* hp = sc.h + (lane & (NS - 1));
    const int grp = lane / NS;
#pragma unroll
    for (int i = 0; i < PRIV_STRIDE * NS / 4; i += 64)
        if (i + lane < PRIV_STRIDE * NS / 4) reinterpret_cast<float4*>(sc.h)[i + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    // samples outside the image (0 < y + yi < height - 1, 0 < x + xi < width - 1
    // fails) are not enumerated
    build_row_table<true>(sc.rowlo, sc.rowpre, radius, cos_s, sin_s, lane, 1 - x, width - 2 - x, 1 - y, height - 2 - y);
    const int total = (kAblate & 64) ? 0 : sc.rowpre[n];  // kAblate bit 6: no samples (per-keypoint overhead)
    if (n_samples) *n_samples += (uint32_t)total;
    // Lane-strided samples: one load instruction touches ~64 neighbouring
    // pixels (2-3 cache lines) instead of 64 scattered ones.  Each iteration
    // takes two samples per lane (k, k + 64) -- packed math, independent
    // chains for the ~2 waves per SIMD the LDS footprint allows -- and the
    // gradient loads of the next two are in flight meanwhile.
    int row = 0;
    auto locate = [&](int k, int& xi, int& yi) {
        while (sc.rowpre[row + 1] <= k) row++;
        yi = row - radius;
        xi = sc.rowlo[row] + (k - sc.rowpre[row]);
    };
    // The gradient reads of a sample (yy, xx) = (y + yi, x + xi): rows yy - 1
    // .. yy + 1 of the window's clipped rows [rb, re] (1 <= rb, re <= H - 2).
    // A buffer resource based one row above rb and one column left of 0:
    // voffset ((yy - rb) * pitch + xx) * 4 (32-bit, < 2^24 products), the row
    // in a uniform soffset and the column in the immediate -- no 64-bit
    // address arithmetic per sample.
    const int rb = max(y - radius, 1), re = min(y + radius, height - 2);
    const __amdgpu_buffer_rsrc_t rs =
        uniform_rsrc(img + (ptrdiff_t)(rb - 1) * pitch - 1, (uint32_t)max(re - rb + 3, 0) * (uint32_t)pitch * 4u);
    const int s1 = __builtin_amdgcn_readfirstlane(4 * pitch), s2 = 2 * s1;
    auto fetch = [&](int xi, int yi, float& l, float& r, float& u, float& d) {
        const int vo = ((int)__umul24((uint32_t)(yi + y - rb), (uint32_t)pitch) + x + xi) * 4;
        r = buffer_load_f32(rs, vo + 8, s1);
        l = buffer_load_f32(rs, vo, s1);
        u = buffer_load_f32(rs, vo + 4, 0);
        d = buffer_load_f32(rs, vo + 4, s2);
    };
    f2v sink = {0.f, 0.f};  // kAblate bit 0: register sink instead of the slice updates
    int nxi[2] = {0, 0}, nyi[2] = {0, 0};
    float nl[2] = {0.f, 0.f}, nr[2] = {0.f, 0.f}, nu[2] = {0.f, 0.f}, nd[2] = {0.f, 0.f};
    if (total > 0) {
#pragma unroll
        for (int u = 0; u < 2; u++) {
            locate(min(lane + 64 * u, total - 1), nxi[u], nyi[u]);
            if (!(kAblate & 8)) fetch(nxi[u], nyi[u], nl[u], nr[u], nu[u], nd[u]);
        }
    }
    for (int k = lane; k - lane < total; k += 128) {
        const int xi[2] = {nxi[0], nxi[1]}, yi[2] = {nyi[0], nyi[1]};
        const f2v gl = {nl[0], nl[1]}, gr = {nr[0], nr[1]}, gu = {nu[0], nu[1]}, gd = {nd[0], nd[1]};
        if (k - lane + 128 < total) {
#pragma unroll
            for (int u = 0; u < 2; u++) {
                locate(min(k + 128 + 64 * u, total - 1), nxi[u], nyi[u]);
                if (!(kAblate & 8)) fetch(nxi[u], nyi[u], nl[u], nr[u], nu[u], nd[u]);
            }
        }
        const f2v fx = {(float)xi[0], (float)xi[1]}, fy = {(float)yi[0], (float)yi[1]};
        const f2v cs = {cos_s, cos_s}, sn = {sin_s, sin_s};
        const f2v col_rot = fx * cs - fy * sn;
        const f2v row_rot = fx * sn + fy * cs;
        f2v row_bin = row_rot + (float)(kDescHist / 2);
        f2v col_bin = col_rot + (float)(kDescHist / 2);
        bool inside[2];
#pragma unroll
        for (int u = 0; u < 2; u++)
            inside[u] = k + 64 * u < total && row_bin[u] > -0.5f && row_bin[u] < (float)kDescHist + 0.5f &&
                        col_bin[u] > -0.5f && col_bin[u] < (float)kDescHist + 0.5f;
        f2v dx, dy;
        if (kAblate & 8) {
            dx = fx * 0.01f + 0.001f;
            dy = fy * 0.01f - 0.002f;
        } else {
            dx = gr - gl;
            dy = gu - gd;
        }
        const f2v wsq = col_rot * col_rot + row_rot * row_rot;
        f2v weight;
        if (kAblate & 4) {
            weight = wsq * (-0.125f) + 1.0f;
        } else {
            const f2v e2 = wsq * (-2.f / (float)(kDescHist * kDescHist)) * 1.44269504088896341f;
            weight = f2v{__builtin_amdgcn_exp2f(e2.x), __builtin_amdgcn_exp2f(e2.y)};
        }
        f2v degf = (kAblate & 2) ? dy * 50.0f + dx : atan2_deg2(dy, dx);
        // (float)(((double)v + 360) % 360) == (v < 0 ? v + 360.0f : v): the f64
        // sum is exact and rounded once either way
#pragma unroll
        for (int u = 0; u < 2; u++) degf[u] = degf[u] < 0.0f ? degf[u] + 360.0f : degf[u];
        const f2v ori = degf - orientation;
        f2v mag = dx * dx + dy * dy;
        mag = f2v{__builtin_amdgcn_sqrtf(mag.x), __builtin_amdgcn_sqrtf(mag.y)};
        row_bin = row_bin - 0.5f;
        col_bin = col_bin - 0.5f;
        mag = mag * weight;
        const f2v obin = ori * BIN_ANGLE_STEP;
        const f2v row_floor = __builtin_elementwise_floor(row_bin), col_floor = __builtin_elementwise_floor(col_bin);
        const f2v ori_floor = __builtin_elementwise_floor(obin);
        const f2v row_frac = row_bin - row_floor, col_frac = col_bin - col_floor, ori_frac = obin - ori_floor;
        const f2v c1 = mag * row_frac, c0 = mag - c1;
        const f2v c11 = c1 * col_frac, c10 = c1 - c11;
        const f2v c01 = c0 * col_frac, c00 = c0 - c01;
        const f2v c111 = c11 * ori_frac, c110 = c11 - c111;
        const f2v c101 = c10 * ori_frac, c100 = c10 - c101;
        const f2v c011 = c01 * ori_frac, c010 = c01 - c011;
        const f2v c001 = c00 * ori_frac, c000 = c00 - c001;
        int a[2][4];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int r1 = (int)row_floor[u] + 1, q1 = (int)col_floor[u] + 1;  // 0..4
            int o0 = (int)ori_floor[u];
            o0 = o0 < 0 ? o0 + kDescBins : (o0 >= kDescBins ? o0 - kDescBins : o0);
            o0 &= kDescBins - 1;
            // slot pair of each footprint corner: (cell, o0 / o0 + 1) of an interior
            // cell, or the corner's own dummy pair (144 + 2 * corner) on the border ring
            const bool rv1 = (uint32_t)(r1 - 1) < 4u, rv2 = (uint32_t)r1 < 4u;  // rows r1, r1 + 1 interior
            const bool qv1 = (uint32_t)(q1 - 1) < 4u, qv2 = (uint32_t)q1 < 4u;
            const int base = ((r1 - 1) * 4 + (q1 - 1)) * 9 + o0;  // o0 + 1 <= 8: no wrap
            a[u][0] = ((rv1 && qv1) ? base : 144) * NS;
            a[u][1] = ((rv1 && qv2) ? base + 9 : 146) * NS;
            a[u][2] = ((rv2 && qv1) ? base + 36 : 148) * NS;
            a[u][3] = ((rv2 && qv2) ? base + 45 : 150) * NS;
        }
        const f2v w[2][4] = {{f2v{c000.x, c001.x}, f2v{c010.x, c011.x}, f2v{c100.x, c101.x}, f2v{c110.x, c111.x}},
                             {f2v{c000.y, c001.y}, f2v{c010.y, c011.y}, f2v{c100.y, c101.y}, f2v{c110.y, c111.y}}};
        if (kAblate & 1) {
#pragma unroll
            for (int u = 0; u < 2; u++)
                if (inside[u])
                    sink += (w[u][0] + w[u][1]) * (w[u][2] + w[u][3]) +
                            f2v{(float)a[u][0], (float)(a[u][1] + a[u][2] + a[u][3])};
            continue;
        }
#pragma unroll
        for (int g = 0; g < kShare; g++) {
#pragma unroll
            for (int u = 0; u < 2; u++) {
                if (!(inside[u] && grp == g)) continue;
                // 4 distinct slot pairs: all reads, then all writes
                f2v h[4];
#pragma unroll
                for (int j = 0; j < 4; j++) h[j] = f2v{hp[a[u][j]], hp[a[u][j] + NS]};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const f2v sum = h[j] + w[u][j];
                    hp[a[u][j]] = sum.x;
                    hp[a[u][j] + NS] = sum.y;
                }
            }
        }
    }
    mid();
    wave_sync();
    // per-bin sum of the 64 private slices: lane l owns flat bins 2l, 2l+1 and
    // starts at slice l (rotated start: the 32 lanes of a half hit 32 banks)
    float acc0 = 0.0f, acc1 = 0.0f;
    const int fb = (lane >> 2) * 9 + 2 * (lane & 3);  // slot of flat bin 2 * lane
    const float* r0 = sc.h + fb * NS;
    const float* r1 = r0 + NS;
    const float* r8 = sc.h + ((lane >> 2) * 9 + 8) * NS;  // orientation-0 alias of the cell
    float acc8 = 0.0f;
    if constexpr (NS % 4 == 0) {
        // four slices per 16-byte read; the start rotates with the lane, so
        // each 8-lane group of a read touches 8 distinct 4-bank groups
#pragma unroll
        for (int j = 0; j < NS / 4; j++) {
            const int jj = 4 * ((j + lane) & (NS / 4 - 1));
            const float4 a = *reinterpret_cast<const float4*>(r0 + jj);
            const float4 b = *reinterpret_cast<const float4*>(r1 + jj);
            const float4 c = *reinterpret_cast<const float4*>(r8 + jj);
            acc0 += a.x;
            acc0 += a.y;
            acc0 += a.z;
            acc0 += a.w;
            acc1 += b.x;
            acc1 += b.y;
            acc1 += b.z;
            acc1 += b.w;
            acc8 += c.x;
            acc8 += c.y;
            acc8 += c.z;
            acc8 += c.w;
        }
    } else {
#pragma unroll 8
        for (int j = 0; j < NS; j++) {
            const int jj = (j + lane) & (NS - 1);
            acc0 += r0[jj];
            acc1 += r1[jj];
            acc8 += r8[jj];
        }
    }
    if ((lane & 3) == 0) acc0 += acc8;
    if (kAblate & 1) acc0 += sink.x + sink.y;
    describe_normalize<true>(acc0, acc1, out, lane);
}

// kMode 0: bit-exact (describe_wave_exact); 1 / 2 / 4: fast path with that
// slice-sharing factor.
// 4 waves per SIMD (<= 128 VGPRs, no spills): the 16 waves per CU the LDS
// footprint allows (141 VGPRs unconstrained = 12 waves; the stage is ~4% faster)
#ifndef SIFT_DESC_WPE
#define SIFT_DESC_WPE 4
#endif
template <int kMode, int kAblate>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kMode == 0 ? 1 : SIFT_DESC_WPE))) void k_describe(const DescLaunch L) {
    constexpr bool kExact = kMode == 0;
    using Scratch = typename std::conditional<kExact, DescScratch, DescScratchFast<kExact ? 1 : kMode>>::type;
    __shared__ __attribute__((aligned(16))) Scratch scr;
    const int lane = threadIdx.x;
    const uint32_t n = min(*L.n, L.bound);
    // one wave per keypoint, taken from a work counter: window sizes (and
    // costs) vary ~20x, a static stride would leave a long tail
    // Keypoints come from kDescQueues interleaved queues (queue q holds
    // keypoints q, q + 8, ...; one wave per keypoint, window costs vary ~20x):
    // a wave drains its home queue (blockIdx % 8, the XCD the block runs on),
    // then the others in turn.
    // The next keypoint is claimed while the current one is processed, and its
    // record is loaded between the current sample loop and its reduction, so
    // neither the queue atomic nor the record load stalls the wave.
    int q = blockIdx.x & (kDescQueues - 1), drained = 0;
    uint32_t pend = 0;
    auto issue = [&]() {
        if (lane == 0) pend = atomicAdd(L.work + q * kDescQueueStride, 1u);
    };
    auto take = [&]() -> uint32_t {  // resolves the claim in flight: keypoint index, or n when all queues are empty
        for (;;) {
            const uint32_t j = __builtin_amdgcn_readfirstlane(__shfl(pend, 0));
            const uint32_t i = j * kDescQueues + q;
            if (i < n) return __builtin_amdgcn_readfirstlane(i);
            if (++drained == kDescQueues) return n;
            q = (q + 1) & (kDescQueues - 1);
            issue();
        }
    };
    auto record = [&](uint32_t i) {
        KpRec r{};
        if (i < n) r = L.kp[L.idx ? L.idx[i] : i];
        return r;
    };
    issue();
    uint32_t i = take();
    KpRec kp = record(i);
    uint32_t nsamp = 0;  // samples enumerated by this wave (sample counting)
    while (i < n) {
        if (drained < kDescQueues) issue();
        const int o = __builtin_amdgcn_readfirstlane(kp.octave);
        const int W = L.ow[o], H = L.oh[o];
        const int pitch = L.opitch[o];
        const float* img = L.gauss[o] + (size_t)(__builtin_amdgcn_readfirstlane(kp.img) - L.img_base) *
                                            L.gauss_img_stride[o] +
                           (size_t)__builtin_amdgcn_readfirstlane(kp.scale) * pitch * H;
        // compute_descriptors (src/lib.rs:759-782)
        const float angle = 360.0f - kp.angle;  // orientation (src/lib.rs:771); kp.sin_d / cos_d its rotation
        const float osf = 1.0f / (float)(1u << o);  // 2_f32.powi(-octave)
        const float kp_size = kp.size * osf;
        uint8_t* out = L.out_desc + (size_t)i * kDescSize;
        uint32_t ni = n;
        KpRec nkp{};
        auto next = [&]() {
            ni = drained < kDescQueues ? take() : n;
            nkp = record(ni);
        };
        if constexpr (kExact) {
            describe_wave_exact<kAblate>(img, pitch, W, H, kp.x * osf, kp.y * osf, kp_size, angle, kp.sin_d, kp.cos_d,
                                         scr, out, lane);
            next();
        } else {
            describe_wave_fast<kExact ? 1 : kMode, kAblate>(img, pitch, W, H, kp.x * osf, kp.y * osf, kp_size, angle,
                                                            kp.sin_d, kp.cos_d, scr, out, lane, next,
                                                            L.samples ? &nsamp : nullptr);
        }
        if (lane == 0) {
            if (L.out_kp) {
                OutKp k;
                k.x = kp.x * 0.5f;  // DELTA_MIN (src/lib.rs:163-176)
                k.y = kp.y * 0.5f;
                k.size = kp.size * 0.5f;
                k.angle = kp.angle;
                k.response = kp.response;
                L.out_kp[i] = k;
            }
            if (L.out_key) L.out_key[i] = kp.key + L.key_base;
        }
        wave_sync();  // the scratch is reused by the next keypoint
        i = ni;
        kp = nkp;
    }
    if (L.samples && lane == 0 && nsamp) atomicAdd(L.samples + (blockIdx.x & 7), (unsigned long long)nsamp);
}

void launch_describe(const DescLaunch& L, hipStream_t st) {
    if (L.bound == 0) return;
    // fast path at kShare 4: ~10 KB of LDS per wave -> 16 resident per CU (exact: 14 KB)
#ifndef SIFT_DESC_SHARE
#define SIFT_DESC_SHARE 4  // lanes per private histogram slice: 9.7 KB of LDS per wave (bench: 4 beats 2 and 8)
#endif
#ifndef SIFT_DESC_WAVES_PER_CU
#define SIFT_DESC_WAVES_PER_CU 16
#endif
    const dim3 grid(std::min<uint32_t>(L.bound, 256 * SIFT_DESC_WAVES_PER_CU));
    if (L.exact)
        hipLaunchKernelGGL((k_describe<0, 0>), grid, dim3(64), 0, st, L);
    else
        hipLaunchKernelGGL((k_describe<SIFT_DESC_SHARE, 0>), grid, dim3(64), 0, st, L);
}

__global__ __launch_bounds__(64) void k_describe_one(const float* img, int w, int h, float x, float y, float scale,
                                                     float orientation, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) DescScratch scr;
    float sn, cs;
    orientation_rotation(orientation, sn, cs);
    describe_wave_exact(img, w, w, h, x, y, scale, orientation, sn, cs, scr, out, threadIdx.x);
}

void launch_describe_one(const float* img, int w, int h, float x, float y, float scale, float orientation,
                         uint8_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_describe_one, dim3(1), dim3(64), 0, st, img, w, h, x, y, scale, orientation, out);
}

}  // namespace siftmi
