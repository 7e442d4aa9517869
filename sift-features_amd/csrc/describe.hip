// 4x4x8 SIFT descriptors on MI355X: one wave per keypoint, four keypoints
// per workgroup, the 6x6x8 trilinear histogram kept in the wave's LDS slice.
//
// Reference: compute_descriptors / compute_descriptor (src/lib.rs:759-990).
// Per-sample arithmetic keeps the reference's operand order; the histogram is
// accumulated with LDS float atomics (ds_add_f32), so the order of additions
// into a bin differs from the reference's sequential sample order: bins
// agree to f32 rounding and the final u8 components to +-1 (tolerance stated
// in tests/test_gpu_parity.py).  The L2 norms use the reference's exact
// chunk-of-4 summation order (src/lib.rs:957-976).
#include <float.h>

#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {

constexpr int HIST_FLOATS = 6 * 6 * kDescBins;  // 288

// Per-wave LDS scratch: 288 histogram bins + the row table of the sample
// enumeration (first column, prefix count) for up to 2*38+1 = 77 rows.
constexpr int ROWS_MAX = 80;
struct DescScratch {
    float hist[HIST_FLOATS];
    int rowlo[ROWS_MAX];
    int rowpre[ROWS_MAX + 1];
};

// Wave-cooperative compute_descriptor (src/lib.rs:785-990).
//
// Only samples whose rotated coordinates fall in the 4x4 histogram region
// (|col_rot|, |row_rot| < 2.5 bin units, about half of the (2r+1)^2 window)
// contribute; each row's candidate column interval is computed in f64 and
// widened by one sample, the compacted (row, col) list is strided over the
// wave's lanes, and the reference's exact f32 predicate is still evaluated
// per sample -- so the accepted set is identical to the reference's.
__device__ __forceinline__ void describe_wave(const float* __restrict__ img, int pitch, int width, int height,
                                              float xf, float yf, float scale, float orientation,
                                              DescScratch& sc, uint8_t* __restrict__ out, int lane) {
    for (int i = lane; i < HIST_FLOATS; i += 64) sc.hist[i] = 0.0f;
    const int32_t x = (int32_t)sat_u32(roundf(xf));
    const int32_t y = (int32_t)sat_u32(roundf(yf));
    const float BIN_ANGLE_STEP = (float)kDescBins / 360.0f;
    const float hist_width = kLambdaDescr * scale;
    int radius = sat_i32(roundf(kLambdaDescr * scale * 1.41421356237309504880f * (float)(kDescHist + 1) * 0.5f));
    radius = radius < 0 ? 0 : (radius > (ROWS_MAX - 2) / 2 ? (ROWS_MAX - 2) / 2 : radius);
    const float rad = orientation * (3.14159265358979323846f / 180.0f);  // f32::to_radians
    const float sin_ori = (float)sin((double)rad), cos_ori = (float)cos((double)rad);
    const float sin_s = sin_ori / hist_width, cos_s = cos_ori / hist_width;
    const int n = 2 * radius + 1;
    // 1. per-row candidate column interval
    for (int row = lane; row < n; row += 64) {
        const double yi = (double)(row - radius);
        const double c = cos_s, s = sin_s;
        double lo = -radius, hi = radius;
        bool empty = false;
        if (fabs(c) > 1e-30) {
            const double a = (yi * s - 2.5) / c, b = (yi * s + 2.5) / c;
            lo = fmax(lo, fmin(a, b) - 1.0);
            hi = fmin(hi, fmax(a, b) + 1.0);
        } else {
            empty = !(fabs(yi * s) < 2.5 + 1e-3);
        }
        if (fabs(s) > 1e-30) {
            const double a = (-yi * c - 2.5) / s, b = (-yi * c + 2.5) / s;
            lo = fmax(lo, fmin(a, b) - 1.0);
            hi = fmin(hi, fmax(a, b) + 1.0);
        } else {
            empty = empty || !(fabs(yi * c) < 2.5 + 1e-3);
        }
        const int ilo = (int)floor(lo), ihi = (int)ceil(hi);
        sc.rowlo[row] = ilo;
        sc.rowpre[row + 1] = (empty || ihi < ilo) ? 0 : ihi - ilo + 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
        int acc = 0;
        sc.rowpre[0] = 0;
        for (int r = 1; r <= n; r++) {
            acc += sc.rowpre[r];
            sc.rowpre[r] = acc;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int total = sc.rowpre[n];
    // 2. lane-chunked walk over the compacted samples: lane l takes samples
    // [l*chunk, (l+1)*chunk), so at any step the 64 lanes sit ~chunk samples
    // apart across the window and their histogram cells rarely coincide
    // (a strided walk puts neighbouring lanes on the same cell and serialises
    // the LDS atomics)
    const int chunk = (total + 63) >> 6;
    int k = lane * chunk;
    const int kend = min(total, k + chunk);
    int row = 0;
    {
        int lo = 0, hi = n;  // first row with rowpre[row + 1] > k
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sc.rowpre[mid + 1] <= k)
                lo = mid + 1;
            else
                hi = mid;
        }
        row = lo;
    }
    for (; k < kend; k++) {
        while (sc.rowpre[row + 1] <= k) row++;
        const int yi = row - radius;
        const int xi = sc.rowlo[row] + (k - sc.rowpre[row]);
        const float col_rot = (float)xi * cos_s - (float)yi * sin_s;
        const float row_rot = (float)xi * sin_s + (float)yi * cos_s;
        float row_bin = row_rot + (float)(kDescHist / 2);
        float col_bin = col_rot + (float)(kDescHist / 2);
        const int32_t ay = y + yi, ax = x + xi;
        if (!(row_bin > -0.5f && row_bin < (float)kDescHist + 0.5f && col_bin > -0.5f &&
              col_bin < (float)kDescHist + 0.5f && ay > 0 && ay < height - 1 && ax > 0 && ax < width - 1))
            continue;
        const float* rw = img + (size_t)ay * pitch;
        const float dx = rw[ax + 1] - rw[ax - 1];
        const float dy = rw[ax - pitch] - rw[ax + pitch];
        const float wsq = col_rot * col_rot + row_rot * row_rot;
        const float weight = exp_f32(wsq * (-2.f / (float)(kDescHist * kDescHist)));
        // ((atan2(dy, dx).to_degrees() + 360) % 360) as f32 - orientation; the
        // f64 remainder of v in [180, 540] by 360 is exactly v or v - 360
        double deg = atan2((double)dy, (double)dx) * (180.0 / 3.14159265358979323846) + 360.0;
        deg = deg >= 360.0 ? deg - 360.0 : deg;
        const float ori = (float)deg - orientation;
        float mag = sqrtf(dx * dx + dy * dy);
        row_bin = row_bin - 0.5f;
        col_bin = col_bin - 0.5f;
        mag = mag * weight;
        const float obin = ori * BIN_ANGLE_STEP;
        const float row_floor = floorf(row_bin), col_floor = floorf(col_bin), ori_floor = floorf(obin);
        const float row_frac = row_bin - row_floor, col_frac = col_bin - col_floor, ori_frac = obin - ori_floor;
        const float c1 = mag * row_frac, c0 = mag - c1;
        const float c11 = c1 * col_frac, c10 = c1 - c11;
        const float c01 = c0 * col_frac, c00 = c0 - c01;
        const float c111 = c11 * ori_frac, c110 = c11 - c111;
        const float c101 = c10 * ori_frac, c100 = c10 - c101;
        const float c011 = c01 * ori_frac, c010 = c01 - c011;
        const float c001 = c00 * ori_frac, c000 = c00 - c001;
        // row_floor in [-1, 3], col_floor in [-1, 3] inside the accepted region;
        // ori_floor in [-8, 7] for orientation in [0, 360] (host-checked)
        const int r1 = (int)row_floor + 1, q1 = (int)col_floor + 1;
        int o0 = (int)ori_floor;
        o0 = o0 < 0 ? o0 + kDescBins : (o0 >= kDescBins ? o0 - kDescBins : o0);
        if ((unsigned)r1 > 4u || (unsigned)q1 > 4u || (unsigned)o0 >= (unsigned)kDescBins) continue;
        const int o1 = o0 + 1 >= kDescBins ? 0 : o0 + 1;
        float* h11 = sc.hist + (r1 * 6 + q1) * kDescBins;
        float* h12 = h11 + kDescBins;
        float* h21 = h11 + 6 * kDescBins;
        float* h22 = h21 + kDescBins;
        atomicAdd(h11 + o0, c000);
        atomicAdd(h11 + o1, c001);
        atomicAdd(h12 + o0, c010);
        atomicAdd(h12 + o1, c011);
        atomicAdd(h21 + o0, c100);
        atomicAdd(h21 + o1, c101);
        atomicAdd(h22 + o0, c110);
        atomicAdd(h22 + o1, c111);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // lane l < 32 owns flat components 4l..4l+3 (= reference chunk l)
    float v[4];
    const int l = lane & 31;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int i = 4 * l + j;
        const int rr = 1 + (i >> 5), cc = 1 + ((i >> 3) & 3), oo = i & 7;
        v[j] = sc.hist[(rr * 6 + cc) * kDescBins + oo];
    }
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; j++) s += v[j] * v[j];
    float l2 = __shfl(s, 0);
    for (int c = 1; c < 32; c++) l2 = l2 + __shfl(s, c);
    l2 = sqrtf(l2);
    const float cap = l2 * 0.2f;
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = fminf(v[j], cap);
    s = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; j++) s += v[j] * v[j];
    float l2c = __shfl(s, 0);
    for (int c = 1; c < 32; c++) l2c = l2c + __shfl(s, c);
    l2c = sqrtf(l2c);
    const float norm = 512.0f / fmaxf(l2c, FLT_EPSILON);
    if (lane < 32) {
        uint32_t packed = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int32_t q = sat_i32(roundf(v[j] * norm));
            const uint32_t u = q > 255 ? 255u : (uint32_t)(uint8_t)q;
            packed |= u << (8 * j);
        }
        reinterpret_cast<uint32_t*>(out)[lane] = packed;
    }
}

__global__ __launch_bounds__(256) void k_describe(const DescLaunch L) {
    __shared__ DescScratch scr[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * 4 + wave;
    if (i >= L.n) return;  // whole wave; no workgroup barrier below
    const KpRec kp = L.kp[L.idx ? L.idx[i] : i];
    const int o = kp.octave;
    const int W = L.ow[o], H = L.oh[o];
    const int pitch = L.opitch[o];
    const float* img =
        L.gauss[o] + (size_t)(kp.img - L.img_base) * L.gauss_img_stride[o] + (size_t)kp.scale * pitch * H;
    // compute_descriptors (src/lib.rs:759-782)
    const float angle = 360.0f - kp.angle;
    const float osf = 1.0f / (float)(1u << o);  // 2_f32.powi(-octave)
    const float kp_size = kp.size * osf;
    describe_wave(img, pitch, W, H, kp.x * osf, kp.y * osf, kp_size, angle, scr[wave],
                  L.out_desc + (size_t)i * kDescSize, lane);
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
        if (L.out_key) L.out_key[i] = kp.key;
    }
}

void launch_describe(const DescLaunch& L, hipStream_t st) {
    if (L.n == 0) return;
    dim3 grid((L.n + 3) / 4);
    hipLaunchKernelGGL(k_describe, grid, dim3(256), 0, st, L);
}

__global__ __launch_bounds__(64) void k_describe_one(const float* img, int w, int h, float x, float y, float scale,
                                                     float orientation, uint8_t* out) {
    __shared__ DescScratch scr;
    describe_wave(img, w, w, h, x, y, scale, orientation, scr, out, threadIdx.x);
}

void launch_describe_one(const float* img, int w, int h, float x, float y, float scale, float orientation,
                         uint8_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_describe_one, dim3(1), dim3(64), 0, st, img, w, h, x, y, scale, orientation, out);
}

}  // namespace siftmi
