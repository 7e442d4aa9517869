// Brute-force descriptor matching on the MFMA units (SURVEY.md 8(f) row 3:
// the step after the path).
//
// Reference: examples/sift-match.rs:30-35 matches two SiftResults with
// cv::BFMatcher(NORM_L2, crossCheck = true).match(query, train):
//   * distance = sqrt((float) sum (q_k - t_k)^2), the integer sum exact
//     (batchDistL2_8u32f);
//   * each query's nearest train row, lowest index on ties (strict <);
//   * cross check keeps query i only if its nearest train row's nearest query
//     is i (cv::batchDistance crosscheck); matches come out in query order.
//
// Dot products run as bf16 MFMA (mfma_f32_32x32x16_bf16): u8 values are exact
// in bf16 and every partial sum (< 128 * 255^2 < 2^24) is an exact f32
// integer, so d^2 = |q|^2 + |t|^2 - 2 q.t is the exact integer.  A 256-thread
// workgroup owns a 128 x 128 (query x train) tile, each wave 64 x 64 (2 x 2
// MFMA tiles, 8 k-steps); the tile's row / column minima are folded into
// global per-query and per-train (d^2 << 32 | index) keys with 64-bit
// atomicMin, which also gives the lowest-index tie break.
#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ short u8_to_bf16(uint32_t v) {
    return (short)(__float_as_uint((float)v) >> 16);  // exact for 0..255
}

// 8 consecutive u8 of one descriptor row -> bf16 MFMA fragment
__device__ __forceinline__ bf16x8 load_frag(const uint8_t* __restrict__ base, int row, int n, int k0) {
    bf16x8 f;
    if (row < n) {
        const uint2 w = *reinterpret_cast<const uint2*>(base + (size_t)row * kDescSize + k0);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            f[j] = u8_to_bf16((w.x >> (8 * j)) & 0xff);
            f[4 + j] = u8_to_bf16((w.y >> (8 * j)) & 0xff);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) f[j] = 0;
    }
    return f;
}

__global__ __launch_bounds__(256) void k_match_norms(const uint8_t* __restrict__ d, int n, float* __restrict__ nrm) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(d + (size_t)i * kDescSize);
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < kDescSize / 16; c++) {
        const uint4 w = p[c];
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t b = (ws[q] >> (8 * j)) & 0xff;
                s += b * b;
            }
    }
    nrm[i] = (float)s;  // < 2^24: exact
}

__device__ __forceinline__ uint64_t min_u64(uint64_t a, uint64_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)v, m), hi = __shfl_xor((uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(256) void k_match_tiles(const uint8_t* __restrict__ q, int nq,
                                                     const uint8_t* __restrict__ t, int nt,
                                                     const float* __restrict__ qn, const float* __restrict__ tn,
                                                     unsigned long long* __restrict__ row_best,
                                                     unsigned long long* __restrict__ col_best) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int q0 = blockIdx.x * 128 + (wave >> 1) * 64;  // this wave's 64 query rows
    const int t0 = blockIdx.y * 128 + (wave & 1) * 64;   // and 64 train rows
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int e = 0; e < 16; e++) acc[a][b][e] = 0.0f;
#pragma unroll
    for (int s = 0; s < kDescSize / 16; s++) {
        const int k0 = 16 * s + 8 * h;
        bf16x8 fa[2], fb[2];
#pragma unroll
        for (int a = 0; a < 2; a++) fa[a] = load_frag(q, q0 + 32 * a + r, nq, k0);
#pragma unroll
        for (int b = 0; b < 2; b++) fb[b] = load_frag(t, t0 + 32 * b + r, nt, k0);
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
                acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
    }
    // C/D: column (train) = lane & 31, row (query) = (e & 3) + 8 * (e >> 2) + 4 * h
    const uint64_t INF = ~0ull;
    float tnorm[2];
    int tc[2];
#pragma unroll
    for (int b = 0; b < 2; b++) {
        tc[b] = t0 + 32 * b + r;
        tnorm[b] = tc[b] < nt ? tn[tc[b]] : 0.0f;
    }
    uint64_t colmin[2] = {INF, INF};
#pragma unroll
    for (int a = 0; a < 2; a++) {
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const int qr = q0 + 32 * a + (e & 3) + 8 * (e >> 2) + 4 * h;
            const float qnv = qr < nq ? qn[qr] : 0.0f;
            uint64_t rowkey = INF;
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const float d2 = qnv + tnorm[b] - 2.0f * acc[a][b][e];  // exact integer
                const bool valid = qr < nq && tc[b] < nt;
                const uint32_t di = (uint32_t)d2;
                const uint64_t kr = valid ? ((uint64_t)di << 32) | (uint32_t)tc[b] : INF;
                const uint64_t kc = valid ? ((uint64_t)di << 32) | (uint32_t)qr : INF;
                rowkey = min_u64(rowkey, kr);
                colmin[b] = min_u64(colmin[b], kc);
            }
            // row minimum over the 32 train columns of this lane half
#pragma unroll
            for (int m = 16; m >= 1; m >>= 1) rowkey = min_u64(rowkey, shfl_xor_u64(rowkey, m));
            if (r == 0 && rowkey != INF) atomicMin(&row_best[qr], (unsigned long long)rowkey);
        }
    }
    // column minimum over both lane halves
#pragma unroll
    for (int b = 0; b < 2; b++) {
        const uint64_t k = min_u64(colmin[b], shfl_xor_u64(colmin[b], 32));
        if (h == 0 && k != INF) atomicMin(&col_best[tc[b]], (unsigned long long)k);
    }
}

__global__ __launch_bounds__(256) void k_match_final(const unsigned long long* __restrict__ row_best,
                                                     const unsigned long long* __restrict__ col_best, int nq,
                                                     int cross_check, int* __restrict__ train_idx,
                                                     float* __restrict__ dist) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nq) return;
    const uint64_t rb = row_best[i];
    int tix = -1;
    float d = 0.0f;
    if (rb != ~0ull) {
        const int tt = (int)(uint32_t)rb;
        if (!cross_check || (int)(uint32_t)col_best[tt] == i) {
            tix = tt;
            d = sqrtf((float)(uint32_t)(rb >> 32));  // batchDistL2_8u32f: sqrt((float) int)
        }
    }
    train_idx[i] = tix;
    dist[i] = d;
}

void launch_match(const uint8_t* q, int nq, const uint8_t* t, int nt, int cross_check, float* qn, float* tn,
                  unsigned long long* row_best, unsigned long long* col_best, int* train_idx, float* dist,
                  hipStream_t st) {
    if (nq <= 0) return;
    (void)hipMemsetAsync(row_best, 0xff, (size_t)nq * 8, st);
    if (nt > 0) (void)hipMemsetAsync(col_best, 0xff, (size_t)nt * 8, st);
    hipLaunchKernelGGL(k_match_norms, dim3((nq + 255) / 256), dim3(256), 0, st, q, nq, qn);
    if (nt > 0) {
        hipLaunchKernelGGL(k_match_norms, dim3((nt + 255) / 256), dim3(256), 0, st, t, nt, tn);
        hipLaunchKernelGGL(k_match_tiles, dim3((nq + 127) / 128, (nt + 127) / 128), dim3(256), 0, st, q, nq, t, nt, qn,
                           tn, row_best, col_best);
    }
    hipLaunchKernelGGL(k_match_final, dim3((nq + 255) / 256), dim3(256), 0, st, row_best, col_best, nq, cross_check,
                       train_idx, dist);
}

}  // namespace siftmi
