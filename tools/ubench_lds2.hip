// LDS accumulation micro-benchmark, conflict-free layout (performance
// experiments only): bin-major / slice-minor h[bin * 64 + slice] as in
// describe.hip.  Cost per wave of one scatter round (8 bin updates per lane)
// for: ds_add_f32 lane-private (64 slices), plain read-add-write lane-private,
// ds_add_f32 with 16 / 4 shared slices, and the product's exec-masked
// read-add-write (16 slices, 4 groups of 16 lanes).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

constexpr int ITERS = 1024;
constexpr int NB = 152;

template <int MODE>
__global__ __launch_bounds__(64) void k_lds2(float* out, int seed) {
    __shared__ float h[NB * 64];
    const int lane = threadIdx.x;
    for (int i = lane; i < NB * 64; i += 64) h[i] = 0.f;
    __builtin_amdgcn_wave_barrier();
    uint32_t r = seed * 2654435761u + lane * 40503u;
    const float v = 1.0f + lane;
    for (int it = 0; it < ITERS; it++) {
        int b[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            r = r * 1664525u + 1013904223u;
            b[j] = (int)((r >> 16) % NB);
        }
        if (MODE == 0 || MODE == 2 || MODE == 3) {
            const int NS = MODE == 0 ? 64 : (MODE == 2 ? 16 : 4);
#pragma unroll
            for (int j = 0; j < 8; j++) atomicAdd(&h[b[j] * 64 + (lane & (NS - 1))], v);
        } else if (MODE == 1) {
            float t[8];
#pragma unroll
            for (int j = 0; j < 8; j++) t[j] = h[b[j] * 64 + lane];
#pragma unroll
            for (int j = 0; j < 8; j++) h[b[j] * 64 + lane] = t[j] + v;  // (distinct bins not enforced: timing only)
        } else {  // exec-masked groups of 16 lanes, 16 slices
#pragma unroll
            for (int g = 0; g < 4; g++) {
                if ((lane >> 4) == g) {
                    float t[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) t[j] = h[b[j] * 64 + (lane & 15)];
#pragma unroll
                    for (int j = 0; j < 8; j++) h[b[j] * 64 + (lane & 15)] = t[j] + v;
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    out[blockIdx.x * 64 + lane] = h[lane] + h[64 * 100 + lane];
}

template <int MODE>
void run(const char* name, float* d, int blocks) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_lds2<MODE>, dim3(blocks), dim3(64), 0, 0, d, 1);
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_lds2<MODE>, dim3(blocks), dim3(64), 0, 0, d, 2);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double cyc = ms * 1e-3 * 2.4e9 / ((double)blocks / 256 * ITERS);
    std::printf("  %-40s %8.3f ms  ~%.1f CU-cycles per wave-round (8 updates / lane)\n", name, ms, cyc);
}

int main() {
    float* d;
    const int blocks = 256 * 8;  // 8 waves per CU (38 KB LDS each: 4 fit per CU at a time)
    CK(hipMalloc(&d, (size_t)blocks * 64 * sizeof(float)));
    std::printf("LDS scatter, %d single-wave blocks x %d rounds\n", blocks, ITERS);
    run<0>("ds_add_f32, 64 private slices", d, blocks);
    run<1>("read-add-write, 64 private slices", d, blocks);
    run<2>("ds_add_f32, 16 shared slices", d, blocks);
    run<3>("ds_add_f32, 4 shared slices", d, blocks);
    run<4>("masked read-add-write, 16 slices x 4 groups", d, blocks);
    CK(hipFree(d));
    return 0;
}
