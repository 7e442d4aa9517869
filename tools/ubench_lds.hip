// LDS accumulation micro-benchmark (performance experiments only).
// Measures per-wave-instruction cost of: ds_add_f32 to lane-private
// addresses, plain read-add-write to lane-private addresses, and ds_add_f32
// to pseudo-random addresses among 288 bins.
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

constexpr int ITERS = 4096;

template <int MODE>
__global__ __launch_bounds__(64) void k_lds(float* out, int seed) {
    __shared__ float h[64 * 132];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * 132; i += 64) h[i] = 0.f;
    __builtin_amdgcn_wave_barrier();
    uint32_t r = seed * 2654435761u + lane * 40503u;
    float v = 1.0f + lane;
    for (int it = 0; it < ITERS; it++) {
        r = r * 1664525u + 1013904223u;
        if (MODE == 0) {  // atomic, private slot (padded stride 132)
            atomicAdd(&h[lane * 132 + (r >> 28)], v);
        } else if (MODE == 1) {  // plain RMW, private slot
            float* p = &h[lane * 132 + (r >> 28)];
            *p = *p + v;
        } else if (MODE == 2) {  // atomic, random among 288 bins
            atomicAdd(&h[(r >> 16) % 288], v);
        } else {  // atomic, 8 distinct bins chosen by lane & 7 (8-way conflicts)
            atomicAdd(&h[(lane & 7) * 36 + (r >> 28)], v);
        }
    }
    __builtin_amdgcn_wave_barrier();
    out[blockIdx.x * 64 + lane] = h[lane * 132] + h[lane];
}

template <int MODE>
void run(const char* name, float* d, int blocks) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_lds<MODE>, dim3(blocks), dim3(64), 0, 0, d, 1);
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_lds<MODE>, dim3(blocks), dim3(64), 0, 0, d, 2);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    // waves per CU = blocks / 256; cycles per wave-instruction per CU
    const double cyc = ms * 1e-3 * 2.4e9 / ((double)blocks / 256 * ITERS);
    std::printf("  %-28s %8.3f ms  ~%.1f CU-cycles per wave-op\n", name, ms, cyc);
}

int main() {
    float* d;
    const int blocks = 256 * 8;
    CK(hipMalloc(&d, blocks * 64 * 4));
    std::printf("LDS accumulation, %d single-wave blocks x %d ops\n", blocks, ITERS);
    run<0>("ds_add_f32 private", d, blocks);
    run<1>("read+add+write private", d, blocks);
    run<2>("ds_add_f32 random/288", d, blocks);
    run<3>("ds_add_f32 8-way", d, blocks);
    return 0;
}
