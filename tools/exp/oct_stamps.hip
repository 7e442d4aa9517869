// Diagnostic: per-phase cycle shares of k_octave's waves (level row filter,
// column filter, stores, barrier wait; loader wait / issue / barrier) on an
// octave-0-sized batch.  Build + run (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSIFT_OCT_STAMPS \
//         tools/exp/oct_stamps.hip -o tools/exp/oct_stamps && tools/exp/oct_stamps [W H n]
#include "octave.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace siftmi;

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));       \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

__global__ void k_fill(float* p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint32_t h = (uint32_t)i * 2654435761u;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = (float)(h & 0xffff) / 65536.0f;
    }
}

int main(int argc, char** argv) {
    const int W = argc > 1 ? atoi(argv[1]) : 3840, H = argc > 2 ? atoi(argv[2]) : 2160;
    const int n = argc > 3 ? atoi(argv[3]) : 16;
    const int pitch = (W + 63) & ~63;
    const size_t plane = (size_t)pitch * H;
    float *g, *d;
    CK(hipMalloc(&g, plane * 6 * n * 4));
    CK(hipMalloc(&d, plane * 5 * n * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, g, plane * 6 * n);
    OctaveArgs a{};
    a.gauss = g;
    a.g_img_stride = plane * 6;
    a.plane = plane;
    a.dog = d;
    a.dog_img_stride = plane * 5;
    a.W = W;
    a.H = H;
    a.pitch = pitch;
    a.seg_rows = H;
    for (int s = 1; s <= 5; s++)
        for (int t = 0; t <= oct::kR[s]; t++) a.taps[s].k[t] = 1.0f / (2 * oct::kR[s] + 1);
    launch_octave(a, n, 0);
    CK(hipDeviceSynchronize());
#ifdef SIFT_OCT_STAMPS
    unsigned long long z[6][5] = {};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(oct::g_oct_stamps), z, sizeof(z)));
#endif
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = argc > 4 ? atoi(argv[4]) : 1;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; i++) launch_octave(a, n, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
#ifndef SIFT_OCT_STAMPS
    std::printf("k_octave %dx%d x %d: %.3f ms per launch (%d reps)\n", W, H, n, ms, reps);
    return 0;
#else
    unsigned long long st[6][5];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(oct::g_oct_stamps), sizeof(st)));
    std::printf("k_octave %dx%d x %d (stamped build): %.3f ms\n", W, H, n, ms);
    const char* ph[2][4] = {{"vmwait", "issue", "-", "barrier"}, {"rowfilt", "colfilt", "stores", "barrier"}};
    for (int l = 0; l <= 5; l++) {
        const double tot = (double)(st[l][0] + st[l][1] + st[l][2] + st[l][3]);
        std::printf("%s %d  waves=%llu  cycles/wave=%.0f ", l ? "level" : "loader", l, st[l][4],
                    tot / (double)(st[l][4] ? st[l][4] : 1));
        for (int q = 0; q < 4; q++) std::printf(" %s=%.1f%%", ph[l ? 1 : 0][q], 100.0 * st[l][q] / (tot > 0 ? tot : 1));
        std::printf("\n");
    }
    return 0;
#endif
}
