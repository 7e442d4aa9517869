// Kernel micro-benchmarks / ablations on synthetic data (performance
// experiments only; not part of libsift_mi.so).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I sift-features_amd/csrc \
//         tools/ubench_kernels.hip -o tools/ubench_kernels
#include "../sift-features_amd/csrc/describe.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace siftmi;

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

template <bool E, int A>
float time_describe(const DescLaunch& L, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid(L.n);
    hipLaunchKernelGGL((k_describe<E, A>), grid, dim3(64), 0, 0, L);
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL((k_describe<E, A>), grid, dim3(64), 0, 0, L);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int W = 3840, H = 2160, pitch = 3840, NKP = argc > 1 ? atoi(argv[1]) : 200000;
    // one octave image stack (6 planes) with smooth synthetic content
    std::vector<float> img((size_t)6 * pitch * H);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            const float v = 0.5f + 0.25f * sinf(x * 0.07f) * cosf(y * 0.05f) + 0.1f * sinf((x + 2 * y) * 0.31f);
            for (int s = 0; s < 6; s++) img[(size_t)s * pitch * H + (size_t)y * pitch + x] = v;
        }
    std::vector<KpRec> kp(NKP);
    srand(1);
    for (int i = 0; i < NKP; i++) {
        KpRec& k = kp[i];
        k.key = i;
        k.img = 0;
        k.octave = 0;
        k.scale = 1 + (i % 3);
        k.x = 40 + (float)(rand() % (W - 80)) + 0.3f;
        k.y = 40 + (float)(rand() % (H - 80)) + 0.6f;
        k.size = 1.8f + 1.8f * (float)(rand() % 1000) / 1000.f;
        k.angle = 0.5f + (float)(rand() % 3590) / 10.f;
        k.response = 0.1f;
    }
    float* d_img;
    KpRec* d_kp;
    uint8_t* d_desc;
    const float** d_g;
    size_t* d_gs;
    int *d_w, *d_h, *d_p;
    CK(hipMalloc(&d_img, img.size() * 4));
    CK(hipMemcpy(d_img, img.data(), img.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_kp, NKP * sizeof(KpRec)));
    CK(hipMemcpy(d_kp, kp.data(), NKP * sizeof(KpRec), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_desc, (size_t)NKP * 128));
    const float* gp = d_img;
    size_t gs = (size_t)6 * pitch * H;
    CK(hipMalloc(&d_g, sizeof(float*)));
    CK(hipMemcpy(d_g, &gp, sizeof(float*), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_gs, sizeof(size_t)));
    CK(hipMemcpy(d_gs, &gs, sizeof(size_t), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_w, 4));
    CK(hipMalloc(&d_h, 4));
    CK(hipMalloc(&d_p, 4));
    CK(hipMemcpy(d_w, &W, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_h, &H, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_p, &pitch, 4, hipMemcpyHostToDevice));
    DescLaunch L{};
    L.kp = d_kp;
    L.n = NKP;
    L.gauss = d_g;
    L.gauss_img_stride = d_gs;
    L.ow = d_w;
    L.oh = d_h;
    L.opitch = d_p;
    L.out_desc = d_desc;
    const int reps = 5;
    std::printf("describe n=%d\n", NKP);
    std::printf("  exact           %8.3f ms\n", time_describe<true, 0>(L, reps));
    std::printf("  exact -phaseB   %8.3f ms\n", time_describe<true, 1>(L, reps));
    std::printf("  fast            %8.3f ms\n", time_describe<false, 0>(L, reps));
    std::printf("  fast -atan2     %8.3f ms\n", time_describe<false, 2>(L, reps));
    std::printf("  fast -exp       %8.3f ms\n", time_describe<false, 4>(L, reps));
    std::printf("  fast -loads     %8.3f ms\n", time_describe<false, 8>(L, reps));
    std::printf("  fast -all       %8.3f ms\n", time_describe<false, 14>(L, reps));
    return 0;
}
