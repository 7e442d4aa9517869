// Kernel micro-benchmarks / ablations on synthetic data (performance
// experiments only; not part of libsift_mi.so).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I sift-features_amd/csrc \
//         tools/ubench_kernels.hip -o tools/ubench_kernels
#include "../sift-features_amd/csrc/describe.hip"
#include "../sift-features_amd/csrc/pyramid.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
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

template <int E, int A>
float time_describe(const DescLaunch& L, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    dim3 grid(std::min<uint32_t>(L.bound, 256 * (E == 4 ? 16 : 8)));  // as launch_describe: 16 waves / CU at kShare 4
    CK(hipMemset(L.work, 0, kDescWorkWords * 4));
    hipLaunchKernelGGL((k_describe<E, A>), grid, dim3(64), 0, 0, L);
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) {
        CK(hipMemsetAsync(L.work, 0, kDescWorkWords * 4, 0));
        hipLaunchKernelGGL((k_describe<E, A>), grid, dim3(64), 0, 0, L);
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// blur variants on an octave-0-sized batch (3840x2160, pitch 3840, 32 frames)
__global__ void k_fill(float* p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint32_t h = (uint32_t)i * 2654435761u;
        h ^= h >> 15;
        h *= 2246822519u;
        h ^= h >> 13;
        p[i] = (float)(h & 0xffff) / 65536.0f;
    }
}

// stride = distance between frames (floats); arena layout puts G_{s-1}, G_s,
// D_{s-1} of one frame inside an 11-plane octave arena, like the product.
template <int R, int TH>
float time_blur(const float* src, float* dst, float* dog, size_t stride, int W, int H, int pitch, int nimg,
                int reps) {
    using G = BlurGeom<R, TH>;
    BlurTaps taps{};
    for (int t = 0; t <= R; t++) taps.k[t] = 1.0f / (2 * R + 1);
    const int tx = (W + G::TW - 1) / G::TW, ty = (H + G::TH - 1) / G::TH;
    dim3 grid(tx, ty, nimg);
    auto go = [&]() {
        hipLaunchKernelGGL((k_blur<R, TH, kProfileOpenCV>), grid, dim3(256), 0, 0, src, stride, dst, stride, dog, stride,
                           (float*)nullptr, (size_t)0, 0, 0, 0, W, H, pitch, taps, 0);
    };
    go();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) go();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// the streaming strip kernel through the product launcher (segments as chosen there)
template <int R>
float time_blur_strip(const float* src, float* dst, size_t stride, int W, int H, int pitch, int nimg, int reps) {
    BlurLaunch L{};
    L.src = src;
    L.src_img_stride = stride;
    L.dst = dst;
    L.dst_img_stride = stride;
    L.W = W;
    L.H = H;
    L.pitch = pitch;
    L.n_img = nimg;
    for (int t = 0; t <= R; t++) L.taps.k[t] = 1.0f / (2 * R + 1);
    launch_blur(R, L, 0);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; i++) launch_blur(R, L, 0);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// octave-0 geometry of the bench (64 frames of the 2x 1080p seed, 3840x2160,
// 6-plane G arena): tile kernel vs strip kernel per radius, 8 B/px
void bench_blur_strip(int N) {
    const int W = 3840, H = 2160, pitch = 3840;
    const size_t plane = (size_t)pitch * H;
    float* base;
    CK(hipMalloc(&base, plane * 6 * N * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, base, plane * 6 * N);
    CK(hipDeviceSynchronize());
    const size_t stride = plane * 6;
    const double bytes = 8.0 * W * H * N;
    std::printf("blur G_{s-1} -> G_s, %d x %dx%d (arena, random): ms, GB/s at 8 B/px\n", N, W, H);
#define B(R, TH)                                                                                                  \
    {                                                                                                             \
        const float mt = time_blur<R, TH>(base, base + plane, nullptr, stride, W, H, pitch, N, 5);                 \
        const float ms = time_blur_strip<R>(base, base + plane, stride, W, H, pitch, N, 5);                       \
        std::printf("  R=%2d tile(TH=%d) %8.3f ms %7.1f GB/s | strip %8.3f ms %7.1f GB/s\n", R, TH, mt,            \
                    bytes / (mt * 1e-3) / 1e9, ms, bytes / (ms * 1e-3) / 1e9);                                      \
    }
    B(5, 32) B(6, 32) B(8, 32) B(10, 64) B(13, 64)
#undef B
    CK(hipFree(base));
}

void bench_blur(int N, bool arena, bool random) {
    const int W = 3840, H = 2160, pitch = 3840;
    const size_t plane = (size_t)pitch * H;
    float *base, *s, *d, *g;
    size_t stride;
    if (arena) {
        CK(hipMalloc(&base, plane * 11 * N * 4));
        stride = plane * 11;
        s = base;
        d = base + plane;
        g = base + 6 * plane;
        if (random) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, base, plane * 11 * N);
        else CK(hipMemset(base, 0, plane * 11 * N * 4));
    } else {
        CK(hipMalloc(&base, plane * 3 * N * 4));
        stride = plane;
        s = base;
        d = base + plane * N;
        g = base + 2 * plane * N;
        if (random) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, base, plane * 3 * N);
        else CK(hipMemset(base, 0, plane * 3 * N * 4));
    }
    CK(hipDeviceSynchronize());
    const double bytes = 12.0 * W * H * N;  // read G_{s-1}, write G_s + D_{s-1}
    std::printf("blur octave-0 batch (%d x %dx%d, %s layout, %s data): ms, effective GB/s (12 B/px)\n", N, W, H,
                arena ? "arena" : "planar", random ? "random" : "zero");
#define B(R, TH)                                                                                         \
    {                                                                                                    \
        const float ms = time_blur<R, TH>(s, d, g, stride, W, H, pitch, N, 5);                           \
        std::printf("  R=%2d TH=%2d %8.3f ms %8.1f GB/s\n", R, TH, ms, bytes / (ms * 1e-3) / 1e9);        \
    }
    B(5, 32) B(5, 64) B(6, 32) B(6, 64) B(8, 32) B(8, 64) B(10, 64) B(10, 128) B(13, 64) B(13, 128)
#undef B
    CK(hipFree(base));
}

// k_octave_tail on the bench's tail geometry (1080p: octaves 5..9 of the 2x
// seed, 64 frames): whole tail and one octave at a time
void bench_tail(int N) {
    const int n_oct = 10;
    TailLaunch L{};
    size_t total = 0;
    for (int o = 0; o < n_oct; o++) {
        L.ow[o] = 3840 >> o;
        L.oh[o] = 2160 >> o;
        L.pitch[o] = (L.ow[o] + 63) & ~63;
        L.gstride[o] = (size_t)6 * L.pitch[o] * L.oh[o];
        total += L.gstride[o] * N;
    }
    float* base;
    CK(hipMalloc(&base, total * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, base, total);
    size_t off = 0;
    for (int o = 0; o < n_oct; o++) {
        L.gauss[o] = base + off;
        off += L.gstride[o] * N;
    }
    const int radii[6] = {0, 5, 6, 8, 10, 13};
    for (int s = 1; s < 6; s++) {
        L.r[s] = radii[s];
        for (int t = 0; t <= radii[s]; t++) L.taps[s].k[t] = 1.0f / (2 * radii[s] + 1);
    }
    L.n_img = N;
    L.profile = kProfileOpenCV;
    auto timeit = [&](int o0, int o1) {
        L.o0 = o0;
        L.n_oct = o1;
        launch_octave_tail(L, 0);
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        for (int i = 0; i < 10; i++) launch_octave_tail(L, 0);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 10;
    };
#ifdef SIFT_TAIL_PROF
    {
        L.o0 = 5;
        L.n_oct = 10;
        for (int rep = 0; rep < 3; rep++) {
            launch_octave_tail(L, 0);
            CK(hipDeviceSynchronize());
        }
        std::vector<unsigned long long> pr(2048);
        CK(hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(g_tail_prof), 2048 * 8));
        std::printf("tail phases (workgroup 0, 100 MHz clock, us since start): tag dt\n");
        unsigned long long t0 = pr[0], tp = pr[0], cp = pr[1] >> 8;
        for (int k = 0; k < 1024; k++) {
            const unsigned long long t = pr[2 * k], tag = pr[2 * k + 1] & 255, c = pr[2 * k + 1] >> 8;
            std::printf("  %3llu %7.2f  +%5.2f us  +%6llu clk  (%.2f GHz)\n", tag, (t - t0) / 100.0, (t - tp) / 100.0,
                        c - cp, t > tp ? (c - cp) / ((t - tp) * 10.0) : 0.0);
            tp = t;
            cp = c;
            if (tag == 99) break;
        }
    }
#endif
    std::printf("octave tail, %d frames (1080p seed geometry)\n", N);
    std::printf("  octaves 5..9: %8.1f us\n", 1e3 * timeit(5, 10));
    for (int o = 5; o < 10; o++) std::printf("  octave %d alone (%dx%d): %8.1f us\n", o, L.ow[o], L.oh[o], 1e3 * timeit(o, o + 1));
    CK(hipFree(base));
}

// k_blur2_strip (two blurs in one pass) vs the two strip launches, octave-0
// geometry of the bench (64 frames of 3840x2160 in a 6-plane arena)
void bench_pair(int N, int W, int H) {
    const int pitch = (W + 63) & ~63;
    const size_t plane = (size_t)pitch * H;
    float* base;
    CK(hipMalloc(&base, plane * 6 * N * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, base, plane * 6 * N);
    CK(hipDeviceSynchronize());
    auto mk = [&](int s, int R) {
        BlurLaunch L{};
        L.src = base + (s - 1) * plane;
        L.dst = base + s * plane;
        L.src_img_stride = L.dst_img_stride = plane * 6;
        L.W = W;
        L.H = H;
        L.pitch = pitch;
        L.n_img = N;
        for (int t = 0; t <= R; t++) L.taps.k[t] = 1.0f / (2 * R + 1);
        return L;
    };
    auto timeit = [&](auto&& f) {
        f();
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        for (int i = 0; i < 5; i++) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 5;
    };
    const double px = (double)W * H * N;
    std::printf("blur pairs, %d x %dx%d: two strip launches (16 B/px) vs k_blur2_strip (12 B/px)\n", N, W, H);
    const int pr[2][2] = {{5, 6}, {8, 10}};
    for (auto& q : pr) {
        const BlurLaunch A = mk(1, q[0]), B = mk(2, q[1]);
        const float t2 = timeit([&] { launch_blur(q[0], A, 0); launch_blur(q[1], B, 0); });
        if (launch_blur_pair(q[0], q[1], A, B, 0)) {
            std::printf("  R=%d,%d  pair kernel not built (-DSIFT_PAIR_8_10)\n", q[0], q[1]);
            continue;
        }
        const float t1 = timeit([&] { launch_blur_pair(q[0], q[1], A, B, 0); });
        std::printf("  R=%d,%d  singles %8.3f ms %7.1f GB/s | pair %8.3f ms %7.1f GB/s (%.1f GB/s of the singles' bytes)\n",
                    q[0], q[1], t2, 16 * px / (t2 * 1e-3) / 1e9, t1, 12 * px / (t1 * 1e-3) / 1e9,
                    16 * px / (t1 * 1e-3) / 1e9);
    }
    CK(hipFree(base));
}

// segment-count target sweep (SIFT_MI_STRIP_WG) for the strip / pair kernels
// at the bench's octave 0..3 geometries (64 frames)
void bench_segs(int N) {
    const int dims[4][2] = {{3840, 2160}, {1920, 1080}, {960, 540}, {480, 270}};
    const long targets[7] = {1024, 2048, 4096, 8192, 12288, 24576, 49152};
    for (auto& d : dims) {
        const int W = d[0], H = d[1], pitch = (W + 63) & ~63;
        const size_t plane = (size_t)pitch * H;
        float* base;
        CK(hipMalloc(&base, plane * 6 * N * 4));
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, base, plane * 6 * N);
        CK(hipDeviceSynchronize());
        auto mk = [&](int s, int R) {
            BlurLaunch L{};
            L.src = base + (s - 1) * plane;
            L.dst = base + s * plane;
            L.src_img_stride = L.dst_img_stride = plane * 6;
            L.W = W;
            L.H = H;
            L.pitch = pitch;
            L.n_img = N;
            for (int t = 0; t <= R; t++) L.taps.k[t] = 1.0f / (2 * R + 1);
            return L;
        };
        auto timeit = [&](auto&& f) {
            f();
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            CK(hipEventRecord(a));
            for (int i = 0; i < 5; i++) f();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            return ms / 5;
        };
        std::printf("%dx%d x %d: us per launch (R=8 | R=13 | pair 5,6) by workgroup target\n", W, H, N);
        for (long t : targets) {
            char buf[32];
            std::snprintf(buf, sizeof buf, "%ld", t);
            setenv("SIFT_MI_STRIP_WG", buf, 1);
            const BlurLaunch A = mk(1, 8), C = mk(1, 13), P1 = mk(1, 5), P2 = mk(2, 6);
            const float t8 = timeit([&] { launch_blur(8, A, 0); });
            const float t13 = timeit([&] { launch_blur(13, C, 0); });
            const float tp = timeit([&] { launch_blur_pair(5, 6, P1, P2, 0); });
            std::printf("  %6ld: %8.1f %8.1f %8.1f\n", t, 1e3 * t8, 1e3 * t13, 1e3 * tp);
        }
        unsetenv("SIFT_MI_STRIP_WG");
        CK(hipFree(base));
    }
}


// seed (u8 -> 2x bilinear -> R = 5 blur): the product launcher's strip kernel
// vs the tile kernel (SIFT_MI_BLUR_KERNEL=tile), bit-identical check + time,
// N frames of sw x sh (row stride `stride` >= sw)
static void cv_linear_tab(int ssz, int dsz, std::vector<int>& ofs, std::vector<float>& a0, std::vector<float>& a1,
                          int* lim) {
    const double scale = 1. / ((double)dsz / ssz);
    int xmax = dsz;
    ofs.resize(dsz);
    a0.resize(dsz);
    a1.resize(dsz);
    for (int d = 0; d < dsz; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)floorf(f);
        f -= (float)s;
        if (s < 0) { f = 0; s = 0; }
        if (s + 1 >= ssz) {
            if (d < xmax) xmax = d;
            if (s >= ssz - 1) { f = 0; s = ssz - 1; }
        }
        ofs[d] = s;
        a0[d] = 1.f - f;
        a1[d] = f;
    }
    *lim = xmax;
}

void bench_seed(int N, int sw, int sh, int stride) {
    const int W = 2 * sw, H = 2 * sh, pitch = (W + 63) & ~63;
    std::vector<uint8_t> hf((size_t)N * stride * sh);
    uint32_t x = 12345;
    for (auto& v : hf) { x = x * 1664525u + 1013904223u; v = (uint8_t)(x >> 24); }
    uint8_t* df;
    CK(hipMalloc(&df, hf.size()));
    CK(hipMemcpy(df, hf.data(), hf.size(), hipMemcpyHostToDevice));
    std::vector<int> xo, yo;
    std::vector<float> xa, xb, ya, yb;
    int xmax, ymax;
    cv_linear_tab(sw, W, xo, xa, xb, &xmax);
    cv_linear_tab(sh, H, yo, ya, yb, &ymax);
    int *dxo, *dyo;
    float *dxa, *dxb, *dya, *dyb;
    CK(hipMalloc(&dxo, W * 4)); CK(hipMalloc(&dxa, W * 4)); CK(hipMalloc(&dxb, W * 4));
    CK(hipMalloc(&dyo, H * 4)); CK(hipMalloc(&dya, H * 4)); CK(hipMalloc(&dyb, H * 4));
    CK(hipMemcpy(dxo, xo.data(), W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxa, xa.data(), W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxb, xb.data(), W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dyo, yo.data(), H * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dya, ya.data(), H * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dyb, yb.data(), H * 4, hipMemcpyHostToDevice));
    const size_t plane = (size_t)pitch * H;
    float *d0, *d1;
    CK(hipMalloc(&d0, plane * N * 4));
    CK(hipMalloc(&d1, plane * N * 4));
    SeedLaunch L{};
    L.frames = df;
    L.frame_pitch = (size_t)stride * sh;
    L.row_stride = stride;
    L.sh = sh;
    L.sw = sw;
    L.tab = ResizeTab{dxo, dxa, dxb, dyo, dya, dyb, xmax};
    L.profile = kProfileOpenCV;
    L.dst_img_stride = plane;
    L.W = W;
    L.H = H;
    L.pitch = pitch;
    L.n_img = N;
    const double s = 1.2489996;
    for (int t = 0; t <= 5; t++) L.taps.k[t] = (float)std::exp(-(t * t) / (2 * s * s)) / 3.1f;
    auto timeit = [&](float* dst) {
        L.dst = dst;
        launch_seed(5, L, 0);
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        for (int i = 0; i < 10; i++) launch_seed(5, L, 0);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 10;
    };
    CK(hipMemset(d0, 0, plane * N * 4));
    CK(hipMemset(d1, 0, plane * N * 4));
    setenv("SIFT_MI_BLUR_KERNEL", "tile", 1);
    const float t_old = timeit(d0);
    unsetenv("SIFT_MI_BLUR_KERNEL");
    const float t_new = timeit(d1);
    std::vector<float> h0(plane * N), h1(plane * N);
    CK(hipMemcpy(h0.data(), d0, plane * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), d1, plane * N * 4, hipMemcpyDeviceToHost));
    size_t diff = 0, first = (size_t)-1;
    for (int b = 0; b < N; b++)
        for (int y = 0; y < H; y++)
            for (int xx = 0; xx < W; xx++) {
                const size_t i = (size_t)b * plane + (size_t)y * pitch + xx;
                if (std::memcmp(&h0[i], &h1[i], 4)) {
                    if (!diff) first = i;
                    diff++;
                }
            }
    const double bytes = (double)N * (sw * (double)sh + 4.0 * W * H);
    std::printf("seed %d x %dx%d (stride %d): tile %8.1f us %6.2f TB/s | strip %8.1f us %6.2f TB/s | differing px %zu",
                N, sw, sh, stride, 1e3 * t_old, bytes / (t_old * 1e-3) / 1e12, 1e3 * t_new,
                bytes / (t_new * 1e-3) / 1e12, diff);
    if (diff) std::printf(" (first at frame %zu y %zu x %zu)", first / plane, (first % plane) / pitch, first % pitch);
    std::printf("\n");
    CK(hipFree(df)); CK(hipFree(d0)); CK(hipFree(d1));
    CK(hipFree(dxo)); CK(hipFree(dxa)); CK(hipFree(dxb)); CK(hipFree(dyo)); CK(hipFree(dya)); CK(hipFree(dyb));
}

// octave-0 head of the bench (N frames of 1920x1080 -> 3840x2160, 6-plane
// arena + the next octave's plane): seed, (5, 6) pair, blur 3 with the next
// base (round 3) vs k_seed_pair then the (6, 8) pair with the next base
// (round 4); G_0..G_3 and the next base compared bit for bit
void bench_head(int N, int profile) {
    const int sw = 1920, sh = 1080, W = 2 * sw, H = 2 * sh, pitch = (W + 63) & ~63;
    const int wn = W / 2, hn = H / 2, pn = (wn + 63) & ~63;
    std::vector<uint8_t> hf((size_t)N * sw * sh);
    uint32_t x = 12345;
    for (size_t i = 0; i < hf.size(); i++) {
        const size_t px = i % ((size_t)sw * sh);
        const int xx = (int)(px % sw), yy = (int)(px / sw);
        x = x * 1664525u + 1013904223u;  // smooth field + noise
        hf[i] = (uint8_t)(128 + 60 * std::sin(xx * 0.05) * std::cos(yy * 0.03) + (int)(x >> 29));
    }
    uint8_t* df;
    CK(hipMalloc(&df, hf.size()));
    CK(hipMemcpy(df, hf.data(), hf.size(), hipMemcpyHostToDevice));
    std::vector<int> xo, yo;
    std::vector<float> xa, xb, ya, yb;
    int xmax, ymax;
    cv_linear_tab(sw, W, xo, xa, xb, &xmax);
    cv_linear_tab(sh, H, yo, ya, yb, &ymax);
    int *dxo, *dyo;
    float *dxa, *dxb, *dya, *dyb;
    CK(hipMalloc(&dxo, W * 4)); CK(hipMalloc(&dxa, W * 4)); CK(hipMalloc(&dxb, W * 4));
    CK(hipMalloc(&dyo, H * 4)); CK(hipMalloc(&dya, H * 4)); CK(hipMalloc(&dyb, H * 4));
    CK(hipMemcpy(dxo, xo.data(), W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxa, xa.data(), W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dxb, xb.data(), W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dyo, yo.data(), H * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dya, ya.data(), H * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dyb, yb.data(), H * 4, hipMemcpyHostToDevice));
    const size_t plane = (size_t)pitch * H, nplane = (size_t)pn * hn;
    const size_t stride = plane * 6;
    float *g[2], *nx[2];
    for (int v = 0; v < 2; v++) {
        CK(hipMalloc(&g[v], stride * N * 4));
        CK(hipMalloc(&nx[v], nplane * N * 4));
        CK(hipMemset(g[v], 0, stride * N * 4));
        CK(hipMemset(nx[v], 0, nplane * N * 4));
    }
    // taps: normalised Gaussians of the radii (the arithmetic, not the sigmas, matters here)
    auto taps = [](int R) {
        BlurTaps t{};
        double s = 0;
        for (int k = -R; k <= R; k++) s += std::exp(-(k * k) / (2.0 * (R / 4.0) * (R / 4.0)));
        for (int k = 0; k <= R; k++) t.k[k] = (float)(std::exp(-(k * k) / (2.0 * (R / 4.0) * (R / 4.0))) / s);
        return t;
    };
    const bool ip = profile == kProfileImageproc;
    const int rs = ip ? 3 : 5, r1 = ip ? 3 : 5, r2 = ip ? 4 : 6, r3 = ip ? 4 : 8;
    auto seedl = [&](int v) {
        SeedLaunch L{};
        L.frames = df;
        L.frame_pitch = (size_t)sw * sh;
        L.row_stride = sw;
        L.sh = sh;
        L.sw = sw;
        L.tab = ResizeTab{dxo, dxa, dxb, dyo, dya, dyb, xmax};
        L.profile = profile;
        L.dst = g[v];
        L.dst_img_stride = stride;
        L.W = W;
        L.H = H;
        L.pitch = pitch;
        L.n_img = N;
        L.taps = taps(rs);
        return L;
    };
    auto blurl = [&](int v, int s, int R) {
        BlurLaunch L{};
        L.src = g[v] + (s - 1) * plane;
        L.dst = g[v] + s * plane;
        L.src_img_stride = L.dst_img_stride = stride;
        L.W = W;
        L.H = H;
        L.pitch = pitch;
        L.n_img = N;
        L.taps = taps(R);
        L.profile = profile;
        if (s == 3) {
            L.nxt = nx[v];
            L.nxt_img_stride = nplane;
            L.pitch_n = pn;
            L.wn = wn;
            L.hn = hn;
        }
        return L;
    };
    auto timeit = [&](auto&& f) {
        f();
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        for (int i = 0; i < 5; i++) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 5;
    };
    int rc = 0;
    const float t_old = timeit([&] {
        rc |= launch_seed(rs, seedl(0), 0);
        rc |= launch_blur_pair(r1, r2, blurl(0, 1, r1), blurl(0, 2, r2), 0);
        rc |= launch_blur(r3, blurl(0, 3, r3), 0);
    });
    const float ts = timeit([&] { launch_seed(rs, seedl(0), 0); });
    const float tp = timeit([&] { launch_blur_pair(r1, r2, blurl(0, 1, r1), blurl(0, 2, r2), 0); });
    const float t3 = timeit([&] { launch_blur(r3, blurl(0, 3, r3), 0); });
    const float t_new = timeit([&] {
        rc |= launch_seed_pair(rs, r1, seedl(1), blurl(1, 1, r1), 0);
        rc |= launch_blur_pair(r2, r3, blurl(1, 2, r2), blurl(1, 3, r3), 0);
    });
    const float tsp = timeit([&] { launch_seed_pair(rs, r1, seedl(1), blurl(1, 1, r1), 0); });
    const float tp23 = timeit([&] { launch_blur_pair(r2, r3, blurl(1, 2, r2), blurl(1, 3, r3), 0); });
    CK(hipDeviceSynchronize());
    std::vector<float> h0(stride * N), h1(stride * N), n0(nplane * N), n1(nplane * N);
    CK(hipMemcpy(h0.data(), g[0], stride * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), g[1], stride * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(n0.data(), nx[0], nplane * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(n1.data(), nx[1], nplane * N * 4, hipMemcpyDeviceToHost));
    size_t diff[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < N; b++)
        for (int s = 0; s < 4; s++)
            for (int y = 0; y < H; y++)
                diff[s] += std::memcmp(&h0[b * stride + s * plane + (size_t)y * pitch],
                                       &h1[b * stride + s * plane + (size_t)y * pitch], W * 4) != 0;
    for (int b = 0; b < N; b++)
        for (int y = 0; y < hn; y++)
            diff[4] += std::memcmp(&n0[b * nplane + (size_t)y * pn], &n1[b * nplane + (size_t)y * pn], wn * 4) != 0;
    // each path's next base against its own G_3 (nearest 1/2: (2x, 2y) / (2x + 1, 2y + 1))
    for (int v = 0; v < 2; v++) {
        const std::vector<float>& gg = v ? h1 : h0;
        const std::vector<float>& nn = v ? n1 : n0;
        size_t bad = 0;
        int fb = -1, fy = -1, fx = -1;
        for (int b = 0; b < N; b++)
            for (int yy = 0; yy < hn; yy++)
                for (int xx = 0; xx < wn; xx++) {
                    const float e = gg[b * stride + 3 * plane + (size_t)(2 * yy + ip) * pitch + 2 * xx + ip];
                    if (std::memcmp(&e, &nn[b * nplane + (size_t)yy * pn + xx], 4)) {
                        if (!bad) fb = b, fy = yy, fx = xx;
                        bad++;
                    }
                }
        std::printf("  %s path: next base vs its G_3: %zu px differ (first frame %d y %d x %d)\n", v ? "new" : "old",
                    bad, fb, fy, fx);
        if (bad) {
            int rows[8], nr = 0;
            for (int yy = 0; yy < hn && nr < 8; yy++) {
                bool d = false;
                for (int xx = 0; xx < wn; xx++) {
                    const float e = gg[3 * plane + (size_t)(2 * yy + ip) * pitch + 2 * xx + ip];
                    d |= std::memcmp(&e, &nn[(size_t)yy * pn + xx], 4) != 0;
                }
                if (d) rows[nr++] = yy;
            }
            std::printf("    frame 0 rows:");
            for (int i = 0; i < nr; i++) std::printf(" %d", rows[i]);
            std::printf("\n    next[y=%d][0..3] = %g %g %g %g, G3 = %g %g %g %g\n", fy, nn[(size_t)fy * pn],
                        nn[(size_t)fy * pn + 1], nn[(size_t)fy * pn + 2], nn[(size_t)fy * pn + 3],
                        gg[3 * plane + (size_t)(2 * fy + ip) * pitch + ip], gg[3 * plane + (size_t)(2 * fy + ip) * pitch + 2 + ip],
                        gg[3 * plane + (size_t)(2 * fy + ip) * pitch + 4 + ip], gg[3 * plane + (size_t)(2 * fy + ip) * pitch + 6 + ip]);
        }
    }
    const double px = (double)W * H * N;
    std::printf("octave-0 head (%s), %d x %dx%d -> G_0..G_3 + next base: rc %d\n", ip ? "imageproc" : "opencv", N,
                sw, sh, rc);
    std::printf("  round 3: seed %7.1f + pair(1,2) %7.1f + blur3 %7.1f us = %7.1f us in sequence (%7.1f us), "
                "%.2f TB/s of its %.2f B/px\n", 1e3 * ts, 1e3 * tp, 1e3 * t3, 1e3 * (ts + tp + t3), 1e3 * t_old,
                (0.25 + 24.25) * px / (t_old * 1e-3) / 1e12, 0.25 + 24.25);
    std::printf("  round 4: seed pair %7.1f + pair(2,3) %7.1f us = %7.1f us in sequence (%7.1f us), "
                "%.2f TB/s of its %.2f B/px\n", 1e3 * tsp, 1e3 * tp23, 1e3 * (tsp + tp23), 1e3 * t_new,
                (0.25 + 20.25) * px / (t_new * 1e-3) / 1e12, 0.25 + 20.25);
    std::printf("  rows differing: G0 %zu G1 %zu G2 %zu G3 %zu next %zu\n", diff[0], diff[1], diff[2], diff[3],
                diff[4]);
    for (int v = 0; v < 2; v++) {
        CK(hipFree(g[v]));
        CK(hipFree(nx[v]));
    }
    CK(hipFree(df));
    CK(hipFree(dxo)); CK(hipFree(dxa)); CK(hipFree(dxb)); CK(hipFree(dyo)); CK(hipFree(dya)); CK(hipFree(dyb));
}

// k_seed_strip timing ablations (ABL bits: 1 no plane stores, 2 no loads /
// upsample, 4 no row pass), 64 frames of 1920x1080 -> 3840x2160
template <int ABL>
float time_seed_abl(const uint8_t* df, float* dst, int N) {
    const int sw = 1920, sh = 1080, W = 3840, H = 2160, pitch = 3840;
    using G = StripGeom<5>;
    const int strips = W / G::TW;
    BlurTaps taps{};
    for (int t = 0; t <= 5; t++) taps.k[t] = 1.0f / 11;
    const int seg = 360, nseg = H / seg;
    auto go = [&]() {
        hipLaunchKernelGGL((k_seed_strip<5, kProfileOpenCV, ABL>), dim3(strips, nseg, N), dim3(256), 0, 0, df, (size_t)sw * sh,
                           (size_t)sw, sh, sw, dst, (size_t)pitch * H, W, H, pitch, taps, 0, H, seg);
    };
    go();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < 10; i++) go();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 10;
}

void bench_seed_abl(int N) {
    uint8_t* df;
    CK(hipMalloc(&df, (size_t)N * 1920 * 1080));
    CK(hipMemset(df, 77, (size_t)N * 1920 * 1080));
    float* dst;
    CK(hipMalloc(&dst, (size_t)N * 3840 * 2160 * 4));
    std::printf("seed ablations, %d x 1920x1080 (seg 360): us\n", N);
    std::printf("  full           %8.1f\n", 1e3 * time_seed_abl<0>(df, dst, N));
    std::printf("  -stores        %8.1f\n", 1e3 * time_seed_abl<1>(df, dst, N));
    std::printf("  -loader        %8.1f\n", 1e3 * time_seed_abl<2>(df, dst, N));
    std::printf("  -rowpass       %8.1f\n", 1e3 * time_seed_abl<4>(df, dst, N));
    std::printf("  -stores-loader %8.1f\n", 1e3 * time_seed_abl<3>(df, dst, N));
    std::printf("  -loader-rowpass %8.1f\n", 1e3 * time_seed_abl<6>(df, dst, N));
    std::printf("  colpass only (no stores) %8.1f\n", 1e3 * time_seed_abl<7>(df, dst, N));
    CK(hipFree(df));
    CK(hipFree(dst));
}

// HBM ceilings on the octave-0 plane geometry (64 x 3840 x 2160 f32):
// read-only, write-only and copy streams, 16 B per lane, grid-stride
template <int MODE>  // 0 read (sum), 1 write, 2 copy, 3 copy with NT stores, 4 write NT
__global__ __launch_bounds__(256) void k_stream(const float4* __restrict__ a, float4* __restrict__ b, size_t n,
                                                float* sink) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (MODE == 0) {
            const float4 v = a[i];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        } else if (MODE == 1) {
            b[i] = make_float4((float)i, 1.f, 2.f, 3.f);
        } else if (MODE == 4) {
            __builtin_nontemporal_store(f4v{(float)i, 1.f, 2.f, 3.f}, reinterpret_cast<f4v*>(b + i));
        } else if (MODE == 2) {
            b[i] = a[i];
        } else {
            __builtin_nontemporal_store(reinterpret_cast<const f4v*>(a)[i], reinterpret_cast<f4v*>(b + i));
        }
    }
    if (MODE == 0 && acc.x + acc.y + acc.z + acc.w == 12345.f) *sink = 1.f;
}

template <int MODE>
float time_stream(const float4* a, float4* b, size_t n, float* sink, int grid) {
    hipLaunchKernelGGL((k_stream<MODE>), dim3(grid), dim3(256), 0, 0, a, b, n, sink);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < 5; i++) hipLaunchKernelGGL((k_stream<MODE>), dim3(grid), dim3(256), 0, 0, a, b, n, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 5;
}

void bench_stream(int N) {
    const size_t n = (size_t)N * 3840 * 2160 / 4;
    float4 *a, *b;
    float* sink;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(a, 0, n * 16));
    const double gb = n * 16 / 1e9;
    for (int grid : {2048, 8192, 32768}) {
        const float r = time_stream<0>(a, b, n, sink, grid), w = time_stream<1>(a, b, n, sink, grid),
                    wn = time_stream<4>(a, b, n, sink, grid), c = time_stream<2>(a, b, n, sink, grid),
                    cn = time_stream<3>(a, b, n, sink, grid);
        std::printf("stream %d frames-planes, grid %d: read %.2f TB/s | write %.2f | write nt %.2f | copy %.2f (r+w) | copy nt %.2f\n",
                    N, grid, gb / r, gb / w, gb / wn, 2 * gb / c, 2 * gb / cn);
    }
    CK(hipFree(a));
    CK(hipFree(b));
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "all";
    if (!strcmp(mode, "head")) {
        bench_head(argc > 2 ? atoi(argv[2]) : 64, kProfileOpenCV);
        bench_head(argc > 2 ? atoi(argv[2]) : 64, kProfileImageproc);
        return 0;
    }
    if (!strcmp(mode, "segs")) {
        bench_segs(argc > 2 ? atoi(argv[2]) : 64);
        return 0;
    }
    if (!strcmp(mode, "pair")) {
        bench_pair(argc > 2 ? atoi(argv[2]) : 64, 3840, 2160);
        bench_pair(argc > 2 ? atoi(argv[2]) : 64, 1920, 1080);
        bench_pair(argc > 2 ? atoi(argv[2]) : 64, 960, 540);
        return 0;
    }
    if (!strcmp(mode, "stream")) {
        bench_stream(argc > 2 ? atoi(argv[2]) : 64);
        return 0;
    }
    if (!strcmp(mode, "seedabl")) {
        bench_seed_abl(argc > 2 ? atoi(argv[2]) : 64);
        return 0;
    }
    if (!strcmp(mode, "seed")) {
        const int n = argc > 2 ? atoi(argv[2]) : 64;
        bench_seed(n, 1920, 1080, 1920);
        bench_seed(4, 1921, 1079, 1923);
        bench_seed(4, 333, 97, 335);
        bench_seed(4, 80, 40, 81);
        bench_seed(n, 960, 540, 960);
        return 0;
    }
    if (!strcmp(mode, "tail")) {
        bench_tail(argc > 2 ? atoi(argv[2]) : 64);
        return 0;
    }
    if (!strcmp(mode, "strip")) {
        bench_blur_strip(argc > 2 ? atoi(argv[2]) : 64);
        return 0;
    }
    if (!strcmp(mode, "all") || !strcmp(mode, "blur")) {
        bench_blur(16, false, false);
        bench_blur(16, false, true);
        bench_blur(16, true, true);
        bench_blur(2, true, true);
    }
    if (strcmp(mode, "all") && strcmp(mode, "desc")) return 0;
    const int W = 3840, H = 2160, pitch = 3840, NKP = 200000;
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
    uint32_t* d_n;
    CK(hipMalloc(&d_n, 4));
    CK(hipMemcpy(d_n, &NKP, 4, hipMemcpyHostToDevice));
    L.n = d_n;
    L.bound = NKP;
    uint32_t* d_work;
    CK(hipMalloc(&d_work, kDescWorkWords * 4));
    L.work = d_work;
    L.gauss = d_g;
    L.gauss_img_stride = d_gs;
    L.ow = d_w;
    L.oh = d_h;
    L.opitch = d_p;
    L.out_desc = d_desc;
    const int reps = 5;
    std::printf("describe n=%d\n", NKP);
    std::printf("  exact           %8.3f ms\n", time_describe<0, 0>(L, reps));
    std::printf("  exact -phaseB   %8.3f ms\n", time_describe<0, 1>(L, reps));
    std::printf("  fast s1         %8.3f ms\n", time_describe<1, 0>(L, reps));
    std::printf("  fast s2         %8.3f ms\n", time_describe<2, 0>(L, reps));
    std::printf("  fast s4         %8.3f ms\n", time_describe<4, 0>(L, reps));
    std::printf("  fast s4 -rmw    %8.3f ms\n", time_describe<4, 1>(L, reps));
    std::printf("  fast s4 nosample %8.3f ms\n", time_describe<4, 64>(L, reps));
    std::printf("  fast s4 f32sincos %8.3f ms\n", time_describe<4, 128>(L, reps));
    std::printf("  fast s4 nosample f32sincos %8.3f ms\n", time_describe<4, 192>(L, reps));
    std::printf("  fast s4 -atan2  %8.3f ms\n", time_describe<4, 2>(L, reps));
    std::printf("  fast s4 -exp    %8.3f ms\n", time_describe<4, 4>(L, reps));
    std::printf("  fast s4 -loads  %8.3f ms\n", time_describe<4, 8>(L, reps));
    std::printf("  fast s4 -all    %8.3f ms\n", time_describe<4, 14>(L, reps));
    std::printf("  fast s4 -all -rmw %8.3f ms\n", time_describe<4, 15>(L, reps));
    std::printf("  fast s2 -rmw    %8.3f ms\n", time_describe<2, 1>(L, reps));
    std::printf("  fast s2 nosample %8.3f ms\n", time_describe<2, 64>(L, reps));
    std::printf("  fast s2 -atan2  %8.3f ms\n", time_describe<2, 2>(L, reps));
    std::printf("  fast s2 -exp    %8.3f ms\n", time_describe<2, 4>(L, reps));
    std::printf("  fast s2 -loads  %8.3f ms\n", time_describe<2, 8>(L, reps));
    std::printf("  fast s2 -all    %8.3f ms\n", time_describe<2, 14>(L, reps));
    std::printf("  fast s2 -all -rmw %8.3f ms\n", time_describe<2, 15>(L, reps));
    return 0;
}
