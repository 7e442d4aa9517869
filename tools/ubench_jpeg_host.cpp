// Host entropy-decoder microbenchmark (no GPU needed): parse + entropy-decode
// JPEG files with jpeg.hip's host code, report ms per frame and an FNV-1a
// checksum of the quantised coefficients (identical across decoder changes).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/ubench_jpeg_host.cpp -o /tmp/ubj -lpthread
//   /tmp/ubj reps file.jpg [file.jpg ...]
#include "../sift-features_amd/csrc/jpeg.hip"

#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>

using namespace siftmi;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int reps = atoi(argv[1]);
    double total_ms = 0;
    int frames = 0;
    for (int a = 2; a < argc; a++) {
        std::ifstream f(argv[a], std::ios::binary);
        std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        std::string err;
        jpg::Header H;
        if (jpg::parse(d.data(), d.size(), H, err)) return printf("%s: %s\n", argv[a], err.c_str()), 1;
        const jpg::Geom g = jpg::geometry(H);
        std::vector<int16_t> coef(g.total * 64);
        uint64_t h = 1469598103934665603ull;
        double best = 1e30;
        for (int r = 0; r < reps; r++) {
            const auto t0 = std::chrono::steady_clock::now();
            if (jpg::entropy_decode(d.data(), d.size(), H, g, coef.data(), err))
                return printf("%s: %s\n", argv[a], err.c_str()), 1;
            best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        total_ms += best;  // best of `reps` per file (the host is shared)
        frames++;
        for (int16_t v : coef) h = (h ^ (uint16_t)v) * 1099511628211ull;
        printf("%s %dx%d checksum %016llx\n", argv[a], H.w, H.h, (unsigned long long)h);
    }
    printf("%.3f ms per frame (best of %d, %d files)\n", total_ms / frames, reps, frames);
    return 0;
}
