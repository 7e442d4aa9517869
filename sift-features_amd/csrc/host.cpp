// libsift_mi.so host side: the C ABI of include/sift_mi.h over the HIP
// kernels in this directory.  Mirrors the reference's pipeline
// (src/lib.rs:71-177): precompute_images -> find_keypoints -> [limit] ->
// compute_descriptors -> KeyPoint mapping, batched over equal-size frames.
//
// Host arithmetic that feeds the device (octave count, blur sigmas, OpenCV
// kernel taps, resize coefficient tables) is computed exactly as the
// reference / OpenCV compute it (IEEE double / f32, glibc libm).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sift_mi.h"
#include "sift_common.h"
#include "sift_kernels.h"

using namespace siftmi;

hipError_t siftmi::host_wait_event(hipEvent_t e) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t r = hipEventQuery(e);
        if (r != hipErrorNotReady) return r;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(1000))
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) return fail(SIFT_MI_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define CHK(expr)            \
    do {                     \
        int rc_ = (expr);    \
        if (rc_) return rc_; \
    } while (0)

// bumped by every device / pinned (re)allocation and release: a captured
// graph (single-chunk replay) is valid only while it is unchanged
std::atomic<uint64_t> g_alloc_gen{0};

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap && p) return 0;
        g_alloc_gen++;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        if (hipMalloc(&p, bytes) != hipSuccess) {
            p = nullptr;
            return fail(SIFT_MI_ENOMEM, "hipMalloc(" + std::to_string(bytes) + ") failed");
        }
        cap = std::max<size_t>(n, 1);
        return 0;
    }
    void release() {
        if (p) {
            g_alloc_gen++;
            (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
};

// Grows d to at least n elements keeping its first `used` elements (device copy
// on stream st, synchronised).
template <class T>
int grow_keep(DevBuf<T>& d, size_t n, size_t used, hipStream_t st) {
    if (n <= d.cap && d.p) return 0;
    DevBuf<T> nd;
    CHK(nd.ensure(std::max(n, 2 * d.cap)));
    if (used && d.p) HIPCHK(hipMemcpyAsync(nd.p, d.p, used * sizeof(T), hipMemcpyDeviceToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    d.release();
    d.p = nd.p;
    d.cap = nd.cap;
    nd.p = nullptr;
    nd.cap = 0;
    return 0;
}

template <class T>
struct PinBuf {
    T* p = nullptr;
    size_t cap = 0;
    int ensure(size_t n, bool keep = false) {
        if (n <= cap && p) return 0;
        size_t ncap = std::max<size_t>({n, 1, cap * 2});
        g_alloc_gen++;
        T* q = nullptr;
        if (hipHostMalloc(&q, ncap * sizeof(T), hipHostMallocDefault) != hipSuccess)
            return fail(SIFT_MI_ENOMEM, "hipHostMalloc failed");
        if (keep && p && cap) std::memcpy(q, p, cap * sizeof(T));
        if (p) (void)hipHostFree(p);
        p = q;
        cap = ncap;
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// ---------------------------------------------------------------------------
// Reference host arithmetic
// ---------------------------------------------------------------------------
// n_octaves = round(log2(min(2W,2H)) - 2) as usize + 1  (src/lib.rs:133-134)
int n_octaves_for(uint32_t w, uint32_t h) {
    const uint32_t m = std::min(2 * w, 2 * h);
    const float f = roundf(log2f((float)m) - 2.0f);
    const size_t u = (f > 0.0f) ? (size_t)f : 0;  // saturating `as usize`
    return (int)u + 1;
}

double powi_f64(double a, int b) {  // compiler-rt __powidf2 (llvm.powi)
    const bool recip = b < 0;
    double r = 1;
    for (;;) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1 / r : r;
}

// src/lib.rs:220-229
void octave_sigmas(double* sig) {
    const double m = std::pow(2.0, 2.0 / kScalesPerOctave);
    for (int s = 0; s < kImagesPerOctave; s++) {
        const double a = powi_f64(m, s - 1);
        const double b = a * m;
        sig[s] = std::sqrt(b - a) * 0.8 * 2.0;
    }
}
// src/lib.rs:207
double seed_sigma() { return std::sqrt(0.8 * 0.8 - 0.5 * 0.5) * 2.0; }

// cv::GaussianBlur(Size(), sigma), CV_32F: ksize = cvRound(sigma*4*2+1)|1;
// taps from getGaussianKernelBitExact (IEEE double), cast to f32.
int cv_blur_taps(double sigma, BlurTaps* t) {
    const int n = ((int)std::lrint(sigma * 4 * 2 + 1)) | 1;
    const int r = n / 2;
    if (r < 1 || r > 24) return -1;
    const double scale2X = -0.125 / (sigma * sigma);
    const int n2 = (n - 1) / 2;
    double values[64];
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        const double v = std::exp((double)(x * x) * scale2X);
        values[i] = v;
        sum += v;
    }
    sum *= 2;
    sum += 1;
    const double mul1 = 1 / sum;
    std::memset(t, 0, sizeof(*t));
    t->k[0] = (float)(1.0 * mul1);
    for (int i = 0; i < n2; i++) t->k[r - i] = (float)(values[i] * mul1);
    return r;
}

// cv::resize INTER_LINEAR coefficient table (resizeGeneric_)
void cv_linear_coeffs(int ssz, int dsz, std::vector<int>& ofs, std::vector<float>& a0, std::vector<float>& a1,
                      int* lim) {
    const double inv = (double)dsz / ssz;
    const double scale = 1. / inv;
    int xmax = dsz;
    ofs.resize(dsz);
    a0.resize(dsz);
    a1.resize(dsz);
    for (int d = 0; d < dsz; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = (int)floorf(f);
        f -= (float)s;
        if (s < 0) {
            f = 0;
            s = 0;
        }
        if (s + 1 >= ssz) {
            if (d < xmax) xmax = d;
            if (s >= ssz - 1) {
                f = 0;
                s = ssz - 1;
            }
        }
        ofs[d] = s;
        a0[d] = 1.f - f;
        a1[d] = f;
    }
    *lim = xmax;
}

// cv::resize INTER_NEAREST offsets (resizeNN)
void cv_nearest_ofs(int ssz, int dsz, std::vector<int>& ofs) {
    const double ifx = 1. / ((double)dsz / ssz);
    ofs.resize(dsz);
    for (int d = 0; d < dsz; d++) {
        const int s = (int)std::floor(d * ifx);
        ofs[d] = std::min(s, ssz - 1);
    }
}

// ---- ImageprocProcessing profile (src/lib.rs:993-1007) ---------------------
// imageproc 0.25.0 gaussian_kernel_f32 and image 0.25.2 imageops::resize
// sampling weights, restated (third-party code absent from /root/reference;
// parity unpinned -- DESIGN.md).  Same f32 arithmetic as oracle/sift_oracle.c.
int ip_blur_taps(float sigma, BlurTaps* t) {
    const int r = (int)std::ceil(2.0f * sigma);
    if (r < 1 || r > 24) return -1;
    const int n = 2 * r + 1;
    float k[64];
    const float norm = 1.0f / (std::sqrt(2.0f * 3.14159265358979323846f) * sigma);
    for (int i = 0; i <= r; i++) {
        const float x = (float)i;
        const float v = norm * std::exp(-(x * x) / (2.0f * (sigma * sigma)));
        k[r + i] = v;
        k[r - i] = v;
    }
    float sum = 0.0f;
    for (int i = 0; i < n; i++) sum += k[i];
    std::memset(t, 0, sizeof(*t));
    for (int i = 0; i <= r; i++) t->k[i] = k[r + i] / sum;
    return r;
}

// One axis of image's vertical_sample / horizontal_sample: taps [left, left+n)
// with normalised f32 weights; support 1 = Triangle, 0 = Nearest.
int ip_axis(int src, int dst, int out, float support, int* left, float* w) {
    const float ratio = (float)src / (float)dst;
    const float sratio = ratio < 1.0f ? 1.0f : ratio;
    const float src_support = support * sratio;
    float in = ((float)out + 0.5f) * ratio;
    long l = (long)std::floor(in - src_support);
    l = l < 0 ? 0 : (l > src - 1 ? src - 1 : l);
    long rt = (long)std::ceil(in + src_support);
    rt = rt < l + 1 ? l + 1 : (rt > src ? src : rt);
    in = in - 0.5f;
    float sum = 0.0f;
    int n = 0;
    for (long i = l; i < rt; i++) {
        float v = 1.0f;  // box_kernel
        if (support > 0.0f) {
            const float a = std::fabs(((float)i - in) / sratio);
            v = a < 1.0f ? 1.0f - a : 0.0f;
        }
        w[n++] = v;
        sum += v;
    }
    for (int i = 0; i < n; i++) w[i] = w[i] / sum;
    *left = (int)l;
    return n;
}

// Device tables of one resize (both axes), taps padded with zero weights.
struct IpTabDev {
    DevBuf<int> xl, yl;
    DevBuf<float> xw, yw;
    int xtaps = 0, ytaps = 0;
    int upload(int sw, int sh, int dw, int dh, float support, int min_taps, hipStream_t st) {
        auto axis = [&](int src, int dst, std::vector<int>& L, std::vector<float>& Wt, int& taps) {
            std::vector<std::vector<float>> ws(dst);
            L.resize(dst);
            taps = min_taps;
            std::vector<float> w(4096);
            for (int o = 0; o < dst; o++) {
                const int n = ip_axis(src, dst, o, support, &L[o], w.data());
                ws[o].assign(w.begin(), w.begin() + n);
                taps = std::max(taps, n);
            }
            Wt.assign((size_t)dst * taps, 0.0f);
            for (int o = 0; o < dst; o++)
                for (size_t k = 0; k < ws[o].size(); k++) Wt[(size_t)o * taps + k] = ws[o][k];
        };
        std::vector<int> lx, ly;
        std::vector<float> wx, wy;
        axis(sw, dw, lx, wx, xtaps);
        axis(sh, dh, ly, wy, ytaps);
        if (xtaps > 64 || ytaps > 64) return fail(SIFT_MI_EUNSUPPORTED, "resize ratio too large (> 64 taps)");
        CHK(xl.ensure(dw));
        CHK(yl.ensure(dh));
        CHK(xw.ensure(wx.size()));
        CHK(yw.ensure(wy.size()));
        HIPCHK(hipMemcpyAsync(xl.p, lx.data(), dw * sizeof(int), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(yl.p, ly.data(), dh * sizeof(int), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(xw.p, wx.data(), wx.size() * sizeof(float), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(yw.p, wy.data(), wy.size() * sizeof(float), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        return 0;
    }
    IpResizeTab tab() const { return IpResizeTab{xl.p, xw.p, yl.p, yw.p}; }
    void release() {
        xl.release();
        yl.release();
        xw.release();
        yw.release();
    }
};

struct ResizeTabDev {
    DevBuf<int> xofs, yofs;
    DevBuf<float> xa0, xa1, ya0, ya1;
    ResizeTab tab{};
    int upload(int sw, int sh, int dw, int dh, hipStream_t st) {
        std::vector<int> xo, yo;
        std::vector<float> xa, xb, ya, yb;
        int xmax = 0, ymax = 0;
        cv_linear_coeffs(sw, dw, xo, xa, xb, &xmax);
        cv_linear_coeffs(sh, dh, yo, ya, yb, &ymax);
        CHK(xofs.ensure(dw));
        CHK(xa0.ensure(dw));
        CHK(xa1.ensure(dw));
        CHK(yofs.ensure(dh));
        CHK(ya0.ensure(dh));
        CHK(ya1.ensure(dh));
        HIPCHK(hipMemcpyAsync(xofs.p, xo.data(), dw * sizeof(int), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(xa0.p, xa.data(), dw * sizeof(float), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(xa1.p, xb.data(), dw * sizeof(float), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(yofs.p, yo.data(), dh * sizeof(int), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ya0.p, ya.data(), dh * sizeof(float), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ya1.p, yb.data(), dh * sizeof(float), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));  // host vectors go out of scope
        tab.xofs = xofs.p;
        tab.xa0 = xa0.p;
        tab.xa1 = xa1.p;
        tab.yofs = yofs.p;
        tab.ya0 = ya0.p;
        tab.ya1 = ya1.p;
        tab.xmax = xmax;
        return 0;
    }
    void release() {
        xofs.release();
        yofs.release();
        xa0.release();
        xa1.release();
        ya0.release();
        ya1.release();
    }
};

// Frame geometry + pyramid arena for `chunk` frames of w x h.
struct Plan {
    uint32_t w = 0, h = 0, chunk = 0;
    int n_oct = 0;
    int max_oct = 0;  // the context's max_octaves the plan was built for
    std::vector<int> ow, oh, opitch;
    std::vector<size_t> P;           // floats per octave image plane (pitch * H)
    std::vector<size_t> px;          // real pixels per octave image (W * H)
    std::vector<size_t> goff, doff;  // float offsets of octave arenas
    DevBuf<float> arena[2];          // per lane: [G_0 | D_0 | G_1 | D_1 ...], each chunk-major
    size_t arena_floats = 0;
    int profile = SIFT_MI_PROFILE_OPENCV;
    ResizeTabDev seed_tab;  // OpenCV profile
    IpTabDev seed_iptab;    // Imageproc profile
    DevBuf<const float*> d_gauss[2], d_dog[2];  // per lane
    DevBuf<size_t> d_gstride, d_dstride;
    DevBuf<int> d_ow, d_oh, d_opitch;
    BlurTaps seed_taps{};
    int seed_r = 0;
    BlurTaps oct_taps[kImagesPerOctave]{};
    int oct_r[kImagesPerOctave]{};
    uint64_t algo_bytes_per_frame = 0;

    float* gauss(int o, int lane = 0) { return arena[lane].p + goff[o]; }
    float* dog(int o, int lane = 0) { return arena[lane].p + doff[o]; }
    size_t gstride(int o) const { return (size_t)kImagesPerOctave * P[o]; }
    size_t dstride(int o) const { return (size_t)kDogPerOctave * P[o]; }

    void release() {
        for (int l = 0; l < 2; l++) {
            arena[l].release();
            d_gauss[l].release();
            d_dog[l].release();
        }
        arena_floats = 0;
        seed_tab.release();
        seed_iptab.release();
        d_gstride.release();
        d_dstride.release();
        d_ow.release();
        d_oh.release();
        d_opitch.release();
        w = h = chunk = 0;
        n_oct = 0;
    }
};

}  // namespace

// Per-chunk state that outlives the enqueue: device counters, final outputs
// and the events of one in-flight chunk.  Two slots alternate, so chunk k+1's
// kernels run while the host waits for chunk k and copies its results out.
struct Slot {
    // [0] candidates [1] extrema [2] keypoints [3] outputs [4..4+F) frame starts
    // [4+F..4+2F) per-frame outputs [4+2F..4+2F+kTailWords) the tail
    // region's counters (early)
    // [4+2F+kTailWords..+kDescWorkWords) descriptor work queues
    DevBuf<uint32_t> counters;
    PinBuf<uint32_t> h_counts;
    DevBuf<OutKp> out_kp;
    DevBuf<uint8_t> out_desc;
    DevBuf<uint64_t> out_key;
    DevBuf<uint8_t> desc_kp;  // one-frame calls: descriptors in keypoint index order (Slot::desc_first)
    hipEvent_t ev[7] = {};   // stage boundaries on the compute stream (ev[6] = chunk done)
    hipEvent_t copied = {};  // results copied to the host (copy stream)
    hipEvent_t ordered = {};  // desc_first: the ordering stage done (lane 1's stream)
    bool pending_copy = false;
    bool detected = false;  // this chunk's detection is enqueued (stage overlap: inside the pyramid)
    uint32_t fused_mask = 0;  // octaves detected by k_blur_detect (with their blur 5) in the pyramid
    bool graph_run = false;   // the chunk was a graph replay: only ev[0] / ev[6] were recorded
    // ev[0..5] recorded: the one-lane mode times the stages (a marker packet
    // costs ~7 us of the stream's timeline; two-lane calls record only ev[6])
    bool staged = false;
    hipEvent_t oriented = {};  // desc_first: the keypoints are oriented (fork to lane 1's stream)
    // single-chunk calls with octave overlap: refinement + orientation of the
    // octaves below the tail run on the aux stream beside the tail (early),
    // the tail octaves' candidates / extrema in their own region (cand_b,
    // ext_b; counters at counters[4 + 2m + 0 / 1])
    bool early = false;
    // one-frame early calls without a limit: the descriptors are computed in
    // keypoint index order (desc_kp) while lane 1's stream orders the
    // keypoints; k_gather_out then writes the outputs in emission order
    bool desc_first = false;
    // early, two lanes: the aux stream's join event (oct_ev[lane][kTailMaxOct])
    // is recorded but the lane stream has not waited for it yet; the keypoint
    // stage either waits first or, with desc_first, runs the descriptors on
    // the aux stream itself (no cross-stream hop before them)
    bool join_pending = false;
    // the chunk's counter reset is launched right after the seed pass
    // (run_pyramid) instead of before it: the seed does not touch them
    bool init_pending = false;
    uint32_t bcb = 0;
    DevBuf<uint64_t> cand_b;
    DevBuf<ExtRec> ext_b;
    uint32_t m = 0, frame_base = 0, cap_frames = 0;
    uint32_t bc = 0, be = 0, bk = 0;  // candidate / extremum / keypoint bounds used by this chunk
    // detection / description buffers of this slot's lane (the slot's chunks
    // run in its lane's stream order)
    DevBuf<uint64_t> cand;
    DevBuf<ExtRec> ext;
    DevBuf<KpRec> kp;
    DevBuf<uint64_t> keys_a, keys_b;
    DevBuf<uint32_t> vals_a, vals_b, fin;
    DevBuf<uint8_t> sort_tmp;
    DevBuf<uint32_t> seg_off, out_off;
    DevBuf<uint8_t> use_resp;
    void release_bufs() {
        cand.release();
        ext.release();
        cand_b.release();
        ext_b.release();
        kp.release();
        keys_a.release();
        keys_b.release();
        vals_a.release();
        vals_b.release();
        fin.release();
        sort_tmp.release();
        seg_off.release();
        out_off.release();
        use_resp.release();
    }
};

struct sift_mi_ctx {
    int device = 0;
    sift_mi_profile profile = SIFT_MI_PROFILE_OPENCV;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;  // compute stream (own or the caller's)
    hipStream_t cstream = nullptr; // device->host result copies
    hipStream_t own2 = nullptr;    // compute stream of pipeline lane 1 (lane 0 runs on `stream`)
    hipStream_t aux[2] = {};       // per lane: blurs 4, 5 of each octave beside the next octave
    hipStream_t aux2 = nullptr;    // lane 0: blurs 4, 5 of octaves >= 1 while octave 0's fused pass runs
    hipEvent_t aux2_join = nullptr;
    hipStream_t dec = nullptr;     // JPEG batch decoding: a high-priority stream (its own hardware queue)
    hipEvent_t oct_ev[2][kTailMaxOct + 1] = {};  // per lane: octave o's G_3 done / aux joined
    bool lanes_busy = false;       // this call keeps both pipeline lanes busy (no octave overlap then)
    PathOpts opts;                 // kernel-path switches (sift_mi_set_path_option)
    hipEvent_t fork = nullptr;     // orders lane 1 after / before the caller's stream
    int lanes = 2;                 // pipeline lanes (sift_mi_set_pipeline_lanes)
    uint32_t chunk_override = 0;
    int keep_on_device = 0;
    uint32_t band_r = 0, band_n = 1;  // row band of the keypoint stages (sift_mi_set_row_band)
    JpegBatchCache jpeg;              // sift_mi_decode_jpeg_batch buffers
    DevBuf<uint32_t> band_flag;       // a refinement left the restricted rows (row bands)
    bool band_restricted = false;     // this call computes only the band's pyramid rows
    bool band_whole = false;          // re-run of a band on the whole-frame pyramid
    int exact_descriptors = 0;
    int max_octaves = 0;                    // sift_mi_set_max_octaves (0: the crate's formula)
    int count_samples = 0;                  // sift_mi_set_sample_counting (measurement only)
    DevBuf<unsigned long long> samples;     // [0, 8): orientation, [8, 16): descriptor sample counters
    Plan plan;
    DevBuf<uint8_t> staging;  // host-sourced frames
    Slot slot[2];  // slot = pipeline lane: chunk k runs on lane k & 1
    int last_slot = 0;
    // per-frame high-water marks that size the next chunk's bounds
    double pf_cand = 0, pf_ext = 0, pf_kp = 0;
    double pf_cand_b = 0;  // the tail octaves' candidates / extrema (Slot::early)
    // device results of a whole batch (keep_on_device), concatenated in frame order
    DevBuf<OutKp> r_kp;
    DevBuf<uint8_t> r_desc;
    DevBuf<uint64_t> r_key;
    // host results (pinned)
    PinBuf<OutKp> h_kp;
    PinBuf<uint8_t> h_desc;
    PinBuf<uint64_t> h_key;
    size_t n_result = 0;
    bool have_result = false;
    bool have_pyramid = false;  // single-frame precompute state
    size_t dev_result_n = 0;
    int res_slot = -1;  // >= 0: the last call's device results are that slot's outputs (one chunk, no copy)
    int batch_arena = -1;     // >= 0: the last batch call ran as one chunk in this arena (read-back)
    // Single-chunk calls as a HIP graph (PathOpts::graph): the call's ~40
    // launches are captured the second time an identical call (same frames
    // pointer, geometry, bounds, modes, buffers) is seen, then replayed with
    // one hipGraphLaunch.
    struct GraphKey {
        PathOpts opts;  // the switches decide what is captured
        const uint8_t* frames;
        size_t frame_pitch, stride;
        uint32_t m, w, h, bc, be, bk, bcb;
        int64_t limit;
        uint64_t gen;
        int keep, exact, samples, lanes, prof, maxo;
        hipStream_t st;
        bool operator==(const GraphKey& o) const { return std::memcmp(this, &o, sizeof o) == 0; }
    };
    GraphKey gkey{}, gseen{};
    bool gkey_ok = false, gseen_ok = false;
    bool g_early = false;      // the captured chunk's host-side flags
    uint32_t g_fused = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    uint32_t batch_frames = 0;
    sift_mi_stats stats{};
};

namespace {

// slot si's stream and pyramid arena: its own lane with two lanes, else lane 0
hipStream_t lane_stream(sift_mi_ctx* c, int si) { return (si == 1 && c->lanes == 2) ? c->own2 : c->stream; }
int arena_of(const sift_mi_ctx* c, int si) { return c->lanes == 2 ? si : 0; }

int sync_lanes(sift_mi_ctx* c) {
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->own2));
    for (auto& a : c->aux) HIPCHK(hipStreamSynchronize(a));
    if (c->aux2) HIPCHK(hipStreamSynchronize(c->aux2));
    return 0;
}

int set_device(sift_mi_ctx* c) {
    HIPCHK(hipSetDevice(c->device));
    return 0;
}

uint32_t auto_chunk(const Plan& p_probe_w_h, uint32_t w, uint32_t h, uint32_t n, int mode, double avail_bytes) {
    (void)p_probe_w_h;
    // mode 1 (path option chunk_mode, the default since round 6): twice the
    // caps below and no forced second chunk -- a 128-frame 1080p call is one
    // chunk.  Against mode 0's two overlapped 64-frame chunks: 34.49-34.53 vs
    // 34.12-34.43 M keypoints/s, VGA 256 30.32-30.43 vs 30.00-30.21 M
    // (profiles/r06_ab_runs.md): each stage's launches twice as large beat
    // the overlap of two half-size chunks.
    // Up to ~32 GB of pyramid per chunk (two lanes: ~64 GB of the 288 GB HBM)
    // and at most kMaxChunk frames, in balanced chunks, at least two when the
    // batch has two frames (the lanes overlap consecutive chunks).  Bigger
    // chunks amortise each stage's launch tail: 1080p, 128 frames per call,
    // measured 22.8 M keypoints/s at 32-frame chunks, 23.9 M at 64.
    double sum_p = 0;
    uint32_t ow = 2 * w, oh = 2 * h;
    const int no = n_octaves_for(w, h);
    for (int o = 0; o < no; o++) {
        sum_p += (double)ow * oh;
        ow /= 2;
        oh /= 2;
    }
    const double per_frame = 44.0 * sum_p;
    const double scale = mode == 1 ? 2.0 : 1.0;
    uint32_t cmax = (uint32_t)std::max(1.0, std::floor(scale * 32e9 / per_frame));
    // and at most 40% of the device memory this context could use (free +
    // its own arenas) per chunk: the two lanes' arenas stay below 80% however
    // much other work holds (no effect on an idle 288 GB MI355X)
    if (avail_bytes > 0) cmax = std::min<uint32_t>(cmax, (uint32_t)std::max(1.0, std::floor(0.4 * avail_bytes / per_frame)));
    // and ~531 M seed pixels (64 frames at 1080p): smaller frames get more
    // frames per chunk, so their octave launches are as large (VGA: 256
    // frames in two chunks of 128 instead of four of 64)
    const double seed_px = 4.0 * w * h;
    cmax = std::min<uint32_t>(cmax, (uint32_t)std::max(1.0, std::floor(scale * 64.0 * 3840.0 * 2160.0 / seed_px)));
    cmax = std::min<uint32_t>(cmax, 256);
    uint32_t k = std::max<uint32_t>((n + cmax - 1) / cmax, (n >= 2 && mode != 1) ? 2u : 1u);  // chunks
    return std::max<uint32_t>(1, (n + k - 1) / k);
}

// Pyramid arena of one pipeline lane (chunks alternate between two lanes so
// that one chunk's kernels overlap the other's) and its device pointer tables.
int ensure_lane(sift_mi_ctx* c, int lane) {
    Plan& p = c->plan;
    if (p.arena[lane].p && p.d_gauss[lane].p) return 0;
    CHK(p.arena[lane].ensure(p.arena_floats));
    std::vector<const float*> gp(p.n_oct), dp(p.n_oct);
    for (int o = 0; o < p.n_oct; o++) {
        gp[o] = p.gauss(o, lane);
        dp[o] = p.dog(o, lane);
    }
    CHK(p.d_gauss[lane].ensure(p.n_oct));
    CHK(p.d_dog[lane].ensure(p.n_oct));
    HIPCHK(hipMemcpyAsync(p.d_gauss[lane].p, gp.data(), p.n_oct * sizeof(float*), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(p.d_dog[lane].p, dp.data(), p.n_oct * sizeof(float*), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int ensure_plan(sift_mi_ctx* c, uint32_t w, uint32_t h, uint32_t chunk) {
    Plan& p = c->plan;
    if (p.w == w && p.h == h && p.chunk >= chunk && p.arena[0].p && p.profile == (int)c->profile &&
        p.max_oct == c->max_octaves)
        return 0;
    c->batch_arena = -1;  // the arenas are re-sized or re-planned: no batch read-back
    if (!(p.w == w && p.h == h && p.profile == (int)c->profile && p.max_oct == c->max_octaves)) {
        p.release();
        // per-frame stage high-water marks belong to a frame size
        c->pf_cand = c->pf_ext = c->pf_kp = 0;
        c->pf_cand_b = 0;
    }
    p.profile = (int)c->profile;
    const bool ip = c->profile == SIFT_MI_PROFILE_IMAGEPROC;
    p.w = w;
    p.h = h;
    p.chunk = chunk;
    p.n_oct = n_octaves_for(w, h);
    // labelled extension (sift_mi_set_max_octaves): fewer octaves than the
    // crate's formula (src/lib.rs:133-134); the kept octaves are unchanged
    if (c->max_octaves > 0) p.n_oct = std::min(p.n_oct, c->max_octaves);
    p.max_oct = c->max_octaves;
    p.ow.assign(p.n_oct, 0);
    p.oh.assign(p.n_oct, 0);
    p.opitch.assign(p.n_oct, 0);
    p.P.assign(p.n_oct, 0);
    p.px.assign(p.n_oct, 0);
    p.goff.assign(p.n_oct, 0);
    p.doff.assign(p.n_oct, 0);
    int ow = 2 * (int)w, oh = 2 * (int)h;
    size_t total = 0;
    uint64_t sum_p = 0;
    for (int o = 0; o < p.n_oct; o++) {
        if (ow < 1 || oh < 1) return fail(SIFT_MI_EINVAL, "image too small for the octave count");
        p.ow[o] = ow;
        p.oh[o] = oh;
        p.opitch[o] = (ow + 63) & ~63;  // 256-B aligned rows
        p.P[o] = (size_t)p.opitch[o] * oh;
        p.px[o] = (size_t)ow * oh;
        sum_p += p.px[o];
        p.goff[o] = total;
        total += (size_t)chunk * kImagesPerOctave * p.P[o];
        p.doff[o] = total;
        // D_0..D_4 for ONE frame: only precompute_images materialises the
        // DoG (run_pyramid's `full`, one frame on lane 0); the batch path
        // forms D where it reads it.  (Rounds 1-5 reserved them per chunk
        // frame: 5 / 11 of the arena never written -- 28 GB per lane at 128 x
        // 1080p.)
        total += (size_t)kDogPerOctave * p.P[o];
        total = (total + 63) & ~(size_t)63;  // 256-B aligned octave arenas
        if (o + 1 < p.n_oct) {
            // nearest 1/2 must be source pixel (2x, 2y) (OpenCV INTER_NEAREST)
            // or (2x + 1, 2y + 1) (image Nearest) for the fused epilogue
            const int par = ip ? 1 : 0;
            for (int axis = 0; axis < 2; axis++) {
                const int src = axis ? oh : ow, dst = src / 2;
                std::vector<int> xo;
                if (ip) {
                    xo.resize(dst);
                    float wt[8];
                    for (int i = 0; i < dst; i++) {
                        const int n = ip_axis(src, dst, i, 0.0f, &xo[i], wt);
                        if (n != 1) return fail(SIFT_MI_EUNSUPPORTED, "nearest 1/2 with more than one tap");
                    }
                } else {
                    cv_nearest_ofs(src, dst, xo);
                }
                for (int i = 0; i < dst; i++)
                    if (xo[i] != 2 * i + par) return fail(SIFT_MI_EUNSUPPORTED, "nearest 1/2 offset is not 2x (+1)");
            }
        }
        ow /= 2;
        oh /= 2;
    }
    // algorithmic bytes: the u8 frame read once and every
    // image of PrecomputedImages (G_0..G_5, D_0..D_4: 44 B per octave pixel)
    // written once -- the fixed yardstick for every path.  The batch path
    // itself writes only G_0..G_5 and forms D where detection reads it, so
    // its pyramid kernels move ~44 B per octave pixel counting their reads
    // (DESIGN.md 3.1).
    p.algo_bytes_per_frame = (uint64_t)w * h + 44ull * sum_p;
    p.arena_floats = total;
    for (int l = 0; l < 2; l++) {  // a larger chunk re-sizes both lanes
        p.arena[l].release();
        p.d_gauss[l].release();
        p.d_dog[l].release();
    }
    hipStream_t st = c->stream;
    if (ip)
        CHK(p.seed_iptab.upload((int)w, (int)h, 2 * (int)w, 2 * (int)h, 1.0f, kIpTaps, st));
    else
        CHK(p.seed_tab.upload((int)w, (int)h, 2 * (int)w, 2 * (int)h, st));
    if (ip && (p.seed_iptab.xtaps > kIpTaps || p.seed_iptab.ytaps > kIpTaps))
        return fail(SIFT_MI_EUNSUPPORTED, "2x Triangle upsample with more than 3 taps");
    std::vector<size_t> gs(p.n_oct), ds(p.n_oct);
    for (int o = 0; o < p.n_oct; o++) {
        gs[o] = p.gstride(o);
        ds[o] = p.dstride(o);
    }
    CHK(p.d_gstride.ensure(p.n_oct));
    CHK(p.d_dstride.ensure(p.n_oct));
    HIPCHK(hipMemcpyAsync(p.d_dstride.p, ds.data(), p.n_oct * sizeof(size_t), hipMemcpyHostToDevice, st));
    CHK(p.d_ow.ensure(p.n_oct));
    CHK(p.d_oh.ensure(p.n_oct));
    CHK(p.d_opitch.ensure(p.n_oct));
    HIPCHK(hipMemcpyAsync(p.d_gstride.p, gs.data(), p.n_oct * sizeof(size_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(p.d_ow.p, p.ow.data(), p.n_oct * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(p.d_oh.p, p.oh.data(), p.n_oct * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(p.d_opitch.p, p.opitch.data(), p.n_oct * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    // P::gaussian_blur(img, sigma: f64); ImageprocProcessing passes sigma as f32
    p.seed_r = ip ? ip_blur_taps((float)seed_sigma(), &p.seed_taps) : cv_blur_taps(seed_sigma(), &p.seed_taps);
    double sig[kImagesPerOctave];
    octave_sigmas(sig);
    for (int s = 1; s < kImagesPerOctave; s++)
        p.oct_r[s] = ip ? ip_blur_taps((float)sig[s], &p.oct_taps[s]) : cv_blur_taps(sig[s], &p.oct_taps[s]);
    return ensure_lane(c, 0);
}

// Detection of octaves [o0, o1) of frames [f0, f0 + nf) of slot si's chunk:
// one multi-octave k_detect_rows launch (candidates into the slot's buffer,
// bounded by S.bc).
int launch_detection(sift_mi_ctx* c, int si, uint32_t f0, uint32_t nf, int o0, int o1, hipStream_t st,
                     uint64_t* cand = nullptr, uint32_t* counter = nullptr, uint32_t cap = 0);
// refinement of the candidates (cand, *n_cand <= cand_cap) into ext (*counter,
// cap), and orientation of those extrema into the slot's keypoints
// (counter_hi / n_ext_hi: two-ended extremum append, RefineLaunch::counter_hi)
int launch_refine_stage(sift_mi_ctx* c, int si, const uint64_t* cand, const uint32_t* n_cand, uint32_t cand_cap,
                        ExtRec* ext, uint32_t* counter, uint32_t cap, hipStream_t st, uint32_t* counter_hi = nullptr);
int launch_orient_stage(sift_mi_ctx* c, int si, const ExtRec* ext, const uint32_t* n_ext, uint32_t ext_cap,
                        uint32_t kp_cap, hipStream_t st, const uint32_t* n_ext_hi = nullptr);

// Row bands with a restricted pyramid: rows a refined keypoint may drift from
// its detection row and still be exact without a re-run, and the rows its
// orientation / descriptor patch reaches (radius <= 16 / 39, plus the
// gradient's neighbour row).
constexpr int kBandDrift = 24, kBandPatch = 41;



// ---------------------------------------------------------------------------
// Stage 1: Gaussian scale space + DoG for n frames (device-resident u8)
// ---------------------------------------------------------------------------
// full: materialise every image (precompute_images / read_dog); the batch
// path writes G_0..G_5 only: detection and refinement form D_s = G_{s+1} - G_s
// where they read it (detect.hip), 16 B per octave pixel less than writing
// the DoG planes and reading them back.
// Octave overlap: octave o + 1 needs only G_3 of octave o (its G_0 is
// written by blur 3), so blurs 4, 5 of each octave run on the lane's aux
// stream beside the next octave's blurs (without: 0.779 vs 0.62 ms per 1080p
// frame, round 4).  Tried and measured slower or no faster (round 3, DESIGN.md
// 3.10): the chunk's
// frames split in two halves on the two streams; seed + octave 0 in
// sub-batches of 2-32 frames for Infinity Cache reuse; a second aux stream;
// only octaves 0 .. k-1 (k = 1, 2, 3) on the aux stream.
// detect_slot >= 0 (stage overlap): the detection of the chunk in that slot
// is launched from here, each part's octaves as soon as their blurs are done.
// cand_slot >= 0 (the keypoint stages follow): octaves whose blur 5 and
// detection run as one pass (k_blur_detect) append their candidates to that
// slot's buffer from here, whatever detect_slot is (Slot::fused_mask).
constexpr int kTailWords = 4;        // Slot counters after the per-frame plan: cand_b, ext_b counts, (unused),
                                     // the two-ended ext's back count (PathOpts::large_first)
void flush_chunk_init(sift_mi_ctx* c, int si);

int run_pyramid(sift_mi_ctx* c, int lane, const uint8_t* d_frames, size_t frame_pitch, size_t row_stride,
                uint32_t n, bool full, int detect_slot = -1, int cand_slot = -1) {
    Plan& p = c->plan;
    if (full && n != 1) return fail(SIFT_MI_EINVAL, "the DoG planes are materialised for one frame");
    hipStream_t st = lane_stream(c, lane);
    lane = arena_of(c, lane);
    hipStream_t aux = c->aux[lane];
    hipStream_t aux2 = lane == 0 ? c->aux2 : nullptr;
    // row bands (sift_mi_set_row_band): the rows of every Gaussian the band's
    // keypoint stages read, propagated back through the blur chain and the
    // octave downsampling.  Detection covers octave rows [H*r/n, H*(r+1)/n);
    // around them a margin of kBandDrift + 1 + kBandPatch rows.  A
    // refinement that reads, or an accepted keypoint whose patch reaches,
    // beyond it sets band_flag (k_refine) and the host re-runs the band on
    // the whole pyramid.
    std::vector<int> rlo((size_t)p.n_oct * kImagesPerOctave, 0), rhi((size_t)p.n_oct * kImagesPerOctave, 0);
    c->band_restricted = c->band_n > 1 && !full && !c->band_whole && p.profile == (int)SIFT_MI_PROFILE_OPENCV;
    int seed_y0 = 0, seed_y1 = 0;
    if (c->band_restricted) {
        int need_lo = 0, need_hi = 0;  // octave o + 1's G_0 rows, in octave o + 1 coordinates
        for (int o = p.n_oct - 1; o >= 0; o--) {
            const int H = p.oh[o], M = kBandDrift + 1 + kBandPatch;
            const int blo = (int)((uint64_t)H * c->band_r / c->band_n), bhi = (int)((uint64_t)H * (c->band_r + 1) / c->band_n);
            int* lo = &rlo[(size_t)o * kImagesPerOctave];
            int* hi = &rhi[(size_t)o * kImagesPerOctave];
            for (int s = 0; s < kImagesPerOctave; s++) {
                lo[s] = blo - 1 - M;
                hi[s] = bhi + 1 + M;
            }
            if (o + 1 < p.n_oct && need_hi > need_lo) {  // nearest 1/2 of G_3: row 2y or 2y + 1
                lo[3] = std::min(lo[3], 2 * need_lo);
                hi[3] = std::max(hi[3], 2 * need_hi + 1);
            }
            for (int s = kImagesPerOctave - 1; s >= 1; s--) {
                lo[s - 1] = std::min(lo[s - 1], lo[s] - p.oct_r[s]);
                hi[s - 1] = std::max(hi[s - 1], hi[s] + p.oct_r[s]);
            }
            for (int s = 0; s < kImagesPerOctave; s++) {
                lo[s] = std::max(lo[s], 0);
                hi[s] = std::min(hi[s], H);
            }
            need_lo = lo[0];
            need_hi = hi[0];
        }
        seed_y0 = rlo[0];
        seed_y1 = std::max(rhi[0], rlo[0] + 1);
    }
    // the small octaves from o_tail on: one k_octave_tail launch
    // (PathOpts::tail = 0: per-blur launches for every octave)
    const PathOpts& po = c->opts;
    const int tail_slot = cand_slot;  // the chunk's slot
    int o_tail = p.n_oct;
    if (po.tail && p.n_oct <= kTailMaxOct) o_tail = tail_octave_start(p.ow.data(), p.oh.data(), p.n_oct, p.oct_r);
    uint64_t bytes = p.algo_bytes_per_frame;  // per frame, SURVEY.md 8(d)
    if (c->band_restricted) {
        // the same yardstick over the rows this band computes: 4 B per pixel
        // of each of its 6 Gaussian rows and 5 DoG rows, plus the input rows
        // the seed reads; the tail launch computes its octaves whole
        double b = (double)p.w * std::min<int>((int)p.h, (seed_y1 - seed_y0 + 1) / 2 + 2);
        for (int o = 0; o < p.n_oct; o++) {
            double rows = 0;
            for (int s = 0; s < kImagesPerOctave; s++) {
                const int r = o >= o_tail ? p.oh[o]
                                          : std::max(0, rhi[(size_t)o * kImagesPerOctave + s] -
                                                            rlo[(size_t)o * kImagesPerOctave + s]);
                rows += (s < kDogPerOctave ? 2.0 : 1.0) * r;
            }
            b += 4.0 * p.ow[o] * rows;
        }
        bytes = (uint64_t)b;
    }
    uint64_t launches = 0;
    // blur s of octave o for frames [f0, f0 + nf)
    auto blur_launch = [&](int o, int s, uint32_t f0, uint32_t nf) {
        float* G = p.gauss(o, lane) + (size_t)f0 * p.gstride(o);
        const size_t P = p.P[o];
        BlurLaunch B{};
        B.src = G + (size_t)(s - 1) * P;
        B.src_img_stride = p.gstride(o);
        B.dst = G + (size_t)s * P;
        B.dst_img_stride = p.gstride(o);
        if (s == 3 && o + 1 < p.n_oct) {
            B.nxt = p.gauss(o + 1, lane) + (size_t)f0 * p.gstride(o + 1);
            B.nxt_img_stride = p.gstride(o + 1);
            B.pitch_n = p.opitch[o + 1];
            B.wn = p.ow[o + 1];
            B.hn = p.oh[o + 1];
        }
        B.W = p.ow[o];
        B.H = p.oh[o];
        B.pitch = p.opitch[o];
        B.n_img = (int)nf;
        B.taps = p.oct_taps[s];
        B.profile = p.profile;
        if (c->band_restricted) {
            B.y0 = rlo[(size_t)o * kImagesPerOctave + s];
            B.y1 = std::max(rhi[(size_t)o * kImagesPerOctave + s], B.y0 + 1);
        }
        return B;
    };
    // the seed and blur 1 ran as one pass (k_seed_pair): octave 0 continues
    // at blur 2, as the (2, 3) pair
    bool seed_pair = false;
    // frames [f0, f0 + nf): seed, octave chain, tail (and their detection) on
    // stream sm; ov: blurs 4, 5 of each octave on the aux stream
    auto seed = [&](uint32_t f0, uint32_t nf, hipStream_t sm) -> int {
        SeedLaunch S{};
        S.frames = d_frames + (size_t)f0 * frame_pitch;
        S.frame_pitch = frame_pitch;
        S.row_stride = row_stride;
        S.sh = (int)p.h;
        S.sw = (int)p.w;
        S.tab = p.seed_tab.tab;
        S.iptab = p.seed_iptab.tab();
        S.profile = p.profile;
        S.dst = p.gauss(0, lane) + (size_t)f0 * p.gstride(0);
        S.dst_img_stride = p.gstride(0);
        S.W = p.ow[0];
        S.H = p.oh[0];
        S.pitch = p.opitch[0];
        S.n_img = (int)nf;
        S.taps = p.seed_taps;
        S.y0 = seed_y0;
        S.y1 = seed_y1;
        // the chunk's counter reset rides on the seed pass (its first workgroup)
        Slot* is = (tail_slot >= 0 && f0 == 0 && c->slot[tail_slot].init_pending) ? &c->slot[tail_slot] : nullptr;
        if (is) {
            S.init_cnt = is->counters.p;
            S.init_m = (int)is->m;
            S.init_words = kDescWorkWords + kTailWords;
        }
        // G_0 and G_1 in one pass where it applies (whole planes: not for a
        // restricted row band); G_0 is then never read back from HBM
        seed_pair = p.n_oct > 0 && launch_seed_pair(p.seed_r, p.oct_r[1], S, blur_launch(0, 1, f0, nf), sm, po) == 0;
        if (seed_pair && is) is->init_pending = false;
        if (seed_pair) {
            launches++;
            return 0;
        }
        if (launch_seed(p.seed_r, S, sm, po)) return fail(SIFT_MI_EUNSUPPORTED, "seed blur radius");
        launches++;
        return 0;
    };
    // octaves [o0, o1) of frames [f0, f0 + nf)
    // the launch that writes an octave's G_3 signals the aux stream's event
    // itself: no marker packet on the main stream (a separate event record
    // after it: 0.626 / 0.629 vs 0.616 / 0.619 ms per 1080p frame, round 4)
    // (not under stream capture: a kernel's stop event does not become a
    // graph dependency, so the captured aux work would not wait)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const bool ext_events = hipStreamIsCapturing(st, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone;
    // Octave 0's fused blur 5 + scan (k_blur_detect, the stage's longest
    // launch) is deferred until octave 1's G_3 is written, and the blurs 4, 5
    // of octaves >= 1 go to a second aux stream: octave 1's blur 3 then does
    // not run starved beside it (round 4: 3.4 ms at 0.35 TB/s), and the small
    // octaves' chain runs beside the long pass instead of after it.
    bool defer0 = false;           // octave 0's blur 5 is pending (deferral)
    BlurDetectLaunch defer_f{};
    bool used_aux2 = false;
    auto octaves = [&](uint32_t f0, uint32_t nf, int o0, int o1, hipStream_t sm, bool ov) -> int {
        hipStream_t s45 = sm;
        for (int o = o0; o < o1; o++) {
            bool g3_signalled = false;
            float* G = p.gauss(o, lane) + (size_t)f0 * p.gstride(o);
            float* D = full ? p.dog(o, lane) + (size_t)f0 * p.dstride(o) : nullptr;  // one frame's D (ensure_plan)
            const size_t P = p.P[o];
            // octave 0 after k_seed_pair starts at blur 2
            for (int s = (o == 0 && seed_pair) ? 2 : 1; s < kImagesPerOctave; s++) {
                if (s == 4 && ov) {
                    if (!g3_signalled) HIPCHK(hipEventRecord(c->oct_ev[lane][o], sm));
                    if (o >= 1 && defer0) {
                        // octave 1's G_3 is on its way: octave 0's fused pass
                        // now, the octaves from here on on the second aux stream
                        HIPCHK(hipStreamWaitEvent(aux, c->oct_ev[lane][o], 0));
                        if (launch_blur_detect(p.oct_r[5], defer_f, aux, po) != 0)
                            return fail(SIFT_MI_EHIP, "deferred blur-detect launch declined");
                        defer0 = false;
                    }
                    hipStream_t a = (o >= 1 && used_aux2) ? aux2 : aux;
                    HIPCHK(hipStreamWaitEvent(a, c->oct_ev[lane][o], 0));
                    s45 = a;
                }
                const BlurLaunch B = blur_launch(o, s, f0, nf);
                // blur 5 and the octave's detection in one pass (k_blur_detect:
                // G_4 / G_5 never read back by the extremum scan)
                if (s == kImagesPerOctave - 1 && cand_slot >= 0 && !full && c->band_n <= 1 && o < 32) {
                    Slot& S = c->slot[cand_slot];
                    BlurDetectLaunch F{};
                    F.gauss = G;
                    F.img_stride = p.gstride(o);
                    F.W = p.ow[o];
                    F.H = p.oh[o];
                    F.pitch = p.opitch[o];
                    F.octave = o;
                    F.n_img = (int)nf;
                    F.img_base = (int)f0;
                    F.profile = p.profile;
                    F.taps = p.oct_taps[s];
                    F.cand = S.cand.p;
                    F.counter = S.counters.p + 0;
                    F.cap = S.bc;
                    // defer octave 0's pass (see above) when it is fused and a
                    // later octave will take the second aux stream
                    if (o == 0 && ov && aux2 && o1 > 1 && blur_detect_applies(p.oct_r[s], F, po)) {
                        defer_f = F;
                        defer0 = true;
                        used_aux2 = true;
                        S.fused_mask |= 1u << o;
                        launches++;
                        continue;
                    }
                    if (launch_blur_detect(p.oct_r[s], F, s45, po) == 0) {
                        S.fused_mask |= 1u << o;
                        launches++;
                        continue;
                    }
                }
                // G_1, G_2 in one pass where the pair kernel applies
                // (k_blur2_strip: G_1 never read back from HBM); after the
                // seed pair, G_2, G_3 (and the next octave's base) instead
                // (the launch that writes G_3: blur 3, or the octave-0 (2, 3) pair)
                const bool g3 = ov && ext_events && (s == 3 || (s == 2 && o == 0 && seed_pair));
                if (g3) set_launch_done_event(c->oct_ev[lane][o]);
                int rc = 1;
                if (s == 1 || (s == 2 && o == 0 && seed_pair))
                    rc = launch_blur_pair(p.oct_r[s], p.oct_r[s + 1], B, blur_launch(o, s + 1, f0, nf), sm, po);
                if (rc == 0) {
                    g3_signalled = g3 && !launch_done_pending();
                    set_launch_done_event(nullptr);
                    launches++;
                    s++;
                    continue;
                }
                // a declined pair launched nothing: the event is still pending
                // for blur s itself only if that is blur 3
                if (g3 && s != 3) set_launch_done_event(nullptr);
                if (launch_blur(p.oct_r[s], B, s >= 4 ? s45 : sm, po)) {
                    set_launch_done_event(nullptr);
                    return fail(SIFT_MI_EUNSUPPORTED, "octave blur radius");
                }
                g3_signalled = g3_signalled || (g3 && s == 3 && !launch_done_pending());
                set_launch_done_event(nullptr);
                launches++;
            }
            // precompute_images: D_s = G_{s+1} - G_s, the same f32 subtraction
            // the keypoint stages form where they read the DoG
            if (full) launch_dog(G, P, p.gstride(o), D, p.dstride(o), p.ow[o], p.oh[o], p.opitch[o], (int)nf, s45);
        }
        return 0;
    };
    auto part = [&](uint32_t f0, uint32_t nf, hipStream_t sm, bool ov) -> int {
        bool aux_done_signalled = false;  // the aux orientation's launch carries the join event
        const bool early =
            detect_slot >= 0 && ov && o_tail > 0 && o_tail < p.n_oct && c->slot[detect_slot].bcb && po.early;
        CHK(seed(f0, nf, sm));
        if (tail_slot >= 0 && f0 == 0) flush_chunk_init(c, tail_slot);  // the chunk's counters, behind the seed
        CHK(octaves(f0, nf, 0, o_tail, sm, ov));
        if (defer0) {  // no later octave took it (cannot happen with o_tail > 1): launch it now
            HIPCHK(hipStreamWaitEvent(aux, c->oct_ev[lane][0], 0));
            if (launch_blur_detect(p.oct_r[5], defer_f, aux, po) != 0)
                return fail(SIFT_MI_EHIP, "deferred blur-detect launch declined");
            defer0 = false;
        }
        if (used_aux2) {  // the aux stream's later work (detection, join) follows the second's
            HIPCHK(hipEventRecord(c->aux2_join, aux2));
            HIPCHK(hipStreamWaitEvent(aux, c->aux2_join, 0));
        }
        if (o_tail < p.n_oct) {
            // whole octaves (a row band's restricted rows are a subset: rows
            // outside them depend only on rows outside them, so the exact rows
            // stay exact)
            TailLaunch T{};
            for (int o = 0; o < p.n_oct; o++) {
                T.gauss[o] = p.gauss(o, lane) + (size_t)f0 * p.gstride(o);
                T.gstride[o] = p.gstride(o);
                T.ow[o] = p.ow[o];
                T.oh[o] = p.oh[o];
                T.pitch[o] = p.opitch[o];
            }
            T.o0 = o_tail;
            T.n_oct = p.n_oct;
            T.n_img = (int)nf;
            T.profile = p.profile;
            for (int s = 1; s < kImagesPerOctave; s++) {
                T.r[s] = p.oct_r[s];
                T.taps[s] = p.oct_taps[s];
            }
            launch_octave_tail(T, sm);
            launches++;
            if (full)
                for (int o = o_tail; o < p.n_oct; o++)
                    launch_dog(p.gauss(o, lane) + (size_t)f0 * p.gstride(o), p.P[o], p.gstride(o),
                               p.dog(o, lane) + (size_t)f0 * p.dstride(o), p.dstride(o), p.ow[o], p.oh[o],
                               p.opitch[o], (int)nf, sm);
        }
        if (early) {
            // one chunk (octave overlap): the octaves below the tail are
            // detected, refined and oriented on the aux stream beside the tail
            // kernel; the tail octaves, after it, into a region of their own
            // (Slot::early; PathOpts::early = 0: off).  Tried and dropped: the
            // large octaves detected on lane 1's stream as each one's G_5
            // lands (0.634 vs 0.613-0.624 ms per 1080p frame: the scan then
            // competes with the blur chain for HBM instead of filling the
            // idle chip beside the one-workgroup tail kernel)
            Slot& S = c->slot[detect_slot];
            uint32_t* cnt = S.counters.p;
            uint32_t* cb = cnt + 4 + 2 * S.m;
            CHK(launch_detection(c, detect_slot, f0, nf, 0, o_tail, aux));
            // (PathOpts::large_first: two-ended extremum append, large
            // descriptor windows first)
            uint32_t* ext_hi = po.large_first ? cb + 3 : nullptr;
            CHK(launch_refine_stage(c, detect_slot, S.cand.p, cnt + 0, S.bc, S.ext.p, cnt + 1, S.be, aux, ext_hi));
            // the aux orientation signals the join event itself (no marker on
            // the aux stream's critical path; not under stream capture)
            if (ov && o_tail > 0 && ext_events) set_launch_done_event(c->oct_ev[lane][kTailMaxOct]);
            const int rc_o = launch_orient_stage(c, detect_slot, S.ext.p, cnt + 1, S.be, S.bk, aux, ext_hi);
            aux_done_signalled = ov && o_tail > 0 && ext_events && !launch_done_pending();
            set_launch_done_event(nullptr);
            CHK(rc_o);
            CHK(launch_detection(c, detect_slot, f0, nf, o_tail, p.n_oct, sm, S.cand_b.p, cb + 0, S.bcb));
            CHK(launch_refine_stage(c, detect_slot, S.cand_b.p, cb + 0, S.bcb, S.ext_b.p, cb + 1, S.bcb, sm));
            CHK(launch_orient_stage(c, detect_slot, S.ext_b.p, cb + 1, S.bcb, S.bk, sm));
            S.early = true;
        } else if (detect_slot >= 0) {
            // octaves [0, o_tail) are complete once their last blur is done:
            // with ov their detection runs on the aux stream beside the tail
            CHK(launch_detection(c, detect_slot, f0, nf, 0, o_tail, ov && o_tail > 0 ? aux : sm));
            CHK(launch_detection(c, detect_slot, f0, nf, o_tail, p.n_oct, sm));
        }
        if (ov && o_tail > 0) {  // join: the aux stream's work before what follows on sm
            if (!aux_done_signalled) HIPCHK(hipEventRecord(c->oct_ev[lane][kTailMaxOct], aux));
            // (not under stream capture: a capture keeps the plain join)
            if (early && c->lanes == 2 && ext_events)
                c->slot[detect_slot].join_pending = true;  // enqueue_keypoints joins
            else
                HIPCHK(hipStreamWaitEvent(sm, c->oct_ev[lane][kTailMaxOct], 0));
        }
        return 0;
    };
    // octave overlap only while the other lane is idle: with two chunks in
    // flight the other lane's kernels already fill the chip, and the extra
    // stream costs ~2% of batch throughput (30.4 vs 29.8 M keypoints/s,
    // 128 1080p frames, three A/B pairs)
    CHK(part(0, n, st, !c->lanes_busy && p.n_oct <= kTailMaxOct));
    HIPCHK(hipGetLastError());
    c->stats.pyramid_launches += launches;
    // pyramid_bytes is SURVEY.md 8(d)'s yardstick alone (W*H + 44*sum P_o per
    // frame).  The octaves whose extremum scan ran inside the stage
    // (k_blur_detect) are reported apart: what the reference's scan reads for
    // them, the five DoG planes once (20 B per octave pixel), so a caller can
    // state the fused stage's figure without mixing the two yardsticks.
    uint64_t scan = 0;
    if (cand_slot >= 0)
        for (int o = 0; o < p.n_oct && o < 32; o++)
            if ((c->slot[cand_slot].fused_mask >> o) & 1) scan += 20ull * p.px[o];
    c->stats.pyramid_bytes += bytes * n;
    c->stats.pyramid_scan_bytes += scan * n;
    return 0;
}

// ---------------------------------------------------------------------------
// Stages 2-4 for the m frames in the pyramid arena: detection, refinement,
// orientation, ordering, features_limit, descriptors -- enqueued on the
// compute stream with no host round trip.  Every stage reads its input count
// from device memory (Slot::counters) and is bounded by a host-side estimate
// (bc / be / bk); finalize_chunk detects a count above its bound and the chunk
// is re-run with larger bounds.
// ---------------------------------------------------------------------------
constexpr uint32_t kMaxChunk = 256;  // frames per chunk (one workgroup plans the output: k_limit_plan)

struct Bounds {
    uint32_t bc, be, bk;
};

Bounds chunk_bounds(sift_mi_ctx* c, uint32_t m) {
    uint64_t sum_p = 0;
    for (int o = 0; o < c->plan.n_oct; o++) sum_p += c->plan.px[o];
    auto est = [&](double pf, double floor_pf) {
        const double per = std::max(pf * 1.3, floor_pf);
        return (uint32_t)std::min<double>(std::ceil(per * m) + 1024, 0x7fffffff);
    };
    Bounds B;
    // first chunk: one candidate per 256 octave pixels; later chunks: 1.3x
    // the per-frame high-water mark.  PathOpts::bound_shrink = k (test path)
    // divides the first-chunk estimates by k and drops the slack, so every
    // chunk enqueued before a high-water mark exists overflows and re-runs.
    const double shrink = std::max(1, c->opts.bound_shrink);
    if (shrink > 1.0 && c->pf_cand == 0) {
        auto tiny = [&](double per) { return (uint32_t)std::max(1.0, std::ceil(per / shrink * m)); };
        B.bc = tiny(sum_p / 256.0);
        B.be = std::min(B.bc, tiny(sum_p / 512.0));
        B.bk = tiny(sum_p / 384.0);
        return B;
    }
    B.bc = est(c->pf_cand, c->pf_cand > 0 ? 64.0 : sum_p / 256.0);
    B.be = est(c->pf_ext, c->pf_ext > 0 ? 64.0 : sum_p / 512.0);
    B.bk = est(c->pf_kp, c->pf_kp > 0 ? 64.0 : sum_p / 384.0);
    B.be = std::min(B.be, B.bc);  // one extremum per candidate at most
    return B;
}

// Grows the shared buffers for bounds B (waits for in-flight work first when a
// buffer has to be reallocated).
// frames: the slot's frame capacity (the plan's chunk); m: this chunk's frames
int reserve_chunk(sift_mi_ctx* c, int si, const Bounds& B, uint32_t frames, uint32_t m) {
    Slot& S = c->slot[si];
    const uint32_t bcb = std::max<uint32_t>(2048, (uint32_t)std::min<double>(std::ceil(c->pf_cand_b * 1.3 * frames) + 1024, 1e9));
    const bool grow = B.bc > S.cand.cap || B.be > S.ext.cap || B.bk > S.kp.cap || B.bk > S.keys_a.cap ||
                      bcb > S.cand_b.cap || bcb > S.ext_b.cap ||
                      frames > S.seg_off.cap || B.bk > S.out_kp.cap ||
                      4 + 2 * frames + kDescWorkWords + kTailWords > S.counters.cap ||
                      (m == 1 && (size_t)B.bk * kDescSize > S.desc_kp.cap);
    if (grow) {
        HIPCHK(hipStreamSynchronize(lane_stream(c, si)));
        HIPCHK(hipStreamSynchronize(c->cstream));
        if (si == 0 && c->lanes == 2) HIPCHK(hipStreamSynchronize(c->own2));  // one-chunk calls' second stream
    }
    CHK(S.cand.ensure(B.bc));
    CHK(S.ext.ensure(B.be));
    // the tail octaves' own candidate / extremum region (Slot::early): a
    // 1.3x per-frame high-water mark, at least 2048
    S.bcb = std::max<uint32_t>(2048, (uint32_t)std::min<double>(std::ceil(c->pf_cand_b * 1.3 * frames) + 1024, 1e9));
    CHK(S.cand_b.ensure(S.bcb));
    CHK(S.ext_b.ensure(S.bcb));
    CHK(S.kp.ensure(B.bk));
    CHK(S.keys_a.ensure(B.bk));
    CHK(S.keys_b.ensure(B.bk));
    CHK(S.vals_a.ensure(B.bk));
    CHK(S.vals_b.ensure(B.bk));
    CHK(S.fin.ensure(B.bk));
    CHK(S.seg_off.ensure(frames));
    CHK(S.out_off.ensure(frames));
    CHK(S.use_resp.ensure(frames));
    CHK(S.counters.ensure(4 + 2 * frames + kDescWorkWords + kTailWords));
    CHK(S.h_counts.ensure(4 + 2 * frames + kTailWords));
    CHK(S.out_kp.ensure(B.bk));
    CHK(S.out_desc.ensure((size_t)B.bk * kDescSize));
    CHK(S.out_key.ensure(B.bk));
    if (m == 1) CHK(S.desc_kp.ensure((size_t)B.bk * kDescSize));  // Slot::desc_first
    return 0;
}

int img_bits_for(uint32_t m) {
    int b = 1;
    while ((1u << b) <= m) b++;  // strictly above the largest frame index: the padding key sorts last
    return b;
}

// Per-chunk state and zeroed counters of slot si, before any of its kernels
// (detection may start inside the pyramid: stage overlap).
void flush_chunk_init(sift_mi_ctx* c, int si) {
    Slot& S = c->slot[si];
    if (!S.init_pending) return;
    S.init_pending = false;
    launch_chunk_init(S.counters.p, (int)S.m, kDescWorkWords + kTailWords, lane_stream(c, si));  // + the tail region's words
}

int prepare_chunk(sift_mi_ctx* c, int si, uint32_t m, uint32_t frame_base, const Bounds& B, bool defer_init) {
    Slot& S = c->slot[si];
    hipStream_t st = lane_stream(c, si);
    S.m = m;
    S.frame_base = frame_base;
    S.cap_frames = m;
    S.bc = B.bc;
    S.be = B.be;
    S.bk = B.bk;
    S.detected = false;
    S.fused_mask = 0;
    S.graph_run = false;
    S.early = false;
    S.join_pending = false;
    (void)st;
    // stage counters, frame starts (~0), descriptor work queues
    S.init_pending = true;
    if (!defer_init) flush_chunk_init(c, si);
    HIPCHK(hipGetLastError());
    return 0;
}

int launch_detection(sift_mi_ctx* c, int si, uint32_t f0, uint32_t nf, int o0, int o1, hipStream_t st,
                     uint64_t* cand, uint32_t* counter, uint32_t cap) {
    Plan& p = c->plan;
    Slot& S = c->slot[si];
    DetectLaunch D{};
    D.n_img = (int)nf;
    D.img_base = (int)f0;  // frame index within the chunk (emission keys)
    D.cand = cand ? cand : S.cand.p;
    D.counter = cand ? counter : S.counters.p + 0;
    D.cap = cand ? cap : S.bc;
    int k = 0;
    for (int o = o0; o < o1; o++) {
        if (p.oh[o] < 2 * kImageBorder || p.ow[o] < 2 * kImageBorder) continue;  // src/lib.rs:315
        if ((S.fused_mask >> o) & 1) continue;  // detected with its blur 5 (k_blur_detect)
        DetectOctave& d = D.oct[k++];
        d.gauss = p.gauss(o, arena_of(c, si)) + (size_t)f0 * p.gstride(o);
        d.img_stride = p.gstride(o);
        d.W = p.ow[o];
        d.H = p.oh[o];
        d.pitch = p.opitch[o];
        d.octave = o;
        // row band: octave rows [H*r/n, H*(r+1)/n) -- the bands of one
        // octave partition its rows, so every candidate (keyed by its
        // initial octave, scale, y, x) belongs to exactly one band
        d.y_lo = (int)((uint64_t)p.oh[o] * c->band_r / c->band_n);
        d.y_hi = (int)((uint64_t)p.oh[o] * (c->band_r + 1) / c->band_n);
    }
    D.n_oct = k;
    if (k) launch_detect(D, st);
    S.detected = true;
    HIPCHK(hipGetLastError());
    return 0;
}

int launch_refine_stage(sift_mi_ctx* c, int si, const uint64_t* cand, const uint32_t* n_cand, uint32_t cand_cap,
                        ExtRec* ext, uint32_t* counter, uint32_t cap, hipStream_t st, uint32_t* counter_hi) {
    Plan& p = c->plan;
    RefineLaunch R{};
    R.counter_hi = counter_hi;
    R.cand = cand;
    R.n_cand = n_cand;
    R.cand_cap = cand_cap;
    R.band_flag = c->band_restricted ? c->band_flag.p : nullptr;
    R.band_r = (int)c->band_r;
    R.band_n = (int)c->band_n;
    R.band_patch = kBandPatch;
    R.band_margin = kBandDrift + 1 + kBandPatch;
    // PathOpts::band_drift narrows the rows the check accepts (down to
    // -kBandPatch: patches may not cross the band edge; tests force the re-run
    // path)
    R.band_margin = kBandPatch + 1 + std::min(kBandDrift, std::max(-kBandPatch, c->opts.band_drift));
    R.gauss = p.d_gauss[arena_of(c, si)].p;
    R.g_img_stride = p.d_gstride.p;
    R.ow = p.d_ow.p;
    R.oh = p.d_oh.p;
    R.opitch = p.d_opitch.p;
    R.n_oct = p.n_oct;
    R.img_base = 0;
    R.out = ext;
    R.counter = counter;
    R.cap = cap;
    launch_refine(R, st);
    HIPCHK(hipGetLastError());
    return 0;
}

int launch_orient_stage(sift_mi_ctx* c, int si, const ExtRec* ext, const uint32_t* n_ext, uint32_t ext_cap,
                        uint32_t kp_cap, hipStream_t st, const uint32_t* n_ext_hi) {
    Plan& p = c->plan;
    Slot& S = c->slot[si];
    OrientLaunch O{};
    O.ext = ext;
    O.n_ext_hi = n_ext_hi;
    O.n_ext = n_ext;
    O.ext_cap = ext_cap;
    O.gauss = p.d_gauss[arena_of(c, si)].p;
    O.gauss_img_stride = p.d_gstride.p;
    O.ow = p.d_ow.p;
    O.oh = p.d_oh.p;
    O.opitch = p.d_opitch.p;
    O.out = S.kp.p;
    O.counter = S.counters.p + 2;
    O.img_base = 0;
    O.cap = kp_cap;
    O.samples = c->count_samples ? c->samples.p : nullptr;
    launch_orient(O, st);
    HIPCHK(hipGetLastError());
    return 0;
}

int enqueue_keypoints(sift_mi_ctx* c, int si, uint32_t m, int64_t limit, uint32_t frame_base, const Bounds& B) {
    Plan& p = c->plan;
    Slot& S = c->slot[si];
    hipStream_t st = lane_stream(c, si);
    (void)frame_base;
    uint32_t* cnt = S.counters.p;
    uint32_t* starts = cnt + 4;
    uint32_t* out_cnt = cnt + 4 + m;
    uint32_t* work = cnt + 4 + 2 * m + kTailWords;  // descriptor work queues (after the tail region's words)
    (void)starts;
    (void)work;
    // one frame, no limit, early detection: the descriptors are computed in
    // keypoint index order beside the ordering stage, which runs on lane 1's
    // idle stream; k_gather_out then writes the outputs in emission order
    // (PathOpts::desc_first = 0: order, then describe in emission order)
    S.desc_first = S.early && m == 1 && limit < 0 && si == 0 && c->lanes == 2 &&
                   S.desc_kp.cap >= (size_t)B.bk * kDescSize && c->opts.desc_first;
    const bool join_pending = S.join_pending;
    S.join_pending = false;
    // completion events carried by kernel launches (not under stream capture)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const bool ext_events = hipStreamIsCapturing(st, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone;
    hipEvent_t aux_done = c->oct_ev[si][kTailMaxOct];  // the aux stream's early stages (join_pending)
    if (join_pending && !S.desc_first) HIPCHK(hipStreamWaitEvent(st, aux_done, 0));
    if (!S.detected) CHK(launch_detection(c, si, 0, m, 0, p.n_oct, st));
    // (early: refinement and orientation were enqueued inside the pyramid)
    if (!S.early) CHK(launch_refine_stage(c, si, S.cand.p, cnt + 0, B.bc, S.ext.p, cnt + 1, B.be, st));
    if (S.staged) HIPCHK(hipEventRecord(S.ev[2], st));
    if (!S.early) CHK(launch_orient_stage(c, si, S.ext.p, cnt + 1, B.be, B.bk, st));
    HIPCHK(hipGetLastError());
    if (S.staged) HIPCHK(hipEventRecord(S.ev[3], st));
    hipStream_t os = S.desc_first ? c->own2 : st;  // the ordering stage's stream
    hipStream_t ds = st;                            // the descriptor stage's stream
    if (S.desc_first) {
        // the ordering stage needs every keypoint: the lane stream's (tail
        // octaves) and, when the join is pending, the aux stream's; the
        // descriptors then run on the aux stream right after its orientation
        // (the lane stream's is long done by then), saving the cross-stream
        // hop in front of them (~15 us per one-frame call)
        HIPCHK(hipEventRecord(S.oriented, st));
        HIPCHK(hipStreamWaitEvent(os, S.oriented, 0));
        if (join_pending) {
            HIPCHK(hipStreamWaitEvent(os, aux_done, 0));
            ds = c->aux[si];
            HIPCHK(hipStreamWaitEvent(ds, S.oriented, 0));
        }
    }
    // emission order: radix sort of the keys (padding sorts last)
    const uint32_t* order = S.vals_b.p;  // emission order -> kp index
    const int img_bits = img_bits_for(m);
    const int end_bit = kKeyImgShift + img_bits;
    const uint64_t pad = (end_bit >= 64) ? ~0ull : ((1ull << end_bit) - 1);
    const bool onesweep = c->opts.onesweep == 1 || (c->opts.onesweep == 2 && B.bk >= kOnesweepMinKeys);
    size_t tmp = sort_pairs_u64(nullptr, 0, S.keys_a.p, S.keys_b.p, S.vals_a.p, S.vals_b.p, B.bk, end_bit, os, onesweep);
    const int rb = 32 + img_bits;
    const uint64_t rpad = (1ull << rb) - 1;
    if (limit >= 0)
        tmp = std::max(tmp, sort_pairs_u64(nullptr, 0, S.keys_a.p, S.keys_b.p, S.vals_a.p, S.fin.p, B.bk, rb, os, onesweep));
    if (!tmp) return fail(SIFT_MI_EHIP, "radix sort sizing failed");
    if (tmp > S.sort_tmp.cap) {
        HIPCHK(hipStreamSynchronize(st));
        if (os != st) HIPCHK(hipStreamSynchronize(os));
        CHK(S.sort_tmp.ensure(tmp));
    }
    launch_make_sort_keys(S.kp.p, cnt + 2, B.bk, pad, S.keys_a.p, S.vals_a.p, os);
    if (!sort_pairs_u64(S.sort_tmp.p, S.sort_tmp.cap, S.keys_a.p, S.keys_b.p, S.vals_a.p, S.vals_b.p, B.bk,
                        end_bit, os, onesweep))
        return fail(SIFT_MI_EHIP, "radix sort failed");
    launch_frame_starts(S.keys_b.p, cnt + 2, B.bk, starts, os);
    // features_limit (src/lib.rs:156-161): per-frame plan on the device
    // (desc_first: the plan's launch signals S.ordered, no marker after it)
    const bool ordered_ext = S.desc_first && ext_events && limit < 0;
    if (ordered_ext) set_launch_done_event(S.ordered);
    launch_limit_plan(starts, cnt + 2, B.bk, (int)m, limit, out_cnt, S.seg_off.p, S.out_off.p, S.use_resp.p,
                      cnt + 3, os);
    const bool ordered_signalled = ordered_ext && !launch_done_pending();
    set_launch_done_event(nullptr);
    if (limit >= 0) {
        // stable sort: response-descending within each frame, emission order on ties
        launch_make_resp_keys(S.kp.p, order, cnt + 2, B.bk, 0, rpad, S.keys_a.p, S.vals_a.p, os);
        if (!sort_pairs_u64(S.sort_tmp.p, S.sort_tmp.cap, S.keys_a.p, S.keys_b.p, S.vals_a.p, S.fin.p, B.bk, rb,
                            os, onesweep))
            return fail(SIFT_MI_EHIP, "response sort failed");
        launch_select(order, S.fin.p, S.seg_off.p, S.out_off.p, S.use_resp.p, (int)m, cnt + 3, B.bk, S.vals_a.p,
                      os);
        order = S.vals_a.p;
    }
    HIPCHK(hipGetLastError());
    if (S.desc_first && !ordered_signalled) HIPCHK(hipEventRecord(S.ordered, os));
    if (S.staged) HIPCHK(hipEventRecord(S.ev[4], st));
    // descriptors into this slot's outputs, once its previous copy-out is done
    if (S.pending_copy) HIPCHK(hipStreamWaitEvent(ds, S.copied, 0));
    DescLaunch DL{};
    DL.kp = S.kp.p;
    DL.idx = S.desc_first ? nullptr : order;
    DL.n = S.desc_first ? cnt + 2 : cnt + 3;
    DL.bound = B.bk;
    DL.work = work;
    DL.key_base = (uint64_t)frame_base << kKeyImgShift;
    DL.gauss = p.d_gauss[arena_of(c, si)].p;
    DL.gauss_img_stride = p.d_gstride.p;
    DL.ow = p.d_ow.p;
    DL.oh = p.d_oh.p;
    DL.opitch = p.d_opitch.p;
    DL.img_base = 0;
    DL.out_kp = S.desc_first ? nullptr : S.out_kp.p;
    DL.out_key = S.desc_first ? nullptr : S.out_key.p;
    DL.out_desc = S.desc_first ? S.desc_kp.p : S.out_desc.p;
    DL.exact = c->exact_descriptors;
    DL.samples = c->count_samples ? c->samples.p + 8 : nullptr;
    launch_describe(DL, ds);
    const int count_words = 4 + 2 * m + kTailWords;  // the frame plan and the tail region's counters (Slot::early)
    bool counts_copied = false;  // by k_gather_out, which then signals ev[6] itself
    if (S.desc_first) {
        HIPCHK(hipStreamWaitEvent(ds, S.ordered, 0));
        const bool in_gather = ext_events && !S.staged;
        if (in_gather) set_launch_done_event(S.ev[6]);
        launch_gather_out(S.kp.p, order, cnt + 3, B.bk, S.desc_kp.p, S.out_desc.p, S.out_kp.p, S.out_key.p,
                          DL.key_base, in_gather ? cnt : nullptr, in_gather ? S.h_counts.p : nullptr, count_words, ds);
        counts_copied = in_gather && !launch_done_pending();
        set_launch_done_event(nullptr);
    }
    HIPCHK(hipGetLastError());
    if (S.staged) HIPCHK(hipEventRecord(S.ev[5], st));
    if (!counts_copied) {
        HIPCHK(hipMemcpyAsync(S.h_counts.p, cnt, count_words * sizeof(uint32_t), hipMemcpyDeviceToHost, ds));
        HIPCHK(hipEventRecord(S.ev[6], ds));
    }
    // the lane stream's next work follows this chunk (and a capture rejoins)
    if (ds != st) HIPCHK(hipStreamWaitEvent(st, S.ev[6], 0));
    return 0;
}

void accumulate_times(sift_mi_ctx* c, Slot& S) {
    float ms;
    if (S.graph_run) {  // a graph replay records only the chunk's ends
        if (hipEventElapsedTime(&ms, S.ev[0], S.ev[6]) == hipSuccess) c->stats.total_ms += ms;
        return;
    }
    if (!S.staged) return;
    if (hipEventElapsedTime(&ms, S.ev[0], S.ev[1]) == hipSuccess) c->stats.pyramid_ms += ms;
    if (hipEventElapsedTime(&ms, S.ev[1], S.ev[2]) == hipSuccess) c->stats.detect_ms += ms;
    if (hipEventElapsedTime(&ms, S.ev[2], S.ev[3]) == hipSuccess) c->stats.orient_ms += ms;
    if (hipEventElapsedTime(&ms, S.ev[3], S.ev[4]) == hipSuccess) c->stats.order_ms += ms;
    if (hipEventElapsedTime(&ms, S.ev[4], S.ev[5]) == hipSuccess) c->stats.descriptor_ms += ms;
    if (hipEventElapsedTime(&ms, S.ev[0], S.ev[6]) == hipSuccess) c->stats.total_ms += ms;
}

// Enqueue pyramid (optional) + keypoint stages of one chunk on slot si.
int enqueue_chunk(sift_mi_ctx* c, int si, const uint8_t* d_frames, size_t frame_pitch, size_t stride, uint32_t m,
                  int64_t limit, uint32_t frame_base, bool pyramid) {
    Slot& S = c->slot[si];
    const Bounds B = chunk_bounds(c, m);
    CHK(ensure_lane(c, arena_of(c, si)));
    CHK(reserve_chunk(c, si, B, c->plan.chunk, m));
    hipStream_t st = lane_stream(c, si);
    S.staged = c->lanes == 1;
    if (S.staged) HIPCHK(hipEventRecord(S.ev[0], st));
    CHK(prepare_chunk(c, si, m, frame_base, B, pyramid));
    // stage overlap (two-lane mode; the one-lane mode times the stages apart):
    // detection starts inside the pyramid (run_pyramid), so ev[1]..ev[2] is
    // then only the refinement
    const bool fused = pyramid && c->lanes == 2;
    if (pyramid) CHK(run_pyramid(c, si, d_frames, frame_pitch, stride, m, false, fused ? si : -1, si));
    flush_chunk_init(c, si);  // (run_pyramid launched it after the seed)
    if (S.staged) HIPCHK(hipEventRecord(S.ev[1], st));
    return enqueue_keypoints(c, si, m, limit, frame_base, B);
}

// Wait for slot si's chunk; on success append its per-frame offsets and start
// the copy of its results to the host.  Returns 1 when a stage count exceeded
// its bound (the caller re-runs the chunk; the high-water marks now cover it).
int finalize_chunk(sift_mi_ctx* c, int si, size_t* offsets, bool only_chunk = false) {
    Slot& S = c->slot[si];
    HIPCHK(host_wait_event(S.ev[6]));
    const uint32_t* h = S.h_counts.p;
    const uint32_t m = S.m;
    const double fm = (double)m;
    // the tail octaves' region (Slot::early): its counts follow the frame plan
    const uint32_t hb0 = S.early ? h[4 + 2 * m] : 0, hb1 = S.early ? h[4 + 2 * m + 1] : 0;
    // the main region's extrema (a two-ended append keeps its back count in the tail words)
    const uint32_t h1 = h[1] + (S.early ? h[4 + 2 * m + 3] : 0);
    c->pf_cand = std::max(c->pf_cand, (h[0] + hb0) / fm);
    c->pf_ext = std::max(c->pf_ext, (h1 + hb1) / fm);
    c->pf_kp = std::max(c->pf_kp, h[2] / fm);
    c->pf_cand_b = std::max(c->pf_cand_b, std::max(hb0, hb1) / fm);
    if (h[0] > S.bc || h1 > S.be || h[2] > S.bk || hb0 > S.bcb || hb1 > S.bcb) {
        c->stats.stage_reruns++;
        return 1;
    }
    const uint32_t n_out = h[3];
    accumulate_times(c, S);
    const size_t base = c->n_result;
    if (offsets) {
        size_t acc = base;
        for (uint32_t f = 0; f < m; f++) {
            offsets[S.frame_base + f] = acc;
            acc += h[4 + m + f];
        }
    }
    c->dev_result_n = n_out;
    c->last_slot = si;
    c->res_slot = -1;
    if (c->keep_on_device && only_chunk) {
        // the call's only chunk: its outputs ARE the batch's device results
        // (valid until the next call, sift_mi_device_results) -- no copy
        c->res_slot = si;
    } else if (c->keep_on_device && n_out) {
        // whole-batch device arena: device-to-device copies on the copy stream
        const size_t need = base + n_out;
        if (need > c->r_kp.cap || need * kDescSize > c->r_desc.cap || need > c->r_key.cap) {
            HIPCHK(hipStreamSynchronize(c->cstream));
            CHK(grow_keep(c->r_kp, need, base, c->cstream));
            CHK(grow_keep(c->r_desc, need * kDescSize, base * kDescSize, c->cstream));
            CHK(grow_keep(c->r_key, need, base, c->cstream));
        }
        HIPCHK(hipStreamWaitEvent(c->cstream, S.ev[6], 0));
        HIPCHK(hipMemcpyAsync(c->r_kp.p + base, S.out_kp.p, n_out * sizeof(OutKp), hipMemcpyDeviceToDevice,
                              c->cstream));
        HIPCHK(hipMemcpyAsync(c->r_desc.p + base * kDescSize, S.out_desc.p, (size_t)n_out * kDescSize,
                              hipMemcpyDeviceToDevice, c->cstream));
        HIPCHK(hipMemcpyAsync(c->r_key.p + base, S.out_key.p, n_out * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                              c->cstream));
        HIPCHK(hipEventRecord(S.copied, c->cstream));
        S.pending_copy = true;
    }
    if (!c->keep_on_device) {
        const size_t need = base + n_out;
        if (need > c->h_kp.cap || need * kDescSize > c->h_desc.cap || need > c->h_key.cap) {
            HIPCHK(hipStreamSynchronize(c->cstream));  // copies in flight into the old buffers
            CHK(c->h_kp.ensure(need, true));
            CHK(c->h_desc.ensure(need * kDescSize, true));
            CHK(c->h_key.ensure(need, true));
        }
        if (n_out) {
            HIPCHK(hipStreamWaitEvent(c->cstream, S.ev[6], 0));
            HIPCHK(hipMemcpyAsync(c->h_kp.p + base, S.out_kp.p, n_out * sizeof(OutKp), hipMemcpyDeviceToHost,
                                  c->cstream));
            HIPCHK(hipMemcpyAsync(c->h_desc.p + base * kDescSize, S.out_desc.p, (size_t)n_out * kDescSize,
                                  hipMemcpyDeviceToHost, c->cstream));
            HIPCHK(hipMemcpyAsync(c->h_key.p + base, S.out_key.p, n_out * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                  c->cstream));
            HIPCHK(hipEventRecord(S.copied, c->cstream));
            S.pending_copy = true;
        }
    }
    c->n_result = base + n_out;
    c->stats.extrema += h1 + hb1;
    c->stats.keypoints += n_out;
    c->stats.frames += m;
    return 0;
}

// Single chunk, synchronous (precompute / sift_with_precomputed paths).
int run_chunk_sync(sift_mi_ctx* c, const uint8_t* d_frames, size_t frame_pitch, size_t stride, uint32_t m,
                   int64_t limit, bool pyramid, size_t* offsets) {
    c->n_result = 0;
    if (c->band_n > 1 && limit >= 0)
        return fail(SIFT_MI_EINVAL, "features_limit ranks a whole frame's keypoints: apply it after merging row bands");
    for (int attempt = 0; attempt < 4; attempt++) {
        CHK(enqueue_chunk(c, 0, d_frames, frame_pitch, stride, m, limit, 0, pyramid));
        const int rc = finalize_chunk(c, 0, offsets);
        if (rc < 0) return rc;
        if (rc == 0) {
            if (offsets) offsets[m] = c->n_result;
            HIPCHK(hipStreamSynchronize(c->cstream));
            return 0;
        }
    }
    return fail(SIFT_MI_ENOMEM, "stage count kept exceeding its buffer bound");
}

int check_frame_args(uint32_t w, uint32_t h, size_t stride) {
    if (w < 1 || h < 1) return fail(SIFT_MI_EINVAL, "empty image");
    if (stride < w) return fail(SIFT_MI_EINVAL, "row_stride < width");
    if (w > kMaxFrameSide || h > kMaxFrameSide) return fail(SIFT_MI_EINVAL, "image larger than 16384 px (key field)");
    return 0;
}

// A single-chunk call replayed as a HIP graph (PathOpts::graph): the first
// call with a given key runs normally (it also sizes every buffer), the
// second identical one is captured (relaxed stream capture of enqueue_chunk:
// the fork / join with the aux stream becomes graph edges) and launched, later
// ones only launch the graph.  Any (re)allocation changes the key (its
// buffers are baked into the graph).  Returns 1 when the chunk was enqueued
// here, 0 when the caller must enqueue it.
int enqueue_single_graph(sift_mi_ctx* c, const uint8_t* d_frames, size_t frame_pitch, size_t stride, uint32_t m,
                         int64_t limit) {
    Slot& S = c->slot[0];
    if (!c->opts.graph || c->band_n > 1 || c->lanes != 2 || S.pending_copy) return 0;
    const Bounds B = chunk_bounds(c, m);
    CHK(ensure_lane(c, arena_of(c, 0)));
    CHK(reserve_chunk(c, 0, B, c->plan.chunk, m));
    hipStream_t st = lane_stream(c, 0);
    sift_mi_ctx::GraphKey k;
    std::memset(&k, 0, sizeof k);
    k.opts = c->opts;
    k.frames = d_frames;
    k.frame_pitch = frame_pitch;
    k.stride = stride;
    k.m = m;
    k.w = c->plan.w;
    k.h = c->plan.h;
    k.bc = B.bc;
    k.be = B.be;
    k.bk = B.bk;
    k.bcb = S.bcb;
    k.limit = limit;
    k.gen = g_alloc_gen.load();
    k.keep = c->keep_on_device;
    k.exact = c->exact_descriptors;
    k.samples = c->count_samples;
    k.lanes = c->lanes;
    k.prof = c->plan.profile;
    k.maxo = c->plan.max_oct;
    k.st = st;
    if (!(c->gkey_ok && c->gkey == k)) {
        if (!(c->gseen_ok && c->gseen == k)) {  // first sighting: a normal run
            c->gseen = k;
            c->gseen_ok = true;
            return 0;
        }
        c->gkey_ok = false;
        if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
        if (c->graph) (void)hipGraphDestroy(c->graph);
        c->gexec = nullptr;
        c->graph = nullptr;
        HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        const int rc = enqueue_chunk(c, 0, d_frames, frame_pitch, stride, m, limit, 0, true);
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(st, &g);
        if (rc || e != hipSuccess || !g || g_alloc_gen.load() != k.gen) {
            if (g) (void)hipGraphDestroy(g);
            c->gseen_ok = false;
            return rc ? rc : fail(SIFT_MI_EHIP, std::string("graph capture failed: ") + hipGetErrorString(e));
        }
        if (hipGraphInstantiate(&c->gexec, g, nullptr, nullptr, 0) != hipSuccess) {
            (void)hipGraphDestroy(g);
            c->gexec = nullptr;
            c->gseen_ok = false;
            return fail(SIFT_MI_EHIP, "hipGraphInstantiate failed");
        }
        c->graph = g;
        c->gkey = k;
        c->gkey_ok = true;
        c->g_early = S.early;
        c->g_fused = S.fused_mask;
    }
    // the host-side chunk state prepare_chunk keeps (finalize_chunk reads it)
    S.m = m;
    S.frame_base = 0;
    S.cap_frames = m;
    S.bc = B.bc;
    S.be = B.be;
    S.bk = B.bk;
    S.detected = true;
    S.graph_run = true;
    S.early = c->g_early;
    S.fused_mask = c->g_fused;
    HIPCHK(hipEventRecord(S.ev[0], st));
    HIPCHK(hipGraphLaunch(c->gexec, st));
    HIPCHK(hipEventRecord(S.ev[6], st));
    return 1;
}

// Device-resident batch pipeline: chunks alternate between two lanes (slot,
// stream, pyramid arena and stage buffers each), so chunk k+1's kernels run
// beside chunk k's -- the small octaves, sorts and kernel tails of one chunk
// leave CUs idle that the other fills -- and chunk k+2 is enqueued as soon as
// chunk k has been finalised.  Results travel on the copy stream.
int extract_device(sift_mi_ctx* c, const uint8_t* d_frames, size_t frame_pitch, uint32_t n, uint32_t w, uint32_t h,
                   size_t stride, int64_t limit, size_t* offsets) {
    CHK(check_frame_args(w, h, stride));
    if (n > (1u << (64 - kKeyImgShift))) return fail(SIFT_MI_EINVAL, "more than 2^22 frames in one call (key field)");
    const sift_mi_stats stats0 = c->stats;  // restored if a banded pass is redone on the whole pyramid
    unsigned long long samples0[16] = {};   // and the device sample counters with it
    if (c->band_n > 1 && c->count_samples && c->samples.p) {
        CHK(sync_lanes(c));
        HIPCHK(hipMemcpy(samples0, c->samples.p, sizeof samples0, hipMemcpyDeviceToHost));
    }
    if (c->band_n > 1 && limit >= 0)
        return fail(SIFT_MI_EINVAL, "features_limit ranks a whole frame's keypoints: apply it after merging row bands");
    double avail = 0;  // device memory this context could hold: free + its own arenas
    if (!c->chunk_override && n > 1) {  // (one frame is one chunk: no query on the latency path)
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            avail = (double)free_b + 4.0 * ((double)c->plan.arena[0].cap + (double)c->plan.arena[1].cap);
    }
    const uint32_t chunk = std::min(kMaxChunk, c->chunk_override ? std::min(c->chunk_override, n)
                                                                 : auto_chunk(c->plan, w, h, n, c->opts.chunk_mode, avail));
    CHK(ensure_plan(c, w, h, chunk));
    c->have_pyramid = false;
    c->n_result = 0;
    c->have_result = false;
    c->batch_arena = -1;
    if (c->band_n > 1) {
        CHK(c->band_flag.ensure(1));
        HIPCHK(hipMemsetAsync(c->band_flag.p, 0, sizeof(uint32_t), c->stream));
    }
    const uint32_t n_chunks = (n + chunk - 1) / chunk;
    auto frames_of = [&](uint32_t k) { return std::min(chunk, n - k * chunk); };
    auto enqueue = [&](uint32_t k) {
        return enqueue_chunk(c, (int)(k & 1), d_frames + (size_t)k * chunk * frame_pitch, frame_pitch, stride,
                             frames_of(k), limit, k * chunk, true);
    };
    // lane 1 starts after the caller's stream (frames produced there); the
    // caller's stream resumes after lane 1's last chunk
    const bool two = n_chunks > 1 && c->lanes == 2;
    c->lanes_busy = two;
    struct Reset {
        sift_mi_ctx* c;
        ~Reset() { c->lanes_busy = false; }
    } reset_busy{c};
    if (two) {
        HIPCHK(hipEventRecord(c->fork, c->stream));
        HIPCHK(hipStreamWaitEvent(c->own2, c->fork, 0));
    }
    if (n_chunks == 1) {
        const int g = enqueue_single_graph(c, d_frames, frame_pitch, stride, n, limit);
        if (g < 0) return g;
        if (g == 0) CHK(enqueue(0));
    } else {
        CHK(enqueue(0));
        CHK(enqueue(1));
    }
    for (uint32_t k = 0; k < n_chunks; k++) {
        int rc = finalize_chunk(c, (int)(k & 1), offsets, n_chunks == 1);
        if (rc < 0) return rc;
        for (int attempt = 0; rc == 1; attempt++) {
            // a stage overflowed its bound: drain both lanes (the other lane's
            // chunk is unaffected), then re-run k on its lane
            if (attempt == 3) return fail(SIFT_MI_ENOMEM, "stage count kept exceeding its buffer bound");
            CHK(sync_lanes(c));
            CHK(enqueue(k));
            rc = finalize_chunk(c, (int)(k & 1), offsets, n_chunks == 1);
            if (rc < 0) return rc;
        }
        if (k + 2 < n_chunks) CHK(enqueue(k + 2));
    }
    if (two) {
        HIPCHK(hipEventRecord(c->fork, c->own2));
        HIPCHK(hipStreamWaitEvent(c->stream, c->fork, 0));
    }
    // every copy of the call done (a device-resident one-chunk call copied
    // nothing: no synchronisation, whose marker round trip costs a few us)
    bool copies = false;
    for (auto& S2 : c->slot) copies = copies || S2.pending_copy;
    if (copies) HIPCHK(hipStreamSynchronize(c->cstream));
    for (auto& S2 : c->slot) S2.pending_copy = false;
    if (offsets) offsets[n] = c->n_result;
    c->have_result = true;
    if (n_chunks == 1 && !c->band_restricted) {
        c->batch_arena = arena_of(c, 0);
        c->batch_frames = n;
    }
    if (c->band_restricted) {
        // a refinement drifted past the computed rows: redo the band on the
        // whole-frame pyramid (exact; the rare case)
        c->band_restricted = false;
        uint32_t flag = 0;
        HIPCHK(hipMemcpy(&flag, c->band_flag.p, sizeof(flag), hipMemcpyDeviceToHost));
        if (flag) {
            // the first pass's work is discarded: report the re-run alone
            const uint64_t reruns = c->stats.band_reruns + 1, stage_reruns = c->stats.stage_reruns;
            c->stats = stats0;
            c->stats.band_reruns = reruns;
            c->stats.stage_reruns = stage_reruns;
            if (c->count_samples && c->samples.p)
                HIPCHK(hipMemcpy(c->samples.p, samples0, sizeof samples0, hipMemcpyHostToDevice));
            c->band_whole = true;
            const int rc = extract_device(c, d_frames, frame_pitch, n, w, h, stride, limit, offsets);
            c->band_whole = false;
            return rc;
        }
    }
    return 0;
}

// image::imageops::resize on a host f32 image (Imageproc profile ops).
int ip_resize_op(sift_mi_ctx* c, const float* src, uint32_t w, uint32_t h, uint32_t dw, uint32_t dh, float support,
                 float* dst) {
    if (w == dw && h == dh) {  // image's resize copies when the size is unchanged
        std::memcpy(dst, src, sizeof(float) * (size_t)w * h);
        return 0;
    }
    IpTabDev tab;
    int rc = tab.upload((int)w, (int)h, (int)dw, (int)dh, support, 1, c->stream);
    DevBuf<float> a, t, b;
    if (!rc) rc = a.ensure((size_t)w * h);
    if (!rc) rc = t.ensure((size_t)w * dh);
    if (!rc) rc = b.ensure((size_t)dw * dh);
    if (!rc) {
        if (hipMemcpyAsync(a.p, src, (size_t)w * h * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            rc = fail(SIFT_MI_EHIP, "H2D failed");
    }
    if (!rc) {
        launch_ip_resize_f32(a.p, (int)w, (int)h, tab.xl.p, tab.xw.p, tab.xtaps, tab.yl.p, tab.yw.p, tab.ytaps, t.p,
                             b.p, (int)dw, (int)dh, c->stream);
        if (hipMemcpyAsync(dst, b.p, (size_t)dw * dh * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            rc = fail(SIFT_MI_EHIP, "resize failed");
    }
    a.release();
    t.release();
    b.release();
    tab.release();
    return rc;
}

int upload_frames(sift_mi_ctx* c, const uint8_t* const* frames, uint32_t n, uint32_t w, uint32_t h, size_t stride) {
    const size_t pitch = (size_t)w * h;
    CHK(c->staging.ensure(pitch * n));
    for (uint32_t i = 0; i < n; i++) {
        if (!frames[i]) return fail(SIFT_MI_EINVAL, "null frame");
        HIPCHK(hipMemcpy2DAsync(c->staging.p + i * pitch, w, frames[i], stride, w, h, hipMemcpyHostToDevice,
                                c->stream));
    }
    return 0;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
namespace {
// Process-wide pool of the contexts' streams (per device, in creation
// order).  HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES,
// 4 by default) as they are created; a context created after another was
// destroyed would otherwise get a different, possibly colliding mapping
// (measured: one 1080p frame per call 0.69 ms in a fresh process, 0.89 ms
// after a closed batch context -- the octave overlap's two streams had landed
// on one queue).  A closed context returns its streams here; the next one
// takes the same stream objects back, so every context sees the queue
// mapping of the first.
struct StreamPool {
    std::mutex mu;
    std::vector<std::vector<hipStream_t>> free_sets[64];  // per device: sets of kCtxStreams
};
StreamPool& stream_pool() {
    static StreamPool* p = new StreamPool();  // never destroyed: streams live until process exit
    return *p;
}
// the order matters for the queue mapping: lane 0, lane 1, lane 0's aux,
// the copy stream, lane 1's aux, lane 0's second aux (with 4 queues the last
// two share the lanes' queues: lane 1's aux is used only when lane 1 is idle,
// the second aux only while lane 1's stream is: a one-lane / one-chunk call)
constexpr int kCtxStreams = 6;
bool take_streams(int dev, hipStream_t (&out)[kCtxStreams]) {
    StreamPool& P = stream_pool();
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto& fs = P.free_sets[dev & 63];
        if (!fs.empty()) {
            for (int i = 0; i < kCtxStreams; i++) out[i] = fs.back()[i];
            fs.pop_back();
            return true;
        }
    }
    for (int i = 0; i < kCtxStreams; i++) {
        if (hipStreamCreateWithFlags(&out[i], hipStreamNonBlocking) != hipSuccess) {
            for (int k = 0; k < i; k++) (void)hipStreamDestroy(out[k]);
            return false;
        }
    }
    return true;
}
void give_streams(int dev, const hipStream_t (&in)[kCtxStreams]) {
    StreamPool& P = stream_pool();
    std::lock_guard<std::mutex> g(P.mu);
    P.free_sets[dev & 63].emplace_back(in, in + kCtxStreams);
}
}  // namespace

extern "C" {

const char* sift_mi_version(void) { return "sift_mi 0.4.0 (gfx950)"; }
const char* sift_mi_last_error(void) { return g_err.c_str(); }

bool create_sync_events(sift_mi_ctx* c);

int sift_mi_create(int device_ordinal, sift_mi_profile profile, sift_mi_ctx** out) {
    if (!out) return fail(SIFT_MI_EINVAL, "out is null");
    *out = nullptr;
    if (profile != SIFT_MI_PROFILE_OPENCV && profile != SIFT_MI_PROFILE_IMAGEPROC)
        return fail(SIFT_MI_EINVAL, "unknown profile");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(SIFT_MI_ENODEV, "no HIP device");
    if (device_ordinal < 0 || device_ordinal >= ndev) return fail(SIFT_MI_ENODEV, "device ordinal out of range");
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device_ordinal));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SIFT_MI_ENODEV, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
    HIPCHK(hipSetDevice(device_ordinal));
    sift_mi_ctx* c = new sift_mi_ctx();
    c->device = device_ordinal;
    c->profile = profile;
    hipStream_t ss[kCtxStreams];
    if (!take_streams(device_ordinal, ss)) {
        delete c;
        return fail(SIFT_MI_EHIP, "hipStreamCreate failed");
    }
    c->own = ss[0];
    c->own2 = ss[1];
    c->aux[0] = ss[2];
    c->cstream = ss[3];
    c->aux[1] = ss[4];
    c->aux2 = ss[5];
    c->stream = c->own;
    bool ok = create_sync_events(c);
    for (auto& S : c->slot) {
        for (auto& e : S.ev) ok = ok && hipEventCreate(&e) == hipSuccess;
        ok = ok && hipEventCreateWithFlags(&S.copied, hipEventDisableTiming) == hipSuccess;
    }
    if (!ok) {
        sift_mi_destroy(c);
        return fail(SIFT_MI_EHIP, "stream / event creation failed");
    }
    *out = c;
    return 0;
}

void sift_mi_destroy(sift_mi_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // every stream that may still run work on this context's buffers first:
    // the caller's stream (sift_mi_set_stream), the context's own lane-0
    // stream (it goes back to the pool below), lane 1, both aux streams
    // (octave blurs 4, 5 and detection write the arenas) and the copy stream
    {
        const hipStream_t ss[] = {c->stream, c->own, c->own2, c->aux[0], c->aux[1], c->aux2, c->cstream, c->dec};
        for (hipStream_t s : ss)
            if (s) (void)hipStreamSynchronize(s);
    }
    c->plan.release();
    c->staging.release();
    c->jpeg.release();
    c->band_flag.release();
    for (auto& S : c->slot) S.release_bufs();
    for (auto& S : c->slot) {
        S.counters.release();
        S.h_counts.release();
        S.out_kp.release();
        S.out_desc.release();
        S.out_key.release();
        S.desc_kp.release();
        for (auto& e : S.ev)
            if (e) (void)hipEventDestroy(e);
        if (S.copied) (void)hipEventDestroy(S.copied);
        if (S.ordered) (void)hipEventDestroy(S.ordered);
        if (S.oriented) (void)hipEventDestroy(S.oriented);
    }
    if (c->fork) (void)hipEventDestroy(c->fork);
    if (c->aux2_join) (void)hipEventDestroy(c->aux2_join);
    for (auto& lane : c->oct_ev)
        for (auto& e : lane)
            if (e) (void)hipEventDestroy(e);
    c->r_kp.release();
    c->r_desc.release();
    c->r_key.release();
    c->h_kp.release();
    c->h_desc.release();
    c->h_key.release();
    if (c->dec) (void)hipStreamDestroy(c->dec);
    if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    if (c->own) {  // the streams go back to the pool (synchronised above)
        const hipStream_t ss[kCtxStreams] = {c->own, c->own2, c->aux[0], c->cstream, c->aux[1], c->aux2};
        give_streams(c->device, ss);
    }
    delete c;
}

int sift_mi_set_stream(sift_mi_ctx* c, void* s) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    c->stream = s ? (hipStream_t)s : c->own;
    return 0;
}

int sift_mi_set_chunk(sift_mi_ctx* c, uint32_t k) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    c->chunk_override = k;
    return 0;
}

int sift_mi_set_max_octaves(sift_mi_ctx* c, int max_octaves) {
    if (!c || max_octaves < 0) return fail(SIFT_MI_EINVAL, "max_octaves must be >= 0");
    CHK(set_device(c));
    CHK(sync_lanes(c));
    c->max_octaves = max_octaves;  // the plan is rebuilt on the next call
    c->have_pyramid = false;
    return 0;
}

int sift_mi_set_exact_descriptors(sift_mi_ctx* c, int exact) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    c->exact_descriptors = exact ? 1 : 0;
    return 0;
}

int sift_mi_set_pipeline_lanes(sift_mi_ctx* c, int lanes) {
    if (!c || (lanes != 1 && lanes != 2)) return fail(SIFT_MI_EINVAL, "lanes must be 1 or 2");
    CHK(set_device(c));
    CHK(sync_lanes(c));
    c->lanes = lanes;
    return 0;
}

int sift_mi_set_row_band(sift_mi_ctx* c, uint32_t band, uint32_t n_bands) {
    if (!c || n_bands == 0 || band >= n_bands) return fail(SIFT_MI_EINVAL, "band must be < n_bands, n_bands >= 1");
    c->band_r = band;
    c->band_n = n_bands;
    return 0;
}

// The events that only order the context's streams on the device (octave
// hand-overs, forks, joins, the one-frame path's oriented / ordered).
// (Measured: a device-scope release, hipEventReleaseToDevice, changed nothing
// -- 0.581-0.583 ms per 1080p frame either way; a signalling kernel still
// costs its stream ~5 us before the next one starts)
bool create_sync_events(sift_mi_ctx* c) {
    auto make = [&](hipEvent_t& e) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
        return hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    };
    bool ok = make(c->fork) && make(c->aux2_join);
    for (auto& lane : c->oct_ev)
        for (auto& e : lane) ok = ok && make(e);
    for (auto& S : c->slot) ok = ok && make(S.ordered) && make(S.oriented);
    return ok;
}

int sift_mi_set_path_option(sift_mi_ctx* c, int option, int value) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    CHK(set_device(c));
    CHK(sync_lanes(c));  // no chunk in flight sees a half-changed path
    PathOpts& o = c->opts;
    const bool b = value == 0 || value == 1;
    switch (option) {
        case SIFT_MI_PATH_TILE_BLUR: if (!b) break; o.tile_blur = value; return 0;
        case SIFT_MI_PATH_PAIR_BLUR: if (!b) break; o.pair = value; return 0;
        case SIFT_MI_PATH_SEED_PAIR: if (!b) break; o.seed_pair = value; return 0;
        case SIFT_MI_PATH_TAIL: if (!b) break; o.tail = value; return 0;
        case SIFT_MI_PATH_FUSED_DETECT: if (value < 0 || value > 2) break; o.fused_detect = value; return 0;
        case SIFT_MI_PATH_EARLY: if (!b) break; o.early = value; return 0;
        case SIFT_MI_PATH_DESC_FIRST: if (!b) break; o.desc_first = value; return 0;
        case SIFT_MI_PATH_GRAPH: if (!b) break; o.graph = value; return 0;
        case SIFT_MI_PATH_BAND_DRIFT: if (value < -kBandPatch || value > kBandDrift) break; o.band_drift = value; return 0;
        case SIFT_MI_PATH_BOUND_SHRINK: if (value < 1) break; o.bound_shrink = value; return 0;
        case SIFT_MI_PATH_LARGE_FIRST: if (!b) break; o.large_first = value; return 0;
        case SIFT_MI_PATH_ONESWEEP: if (value < 0 || value > 2) break; o.onesweep = value; return 0;
        case SIFT_MI_PATH_BD_PAIR: if (value < 0 || value > 2) break; o.bd_pair = value; return 0;
        case SIFT_MI_PATH_BD_WAVES: if (value < 1024 || value > 65536) break; o.bd_waves = value; return 0;
        case SIFT_MI_PATH_CHUNK_MODE: if (value < 0 || value > 1) break; o.chunk_mode = value; return 0;
        default: return fail(SIFT_MI_EINVAL, "unknown path option");
    }
    return fail(SIFT_MI_EINVAL, "path option value out of range");
}

int sift_mi_set_keep_on_device(sift_mi_ctx* c, int keep) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    c->keep_on_device = keep ? 1 : 0;
    return 0;
}

int sift_mi_extract_batch_device(sift_mi_ctx* c, const uint8_t* d_frames, size_t frame_pitch, uint32_t n,
                                 uint32_t w, uint32_t h, size_t stride, int64_t limit, size_t* offsets) {
    if (!c || !d_frames || n == 0) return fail(SIFT_MI_EINVAL, "bad arguments");
    if (frame_pitch < stride * (h - 1) + w && n > 1) return fail(SIFT_MI_EINVAL, "frame_pitch too small");
    CHK(set_device(c));
    return extract_device(c, d_frames, frame_pitch, n, w, h, stride, limit, offsets);
}

int sift_mi_extract_batch(sift_mi_ctx* c, const uint8_t* const* frames, uint32_t n, uint32_t w, uint32_t h,
                          size_t stride, int64_t limit, size_t* offsets) {
    if (!c || !frames || n == 0) return fail(SIFT_MI_EINVAL, "bad arguments");
    CHK(check_frame_args(w, h, stride));
    CHK(set_device(c));
    CHK(upload_frames(c, frames, n, w, h, stride));
    const int keep = c->keep_on_device;
    c->keep_on_device = 0;
    const int rc = extract_device(c, c->staging.p, (size_t)w * h, n, w, h, w, limit, offsets);
    c->keep_on_device = keep;
    return rc;
}

int sift_mi_extract(sift_mi_ctx* c, const uint8_t* pixels, uint32_t w, uint32_t h, size_t stride, int64_t limit,
                    size_t* n_keypoints) {
    if (!c || !pixels) return fail(SIFT_MI_EINVAL, "bad arguments");
    const uint8_t* frames[1] = {pixels};
    size_t offs[2];
    CHK(sift_mi_extract_batch(c, frames, 1, w, h, stride, limit, offs));
    if (n_keypoints) *n_keypoints = offs[1];
    return 0;
}

}  // extern "C"

namespace {
// Host copy of large results: split across threads (the copy is bound by
// page faults on freshly allocated destinations as much as by bandwidth).
void par_memcpy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPerThread = 4u << 20;
    const unsigned hw = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    const unsigned nt = (unsigned)std::min<size_t>(hw, bytes / kPerThread);
    if (nt <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const size_t part = (bytes / nt + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) {
        const size_t a = t * part;
        if (a >= bytes) break;
        const size_t b = std::min(bytes, a + part);
        th.emplace_back([=] { std::memcpy((char*)dst + a, (const char*)src + a, b - a); });
    }
    std::memcpy(dst, src, std::min(bytes, part));
    for (auto& x : th) x.join();
}
}  // namespace

extern "C" {

int sift_mi_fetch(sift_mi_ctx* c, sift_mi_keypoint* kps, uint8_t* desc, size_t cap) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    if (!c->have_result || c->keep_on_device) return fail(SIFT_MI_ESTATE, "no host result to fetch");
    if (cap < c->n_result) return fail(SIFT_MI_EINVAL, "cap < result size");
    static_assert(sizeof(sift_mi_keypoint) == sizeof(OutKp), "layout");
    if (kps && c->n_result) par_memcpy(kps, c->h_kp.p, c->n_result * sizeof(OutKp));
    if (desc && c->n_result) par_memcpy(desc, c->h_desc.p, c->n_result * kDescSize);
    return 0;
}

int sift_mi_fetch_keys(sift_mi_ctx* c, uint64_t* keys, size_t cap) {
    if (!c || !keys) return fail(SIFT_MI_EINVAL, "bad arguments");
    if (!c->have_result || c->keep_on_device) return fail(SIFT_MI_ESTATE, "no host result to fetch");
    if (cap < c->n_result) return fail(SIFT_MI_EINVAL, "cap < result size");
    if (c->n_result) par_memcpy(keys, c->h_key.p, c->n_result * sizeof(uint64_t));
    return 0;
}

int sift_mi_device_results(sift_mi_ctx* c, const sift_mi_keypoint** d_kps, const uint8_t** d_desc, size_t* n) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    if (!c->have_result) return fail(SIFT_MI_ESTATE, "no result");
    if (!c->keep_on_device) return fail(SIFT_MI_ESTATE, "results were copied to the host (keep_on_device is 0)");
    const bool direct = c->res_slot >= 0;
    const Slot& S = c->slot[direct ? c->res_slot : 0];
    if (d_kps) *d_kps = reinterpret_cast<const sift_mi_keypoint*>(direct ? S.out_kp.p : c->r_kp.p);
    if (d_desc) *d_desc = direct ? S.out_desc.p : c->r_desc.p;
    if (n) *n = c->n_result;
    return 0;
}

// ---- precompute_images / sift_with_precomputed (single frame) -------------
int sift_mi_precompute(sift_mi_ctx* c, const uint8_t* pixels, uint32_t w, uint32_t h, size_t stride,
                       size_t* n_octaves) {
    if (!c || !pixels) return fail(SIFT_MI_EINVAL, "bad arguments");
    CHK(check_frame_args(w, h, stride));
    CHK(set_device(c));
    const uint8_t* frames[1] = {pixels};
    c->batch_arena = -1;  // arena 0 is rewritten: the last batch's planes are gone
    CHK(upload_frames(c, frames, 1, w, h, stride));
    CHK(ensure_plan(c, w, h, 1));
    CHK(run_pyramid(c, 0, c->staging.p, (size_t)w * h, w, 1, true));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->have_pyramid = true;
    c->have_result = false;
    if (n_octaves) *n_octaves = (size_t)c->plan.n_oct;
    return 0;
}

int sift_mi_octave_dims(sift_mi_ctx* c, size_t o, uint32_t* w, uint32_t* h) {
    if (!c || !c->have_pyramid) return fail(SIFT_MI_ESTATE, "no precomputed pyramid");
    if (o >= (size_t)c->plan.n_oct) return fail(SIFT_MI_EINVAL, "octave out of range");
    if (w) *w = (uint32_t)c->plan.ow[o];
    if (h) *h = (uint32_t)c->plan.oh[o];
    return 0;
}

int sift_mi_read_scale_space(sift_mi_ctx* c, size_t o, float* out) {
    if (!c || !out || !c->have_pyramid) return fail(SIFT_MI_ESTATE, "no precomputed pyramid");
    if (o >= (size_t)c->plan.n_oct) return fail(SIFT_MI_EINVAL, "octave out of range");
    CHK(set_device(c));
    const Plan& p = c->plan;
    HIPCHK(hipMemcpy2D(out, (size_t)p.ow[o] * sizeof(float), c->plan.gauss((int)o), (size_t)p.opitch[o] * sizeof(float),
                       (size_t)p.ow[o] * sizeof(float), (size_t)kImagesPerOctave * p.oh[o], hipMemcpyDeviceToHost));
    return 0;
}

int sift_mi_batch_octave_dims(sift_mi_ctx* c, size_t o, uint32_t* w, uint32_t* h) {
    if (!c || c->batch_arena < 0) return fail(SIFT_MI_ESTATE, "no single-chunk batch pyramid");
    if (o >= (size_t)c->plan.n_oct) return fail(SIFT_MI_EINVAL, "octave out of range");
    if (w) *w = (uint32_t)c->plan.ow[o];
    if (h) *h = (uint32_t)c->plan.oh[o];
    return 0;
}

int sift_mi_read_batch_scale_space(sift_mi_ctx* c, uint32_t frame, size_t o, float* out, size_t out_floats) {
    if (!c || !out || c->batch_arena < 0) return fail(SIFT_MI_ESTATE, "no single-chunk batch pyramid");
    Plan& p = c->plan;
    if (o >= (size_t)p.n_oct || frame >= c->batch_frames || frame >= p.chunk)
        return fail(SIFT_MI_EINVAL, "frame / octave out of range");
    if (out_floats < (size_t)kImagesPerOctave * p.ow[o] * p.oh[o])
        return fail(SIFT_MI_EINVAL, "out_floats < 6 * width * height of the octave (sift_mi_batch_octave_dims)");
    CHK(set_device(c));
    CHK(sync_lanes(c));
    const float* g = p.gauss((int)o, c->batch_arena) + (size_t)frame * p.gstride((int)o);
    HIPCHK(hipMemcpy2D(out, (size_t)p.ow[o] * sizeof(float), g, (size_t)p.opitch[o] * sizeof(float),
                       (size_t)p.ow[o] * sizeof(float), (size_t)kImagesPerOctave * p.oh[o], hipMemcpyDeviceToHost));
    return 0;
}

int sift_mi_read_dog(sift_mi_ctx* c, size_t o, float* out) {
    if (!c || !out || !c->have_pyramid) return fail(SIFT_MI_ESTATE, "no precomputed pyramid");
    if (o >= (size_t)c->plan.n_oct) return fail(SIFT_MI_EINVAL, "octave out of range");
    CHK(set_device(c));
    const Plan& p = c->plan;
    HIPCHK(hipMemcpy2D(out, (size_t)p.ow[o] * sizeof(float), c->plan.dog((int)o), (size_t)p.opitch[o] * sizeof(float),
                       (size_t)p.ow[o] * sizeof(float), (size_t)kDogPerOctave * p.oh[o], hipMemcpyDeviceToHost));
    return 0;
}

int sift_mi_sift_with_precomputed(sift_mi_ctx* c, int64_t limit, size_t* n_keypoints) {
    if (!c || !c->have_pyramid) return fail(SIFT_MI_ESTATE, "no precomputed pyramid");
    CHK(set_device(c));
    c->batch_arena = -1;  // a later call: the batch read-back is no longer valid
    const int keep = c->keep_on_device;
    c->keep_on_device = 0;
    size_t offs[2];
    const int rc = run_chunk_sync(c, nullptr, 0, 0, 1, limit, false, offs);
    c->keep_on_device = keep;
    CHK(rc);
    c->have_result = true;
    if (n_keypoints) *n_keypoints = offs[1];
    return 0;
}

// ---- compute_descriptor --------------------------------------------------
int sift_mi_compute_descriptor(sift_mi_ctx* c, const float* img, uint32_t w, uint32_t h, float x, float y,
                               float scale, float orientation, uint8_t* out) {
    if (!c || !img || !out || w < 1 || h < 1) return fail(SIFT_MI_EINVAL, "bad arguments");
    // window radius round(10.61 * scale) <= 39 (the device scratch); the
    // pipeline's keypoints have scale < 3.6 (radius <= 38)
    if (!(scale > 0.f) || roundf(3.0f * scale * 1.41421356f * 5.0f * 0.5f) > 39.0f)
        return fail(SIFT_MI_EUNSUPPORTED, "scale outside (0, 3.7]: descriptor window radius > 39");
    // the reference indexes its histogram out of bounds (panics) outside [0, 360]
    if (!(orientation >= 0.f && orientation <= 360.f)) return fail(SIFT_MI_EINVAL, "orientation outside [0, 360]");
    CHK(set_device(c));
    DevBuf<float> dimg;
    DevBuf<uint8_t> dout;
    CHK(dimg.ensure((size_t)w * h));
    CHK(dout.ensure(kDescSize));
    int rc = 0;
    if (hipMemcpyAsync(dimg.p, img, (size_t)w * h * sizeof(float), hipMemcpyHostToDevice, c->stream) != hipSuccess)
        rc = fail(SIFT_MI_EHIP, "H2D failed");
    if (!rc) {
        launch_describe_one(dimg.p, (int)w, (int)h, x, y, scale, orientation, dout.p, c->stream);
        if (hipMemcpyAsync(out, dout.p, kDescSize, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            rc = fail(SIFT_MI_EHIP, "compute_descriptor failed");
    }
    dimg.release();
    dout.release();
    return rc;
}

// ---- Processing ops ------------------------------------------------------
int sift_mi_gaussian_blur(sift_mi_ctx* c, const float* src, uint32_t w, uint32_t h, double sigma, float* dst) {
    if (!c || !src || !dst || w < 2 || h < 2 || !(sigma > 0)) return fail(SIFT_MI_EINVAL, "bad arguments");
    CHK(set_device(c));
    BlurTaps taps;
    const bool ip = c->profile == SIFT_MI_PROFILE_IMAGEPROC;
    const int r = ip ? ip_blur_taps((float)sigma, &taps) : cv_blur_taps(sigma, &taps);
    if (r < 1) return fail(SIFT_MI_EUNSUPPORTED, "blur radius outside 1..24");
    DevBuf<float> a, b;
    const size_t pitch = ((size_t)w + 63) & ~(size_t)63;  // same row alignment as the pyramid
    CHK(a.ensure(pitch * h));
    CHK(b.ensure(pitch * h));
    int rc = 0;
    BlurLaunch L{};
    L.src = a.p;
    L.dst = b.p;
    L.W = (int)w;
    L.H = (int)h;
    L.pitch = (int)pitch;
    L.n_img = 1;
    L.taps = taps;
    L.profile = ip ? kProfileImageproc : kProfileOpenCV;
    if (hipMemcpy2DAsync(a.p, pitch * 4, src, (size_t)w * 4, (size_t)w * 4, h, hipMemcpyHostToDevice, c->stream) !=
            hipSuccess ||
        launch_blur(r, L, c->stream, c->opts) != 0 ||
        hipMemcpy2DAsync(dst, (size_t)w * 4, b.p, pitch * 4, (size_t)w * 4, h, hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        rc = fail(SIFT_MI_EHIP, "gaussian_blur failed");
    a.release();
    b.release();
    return rc;
}

int sift_mi_resize_linear(sift_mi_ctx* c, const float* src, uint32_t w, uint32_t h, uint32_t dw, uint32_t dh,
                          float* dst) {
    if (!c || !src || !dst || !w || !h || !dw || !dh) return fail(SIFT_MI_EINVAL, "bad arguments");
    CHK(set_device(c));
    if (c->profile == SIFT_MI_PROFILE_IMAGEPROC) return ip_resize_op(c, src, w, h, dw, dh, 1.0f, dst);
    ResizeTabDev tab;
    CHK(tab.upload((int)w, (int)h, (int)dw, (int)dh, c->stream));
    DevBuf<float> a, b;
    CHK(a.ensure((size_t)w * h));
    CHK(b.ensure((size_t)dw * dh));
    int rc = 0;
    if (hipMemcpyAsync(a.p, src, (size_t)w * h * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess) rc = -1;
    if (!rc) launch_resize_linear_f32(a.p, (int)w, (int)h, tab.tab, b.p, (int)dw, (int)dh, c->stream);
    if (rc || hipMemcpyAsync(dst, b.p, (size_t)dw * dh * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        rc = fail(SIFT_MI_EHIP, "resize_linear failed");
    a.release();
    b.release();
    tab.release();
    return rc;
}

int sift_mi_resize_nearest(sift_mi_ctx* c, const float* src, uint32_t w, uint32_t h, uint32_t dw, uint32_t dh,
                           float* dst) {
    if (!c || !src || !dst || !w || !h || !dw || !dh) return fail(SIFT_MI_EINVAL, "bad arguments");
    CHK(set_device(c));
    if (c->profile == SIFT_MI_PROFILE_IMAGEPROC) return ip_resize_op(c, src, w, h, dw, dh, 0.0f, dst);
    std::vector<int> xo, yo;
    cv_nearest_ofs((int)w, (int)dw, xo);
    cv_nearest_ofs((int)h, (int)dh, yo);
    DevBuf<float> a, b;
    DevBuf<int> dx, dy;
    CHK(a.ensure((size_t)w * h));
    CHK(b.ensure((size_t)dw * dh));
    CHK(dx.ensure(dw));
    CHK(dy.ensure(dh));
    int rc = 0;
    if (hipMemcpyAsync(a.p, src, (size_t)w * h * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(dx.p, xo.data(), dw * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(dy.p, yo.data(), dh * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        rc = -1;
    if (!rc) launch_resize_nearest_f32(a.p, (int)w, dx.p, dy.p, b.p, (int)dw, (int)dh, c->stream);
    if (rc || hipMemcpyAsync(dst, b.p, (size_t)dw * dh * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        rc = fail(SIFT_MI_EHIP, "resize_nearest failed");
    a.release();
    b.release();
    dx.release();
    dy.release();
    return rc;
}

// ---- descriptor matching (examples/sift-match.rs:30-35) ---------------------
int sift_mi_match_descriptors(sift_mi_ctx* c, const uint8_t* query, size_t nq, const uint8_t* train, size_t nt,
                              int cross_check, sift_mi_match* out, size_t cap, size_t* n_matches) {
    if (!c || !n_matches || (nq && !query) || (nt && !train)) return fail(SIFT_MI_EINVAL, "bad arguments");
    if (nq > 0x7fffffff || nt > 0x7fffffff) return fail(SIFT_MI_EINVAL, "descriptor set too large");
    *n_matches = 0;
    if (nq == 0) return 0;
    CHK(set_device(c));
    DevBuf<uint8_t> dq, dt;
    DevBuf<float> qn, tn, dist;
    DevBuf<unsigned long long> rb, cb;
    DevBuf<int> tix;
    int rc = 0;
    if (!rc) rc = dq.ensure(nq * kDescSize);
    if (!rc) rc = dt.ensure(std::max<size_t>(nt, 1) * kDescSize);
    if (!rc) rc = qn.ensure(nq);
    if (!rc) rc = tn.ensure(std::max<size_t>(nt, 1));
    if (!rc) rc = rb.ensure(nq);
    if (!rc) rc = cb.ensure(std::max<size_t>(nt, 1));
    if (!rc) rc = tix.ensure(nq);
    if (!rc) rc = dist.ensure(nq);
    std::vector<int> h_t(nq);
    std::vector<float> h_d(nq);
    if (!rc) {
        hipStream_t st = c->stream;
        if (hipMemcpyAsync(dq.p, query, nq * kDescSize, hipMemcpyHostToDevice, st) != hipSuccess ||
            (nt && hipMemcpyAsync(dt.p, train, nt * kDescSize, hipMemcpyHostToDevice, st) != hipSuccess))
            rc = fail(SIFT_MI_EHIP, "H2D failed");
        if (!rc) {
            launch_match(dq.p, (int)nq, dt.p, (int)nt, cross_check ? 1 : 0, qn.p, tn.p, rb.p, cb.p, tix.p, dist.p, st);
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(h_t.data(), tix.p, nq * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(h_d.data(), dist.p, nq * sizeof(float), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                rc = fail(SIFT_MI_EHIP, "match failed");
        }
    }
    dq.release();
    dt.release();
    qn.release();
    tn.release();
    rb.release();
    cb.release();
    tix.release();
    dist.release();
    CHK(rc);
    size_t n = 0;
    for (size_t i = 0; i < nq; i++) n += h_t[i] >= 0;
    *n_matches = n;
    if (cap < n || (n && !out)) return fail(SIFT_MI_EINVAL, "cap < number of matches");
    size_t k = 0;
    for (size_t i = 0; i < nq; i++)
        if (h_t[i] >= 0) out[k++] = sift_mi_match{(int32_t)i, h_t[i], h_d[i]};
    return 0;
}

int sift_mi_jpeg_dims(const uint8_t* data, size_t len, uint32_t* width, uint32_t* height) {
    if (!data || !width || !height) return fail(SIFT_MI_EINVAL, "bad arguments");
    std::string err;
    const int rc = jpeg_dims(data, len, width, height, err);
    return rc ? fail(rc, err) : 0;
}

int sift_mi_decode_jpeg(sift_mi_ctx* c, const uint8_t* data, size_t len, uint8_t* out, size_t out_stride,
                        int out_on_device) {
    if (!c || !data || !out) return fail(SIFT_MI_EINVAL, "bad arguments");
    uint32_t w = 0, h = 0;
    std::string err;
    int rc = jpeg_dims(data, len, &w, &h, err);
    if (rc) return fail(rc, err);
    if (out_stride < w) return fail(SIFT_MI_EINVAL, "out_stride < width");
    CHK(set_device(c));
    rc = jpeg_decode_luma(data, len, out, out_stride, out_on_device != 0, c->stream, err);
    return rc ? fail(rc, err) : 0;
}

int sift_mi_decode_jpeg_batch(sift_mi_ctx* c, const uint8_t* const* data, const size_t* len, uint32_t n,
                              uint8_t* d_frames, size_t frame_pitch, size_t row_stride, int threads) {
    if (!c || (n && (!data || !len || !d_frames))) return fail(SIFT_MI_EINVAL, "bad arguments");
    for (uint32_t i = 0; i < n; i++)
        if (!data[i]) return fail(SIFT_MI_EINVAL, "null JPEG");
    if (threads <= 0) threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    CHK(set_device(c));
    std::string err;
    // The reconstruction kernels run on a high-priority stream of their own
    // (ordered after the context's stream): the runtime takes its hardware
    // queue from the high-priority pool, so a decode pipelined beside another
    // context's batch (bench.py configs.jpeg_e2e) does not queue behind that
    // batch's kernels on a shared in-order queue -- normal-priority streams
    // share GPU_MAX_HW_QUEUES (4) queues round robin.  A caller stream
    // (sift_mi_set_stream) is used as is.  Measured (round 4), with the
    // polling host wait (host_wait_event): 2337 -> 3063 frames/s JPEG ->
    // keypoints, pipelined beside sift().
    hipStream_t st = c->stream;
    if (c->stream == c->own) {
        if (!c->dec) {
            int least = 0, greatest = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIPCHK(hipStreamCreateWithPriority(&c->dec, hipStreamNonBlocking, greatest));
        }
        HIPCHK(hipEventRecord(c->fork, c->stream));
        HIPCHK(hipStreamWaitEvent(c->dec, c->fork, 0));
        st = c->dec;
    }
    const int rc = jpeg_decode_batch(data, len, n, d_frames, frame_pitch, row_stride, threads, st, c->jpeg, err);
    return rc ? fail(rc, err) : 0;
}

int sift_mi_get_stats(sift_mi_ctx* c, sift_mi_stats* out) {
    if (!c || !out) return fail(SIFT_MI_EINVAL, "bad arguments");
    *out = c->stats;
    if (c->count_samples && c->samples.p) {
        CHK(set_device(c));
        CHK(sync_lanes(c));
        unsigned long long h[16];
        HIPCHK(hipMemcpy(h, c->samples.p, sizeof h, hipMemcpyDeviceToHost));
        out->orient_samples = out->desc_samples = 0;
        for (int i = 0; i < 8; i++) {
            out->orient_samples += h[i];
            out->desc_samples += h[8 + i];
        }
    }
    return 0;
}

int sift_mi_reset_stats(sift_mi_ctx* c) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    c->stats = sift_mi_stats{};
    if (c->samples.p) {
        CHK(set_device(c));
        CHK(sync_lanes(c));
        HIPCHK(hipMemset(c->samples.p, 0, 16 * sizeof(unsigned long long)));
    }
    return 0;
}

int sift_mi_set_sample_counting(sift_mi_ctx* c, int on) {
    if (!c) return fail(SIFT_MI_EINVAL, "ctx is null");
    CHK(set_device(c));
    CHK(sync_lanes(c));
    if (on && !c->samples.p) {
        CHK(c->samples.ensure(16));
        HIPCHK(hipMemset(c->samples.p, 0, 16 * sizeof(unsigned long long)));
    }
    c->count_samples = on ? 1 : 0;
    return 0;
}

}  // extern "C"
