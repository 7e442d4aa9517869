/*
 * sift_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference SIFT hot path (tnibler/sift-features,
 * src/lib.rs @ 2024-10-22), used as the parity checker for the MI355X HIP
 * path and as the `cpu_baseline` ("port") leg of bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product path (sift-features_amd/) never links or calls it.
 *
 * Pinning: the reference's only test (`sift_end2end`, src/lib.rs:1009-1056)
 * runs `sift_with_processing::<OpenCVProcessing>` and snapshots the result
 * (src/snapshots/sift__sift_end2end*.snap).  tests/test_oracle_golden.py checks this file
 * against those snapshots.  The OpenCV blur/resize semantics restated in the
 * PROFILE_OPENCV section follow OpenCV 4.x (imgproc smooth/filter/resize:
 * bit-exact Gaussian kernel, BORDER_REFLECT_101, FMA row/column passes,
 * half-pixel bilinear, floor nearest) -- a third-party dependency that is not
 * in /root/reference (src/opencv_processing.rs:38-74 is the call site).
 *
 * Arithmetic rules (so results equal the Rust code's on x86-64):
 *  - compiled with -ffp-contract=off: no implicit FMA (Rust never contracts);
 *    explicit fmaf() only where OpenCV's SIMD filters fuse;
 *  - glibc expf/atan2/sinf/cosf/powf/log2f (Rust's f32/f64 methods call the
 *    platform libm);
 *  - Rust `.round()` is half-away-from-zero == C roundf();
 *  - Rust `as` casts saturate (f32 -> int: NaN -> 0).
 */
#include <float.h>
#include <stddef.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SCALES_PER_OCTAVE 3
#define N_IMAGES_PER_OCTAVE (SCALES_PER_OCTAVE + 3)
#define N_DOG_PER_OCTAVE (SCALES_PER_OCTAVE + 2)
#define IMAGE_BORDER 5
#define ORI_BINS 36
#define DESC_HIST 4
#define DESC_BINS 8
#define DESC_SIZE 128

enum { PROFILE_OPENCV = 0, PROFILE_IMAGEPROC = 1 };

typedef struct {
    float x, y, size, angle, response;
} okp_t;

/* Internal keypoint (src/lib.rs:58-68 SiftKeyPoint) + emission key. */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, scale;
    /* emission position (octave, s_init, y_init, x_init, peak k) */
    int32_t s_init, y_init, x_init, peak;
} osk_t;

typedef struct {
    int n_octaves;
    int* w;
    int* h;
    float** gauss; /* [o] -> 6*h*w */
    float** dog;   /* [o] -> 5*h*w */
} opyr_t;

/* ------------------------------------------------------------------ */
/* Rust-cast helpers                                                   */
/* ------------------------------------------------------------------ */
static int64_t sat_i64(float v) {
    if (v != v) return 0;
    if (v >= 9.2233720368547758e18f) return INT64_MAX;
    if (v <= -9.2233720368547758e18f) return INT64_MIN;
    return (int64_t)v;
}
static int32_t sat_i32(float v) {
    if (v != v) return 0;
    if (v >= 2147483647.0f) return INT32_MAX;
    if (v <= -2147483648.0f) return INT32_MIN;
    return (int32_t)v;
}
static uint64_t sat_usize(float v) {
    if (!(v > 0.0f)) return 0; /* NaN and negatives -> 0 */
    if (v >= 1.8446744073709552e19f) return UINT64_MAX;
    return (uint64_t)v;
}

/* compiler-rt __powidf2 (Rust f64::powi lowers to llvm.powi). */
static double powi_f64(double a, int b) {
    const int recip = b < 0;
    double r = 1;
    for (;;) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1 / r : r;
}
static float powi_f32(float a, int b) {
    const int recip = b < 0;
    float r = 1;
    for (;;) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1 / r : r;
}

/* ------------------------------------------------------------------ */
/* PROFILE_OPENCV: OpenCVProcessing (src/opencv_processing.rs:38-74)   */
/* ------------------------------------------------------------------ */

/* cv::GaussianBlur(Size(), sigma) on CV_32F: ksize = cvRound(sigma*4*2+1)|1 */
int oracle_cv_ksize(double sigma) { return ((int)lrint(sigma * 4 * 2 + 1)) | 1; }

/* getGaussianKernelBitExact (OpenCV 4.x) evaluated in IEEE double, cast to f32. */
void oracle_cv_kernel(int n, double sigma, float* out) {
    const double scale2X = -0.125 / (sigma * sigma);
    if (n > 511) n = 511;
    const int n2 = (n - 1) / 2;
    double values[256];
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        double t = exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2;
    sum += 1;
    if ((n & 1) == 0) sum += 1;
    const double mul1 = 1 / sum;
    for (int i = 0; i < n2; i++) {
        double t = values[i] * mul1;
        out[i] = (float)t;
        out[n - 1 - i] = (float)t;
    }
    out[n2] = (float)(1.0 * mul1);
    if ((n & 1) == 0) out[n2 + 1] = out[n2];
}

/* cv::borderInterpolate, BORDER_REFLECT_101 */
static inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) {
        if (p < 0)
            p = -p;
        else
            p = 2 * len - 2 - p;
    }
    return p;
}

/* Arithmetic-variant switch for pinning experiments against the snapshots
 * (tools only; 0 = the restatement documented above). */
static int g_variant = 0;
void oracle_set_variant(int v) { g_variant = v; }

/* Separable filter: RowFilter<float,float,RowVec_32f> (fma chain from the
 * leftmost tap), then SymmColumnFilter<SymmColumnVec_32f> (centre product,
 * then fma of the (below+above) pair sums outwards). */
static void cv_blur(const float* src, int w, int h, double sigma, float* dst) {
    int kx = oracle_cv_ksize(sigma), ky = kx;
    if (h == 1) ky = 1;
    if (w == 1) kx = 1;
    if (kx == 1 && ky == 1) {
        memcpy(dst, src, sizeof(float) * (size_t)w * h);
        return;
    }
    if (oracle_cv_ksize(sigma) > 511) return;
    float kern[512];
    oracle_cv_kernel(oracle_cv_ksize(sigma), sigma, kern);
    float kxv[512], kyv[512];
    if (kx == 1)
        kxv[0] = 1.0f;
    else
        memcpy(kxv, kern, sizeof(float) * kx);
    if (ky == 1)
        kyv[0] = 1.0f;
    else
        memcpy(kyv, kern, sizeof(float) * ky);
    const int rx = kx / 2, ry = ky / 2;
    float* tmp = (float*)malloc(sizeof(float) * (size_t)w * h);
    int* xo = (int*)malloc(sizeof(int) * (size_t)(w + 2 * rx));
    for (int i = 0; i < w + 2 * rx; i++) xo[i] = reflect101(i - rx, w);
    for (int y = 0; y < h; y++) {
        const float* s = src + (size_t)y * w;
        float* t = tmp + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            float acc;
            if (g_variant & 64) {  /* symmetric pairs from the centre */
                acc = s[xo[x + rx]] * kxv[rx];
                for (int k = 1; k <= rx; k++) acc = fmaf(s[xo[x + rx - k]] + s[xo[x + rx + k]], kxv[rx + k], acc);
            } else {
                acc = s[xo[x]] * kxv[0];
                for (int k = 1; k < kx; k++)
                    acc = (g_variant & 8) ? acc + s[xo[x + k]] * kxv[k] : fmaf(s[xo[x + k]], kxv[k], acc);
            }
            t[x] = acc;
        }
    }
    const float* kc = kyv + ry;
    for (int y = 0; y < h; y++) {
        float* d = dst + (size_t)y * w;
        const float* c = tmp + (size_t)y * w;
        if (g_variant & 32) {  /* plain fma chain from the top tap */
            for (int x = 0; x < w; x++) {
                float acc = tmp[(size_t)reflect101(y - ry, h) * w + x] * kyv[0];
                for (int k = 1; k < ky; k++) acc = fmaf(tmp[(size_t)reflect101(y - ry + k, h) * w + x], kyv[k], acc);
                d[x] = acc;
            }
            continue;
        }
        for (int x = 0; x < w; x++) d[x] = c[x] * kc[0];
        for (int k = 1; k <= ry; k++) {
            const float* dn = tmp + (size_t)reflect101(y + k, h) * w;
            const float* up = tmp + (size_t)reflect101(y - k, h) * w;
            for (int x = 0; x < w; x++)
                d[x] = (g_variant & 16) ? d[x] + (dn[x] + up[x]) * kc[k] : fmaf(dn[x] + up[x], kc[k], d[x]);
        }
    }
    free(xo);
    free(tmp);
}

/* cv::resize INTER_LINEAR (resizeGeneric_, HResizeLinear + VResizeLinear,
 * baseline-SIMD build: products rounded separately, no FMA). */
static void cv_resize_coeffs(int ssz, int dsz, int* ofs, float* a0, float* a1, int* lim) {
    const double inv = (double)dsz / ssz;
    const double scale = 1. / inv;
    int xmax = dsz;
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

static void cv_resize_linear(const float* src, int sw, int sh, int dw, int dh, float* dst) {
    int* xo = (int*)malloc(sizeof(int) * dw);
    float* xa0 = (float*)malloc(sizeof(float) * dw);
    float* xa1 = (float*)malloc(sizeof(float) * dw);
    int* yo = (int*)malloc(sizeof(int) * dh);
    float* ya0 = (float*)malloc(sizeof(float) * dh);
    float* ya1 = (float*)malloc(sizeof(float) * dh);
    int xmax, ymax;
    cv_resize_coeffs(sw, dw, xo, xa0, xa1, &xmax);
    cv_resize_coeffs(sh, dh, yo, ya0, ya1, &ymax);
    (void)ymax;
    float* hb = (float*)malloc(sizeof(float) * (size_t)sh * dw);
    for (int y = 0; y < sh; y++) {
        const float* s = src + (size_t)y * sw;
        float* t = hb + (size_t)y * dw;
        for (int x = 0; x < dw; x++) {
            int sx = xo[x];
            if (x < xmax)
                t[x] = (g_variant & 4) ? fmaf(s[sx], xa0[x], s[sx + 1] * xa1[x]) : s[sx] * xa0[x] + s[sx + 1] * xa1[x];
            else
                t[x] = s[sx];
        }
    }
    for (int y = 0; y < dh; y++) {
        int r0 = yo[y], r1 = yo[y] + 1 < sh ? yo[y] + 1 : sh - 1;
        const float* s0 = hb + (size_t)r0 * dw;
        const float* s1 = hb + (size_t)r1 * dw;
        float* d = dst + (size_t)y * dw;
        for (int x = 0; x < dw; x++)
            d[x] = (g_variant & 1)   ? fmaf(s0[x], ya0[y], s1[x] * ya1[y])
                   : (g_variant & 2) ? fmaf(s1[x], ya1[y], s0[x] * ya0[y])
                                     : s0[x] * ya0[y] + s1[x] * ya1[y];
    }
    free(hb);
    free(xo);
    free(xa0);
    free(xa1);
    free(yo);
    free(ya0);
    free(ya1);
}

/* cv::resize INTER_NEAREST (resizeNN): sx = min(floor(x * (1/(dw/sw))), sw-1) */
static void cv_resize_nearest(const float* src, int sw, int sh, int dw, int dh, float* dst) {
    const double ifx = 1. / ((double)dw / sw), ify = 1. / ((double)dh / sh);
    int* xo = (int*)malloc(sizeof(int) * dw);
    for (int x = 0; x < dw; x++) {
        int sx = (int)floor(x * ifx);
        xo[x] = sx < sw - 1 ? sx : sw - 1;
    }
    for (int y = 0; y < dh; y++) {
        int sy = (int)floor(y * ify);
        if (sy > sh - 1) sy = sh - 1;
        const float* s = src + (size_t)sy * sw;
        float* d = dst + (size_t)y * dw;
        for (int x = 0; x < dw; x++) d[x] = s[xo[x]];
    }
    free(xo);
}

/* ------------------------------------------------------------------ */
/* PROFILE_IMAGEPROC: ImageprocProcessing (src/lib.rs:993-1007)         */
/* Third-party code absent from /root/reference, restated from the      */
/* published crates: imageproc 0.25.0 filter::gaussian_blur_f32 and     */
/* image 0.25.2 imageops::resize (Triangle, Nearest).  No reference     */
/* test runs this profile: PARITY UNPINNED.                 */
/* ------------------------------------------------------------------ */

/* imageproc gaussian_kernel_f32: radius ceil(2 sigma), taps
 * (sqrt(2 pi) r)^-1 * exp(-x^2 / (2 r^2)) in f32, normalised by their f32 sum
 * (summed in index order). */
int oracle_ip_kernel(float sigma, float* k) {
    const int r = (int)ceilf(2.0f * sigma);
    const int n = 2 * r + 1;
    const float norm = 1.0f / (sqrtf(2.0f * 3.14159265358979323846f) * sigma);
    for (int i = 0; i <= r; i++) {
        const float x = (float)i;
        const float v = norm * expf(-(x * x) / (2.0f * (sigma * sigma)));
        k[r + i] = v;
        k[r - i] = v;
    }
    float sum = 0.0f;
    for (int i = 0; i < n; i++) sum += k[i];
    for (int i = 0; i < n; i++) k[i] = k[i] / sum;
    return n;
}

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* separable_filter_equal: horizontal then vertical, acc = acc + p * k from the
 * first tap (unfused), clamp-to-edge borders; f32 output is not clamped. */
static void ip_blur(const float* src, int w, int h, float sigma, float* dst) {
    float k[64];
    const int n = oracle_ip_kernel(sigma, k), r = n / 2;
    float* tmp = (float*)malloc(sizeof(float) * (size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            float acc = 0.0f;
            for (int i = 0; i < n; i++) acc = acc + src[(size_t)y * w + clampi(x + i - r, 0, w - 1)] * k[i];
            tmp[(size_t)y * w + x] = acc;
        }
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            float acc = 0.0f;
            for (int i = 0; i < n; i++) acc = acc + tmp[(size_t)clampi(y + i - r, 0, h - 1) * w + x] * k[i];
            dst[(size_t)y * w + x] = acc;
        }
    free(tmp);
}

/* image::imageops::sample weights for one axis (vertical_sample /
 * horizontal_sample): taps [left, right) with f32 weights normalised by their
 * f32 sum.  support 1 = Triangle, 0 = Nearest (box). */
int oracle_ip_axis(int src, int dst, int out, float support, int* left, float* wts) {
    const float ratio = (float)src / (float)dst;
    const float sratio = ratio < 1.0f ? 1.0f : ratio;
    const float src_support = support * sratio;
    float in = ((float)out + 0.5f) * ratio;
    long l = (long)floorf(in - src_support);
    l = l < 0 ? 0 : (l > src - 1 ? src - 1 : l);
    long rt = (long)ceilf(in + src_support);
    rt = rt < l + 1 ? l + 1 : (rt > src ? src : rt);
    in = in - 0.5f;
    float sum = 0.0f;
    int n = 0;
    for (long i = l; i < rt; i++) {
        float wv;
        if (support > 0.0f) {
            const float t = fabsf(((float)i - in) / sratio);
            wv = t < 1.0f ? 1.0f - t : 0.0f;
        } else {
            wv = 1.0f; /* box_kernel */
        }
        wts[n++] = wv;
        sum += wv;
    }
    for (int i = 0; i < n; i++) wts[i] = wts[i] / sum;
    *left = (int)l;
    return n;
}

/* image::imageops::resize: vertical_sample into an f32 intermediate, then
 * horizontal_sample, t = t + p * w (unfused) from the first tap; the result
 * is clamped to [0, 1] (f32 DEFAULT_MIN/MAX_VALUE). */
static void ip_resize(const float* src, int sw, int sh, int dw, int dh, float support, float* dst) {
    if (sw == dw && sh == dh) {
        memcpy(dst, src, sizeof(float) * (size_t)sw * sh);
        return;
    }
    float* tmp = (float*)malloc(sizeof(float) * (size_t)sw * dh);
    float wts[4096];
    for (int y = 0; y < dh; y++) {
        int l;
        const int n = oracle_ip_axis(sh, dh, y, support, &l, wts);
        for (int x = 0; x < sw; x++) {
            float t = 0.0f;
            for (int i = 0; i < n; i++) t = t + src[(size_t)(l + i) * sw + x] * wts[i];
            tmp[(size_t)y * sw + x] = t;
        }
    }
    for (int x = 0; x < dw; x++) {
        int l;
        const int n = oracle_ip_axis(sw, dw, x, support, &l, wts);
        for (int y = 0; y < dh; y++) {
            float t = 0.0f;
            for (int i = 0; i < n; i++) t = t + tmp[(size_t)y * sw + l + i] * wts[i];
            dst[(size_t)y * dw + x] = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
        }
    }
    free(tmp);
}

/* Processing trait (src/lib.rs:86-90) dispatch. */
int oracle_gaussian_blur(const float* src, int w, int h, double sigma, int profile, float* dst) {
    if (profile == PROFILE_IMAGEPROC) {
        ip_blur(src, w, h, (float)sigma, dst);
        return 0;
    }
    if (profile != PROFILE_OPENCV) return -1;
    cv_blur(src, w, h, sigma, dst);
    return 0;
}
int oracle_resize_linear(const float* src, int sw, int sh, int dw, int dh, int profile, float* dst) {
    if (profile == PROFILE_IMAGEPROC) {
        ip_resize(src, sw, sh, dw, dh, 1.0f, dst);
        return 0;
    }
    if (profile != PROFILE_OPENCV) return -1;
    cv_resize_linear(src, sw, sh, dw, dh, dst);
    return 0;
}
int oracle_resize_nearest(const float* src, int sw, int sh, int dw, int dh, int profile, float* dst) {
    if (profile == PROFILE_IMAGEPROC) {
        ip_resize(src, sw, sh, dw, dh, 0.0f, dst);
        return 0;
    }
    if (profile != PROFILE_OPENCV) return -1;
    cv_resize_nearest(src, sw, sh, dw, dh, dst);
    return 0;
}

/* ------------------------------------------------------------------ */
/* precompute_images (src/lib.rs:131-143)                              */
/* ------------------------------------------------------------------ */

/* n_octaves = round(log2(min(2W,2H)) - 2) as usize + 1  (src/lib.rs:133-134) */
int oracle_n_octaves(int w, int h) {
    int m = 2 * w < 2 * h ? 2 * w : 2 * h;
    float f = roundf(log2f((float)m) - 2.0f);
    return (int)sat_usize(f) + 1;
}

/* Incremental blur sigmas (src/lib.rs:220-229), index 0..5 */
void oracle_octave_sigmas(double* sig) {
    const double m = pow(2.0, 2.0 / SCALES_PER_OCTAVE);
    for (int s = 0; s < N_IMAGES_PER_OCTAVE; s++) {
        double a = powi_f64(m, s - 1);
        double b = a * m;
        sig[s] = sqrt(b - a) * 0.8 * 2.0;
    }
}
double oracle_seed_sigma(void) { return sqrt(0.8 * 0.8 - 0.5 * 0.5) * 2.0; }

void oracle_pyramid_free(opyr_t* p) {
    if (!p) return;
    for (int o = 0; o < p->n_octaves; o++) {
        free(p->gauss[o]);
        free(p->dog[o]);
    }
    free(p->gauss);
    free(p->dog);
    free(p->w);
    free(p->h);
    free(p);
}

opyr_t* oracle_precompute(const uint8_t* img, int w, int h, int stride, int profile) {
    if ((profile != PROFILE_OPENCV && profile != PROFILE_IMAGEPROC) || w < 1 || h < 1) return NULL;
    /* create_seed_image (src/lib.rs:196-210) */
    float* f = (float*)malloc(sizeof(float) * (size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) f[(size_t)y * w + x] = (float)img[(size_t)y * stride + x] / 255.0f;
    const int W0 = 2 * w, H0 = 2 * h;
    float* up = (float*)malloc(sizeof(float) * (size_t)W0 * H0);
    oracle_resize_linear(f, w, h, W0, H0, profile, up);
    free(f);
    opyr_t* p = (opyr_t*)calloc(1, sizeof(opyr_t));
    p->n_octaves = oracle_n_octaves(w, h);
    p->w = (int*)calloc(p->n_octaves, sizeof(int));
    p->h = (int*)calloc(p->n_octaves, sizeof(int));
    p->gauss = (float**)calloc(p->n_octaves, sizeof(float*));
    p->dog = (float**)calloc(p->n_octaves, sizeof(float*));
    double sig[N_IMAGES_PER_OCTAVE];
    oracle_octave_sigmas(sig);
    /* build_gaussian_scale_space (src/lib.rs:213-267) */
    int ow = W0, oh = H0;
    for (int o = 0; o < p->n_octaves; o++) {
        const size_t P = (size_t)ow * oh;
        p->w[o] = ow;
        p->h[o] = oh;
        p->gauss[o] = (float*)malloc(sizeof(float) * P * N_IMAGES_PER_OCTAVE);
        p->dog[o] = (float*)malloc(sizeof(float) * P * N_DOG_PER_OCTAVE);
        float* G = p->gauss[o];
        if (o == 0) {
            oracle_gaussian_blur(up, ow, oh, oracle_seed_sigma(), profile, G);
        } else {
            const float* prev = p->gauss[o - 1] + (size_t)3 * p->w[o - 1] * p->h[o - 1];
            oracle_resize_nearest(prev, p->w[o - 1], p->h[o - 1], ow, oh, profile, G);
        }
        for (int s = 1; s < N_IMAGES_PER_OCTAVE; s++)
            oracle_gaussian_blur(G + (s - 1) * P, ow, oh, sig[s], profile, G + s * P);
        /* build_dog (src/lib.rs:271-279) */
        for (int s = 0; s < N_DOG_PER_OCTAVE; s++)
            for (size_t i = 0; i < P; i++) p->dog[o][s * P + i] = G[(s + 1) * P + i] - G[s * P + i];
        ow = ow / 2;
        oh = oh / 2;
    }
    free(up);
    return p;
}

int oracle_pyramid_n_octaves(const opyr_t* p) { return p->n_octaves; }
void oracle_pyramid_dims(const opyr_t* p, int o, int* w, int* h) {
    *w = p->w[o];
    *h = p->h[o];
}
const float* oracle_pyramid_gauss(const opyr_t* p, int o) { return p->gauss[o]; }
const float* oracle_pyramid_dog(const opyr_t* p, int o) { return p->dog[o]; }

/* ------------------------------------------------------------------ */
/* keypoint detection (src/lib.rs:281-757)                             */
/* ------------------------------------------------------------------ */

/* point_is_local_extremum (src/lib.rs:437-506) */
static int is_extremum(const float* prev, const float* curr, const float* next, int w, int x, int y) {
    const float threshold = floorf(0.5f * 0.04f / (float)SCALES_PER_OCTAVE);
    const size_t c = (size_t)y * w + x;
    const float val = curr[c];
    static const int dyv[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
    static const int dxv[8] = {-1, 0, 1, -1, 1, -1, 0, 1};
    if (fabsf(val) <= threshold) return 0;
    const float* sl[3] = {curr, prev, next};
    if (val > 0.0f) {
        for (int s = 0; s < 3; s++)
            for (int i = 0; i < 8; i++)
                if (!(val >= sl[s][c + (ptrdiff_t)dyv[i] * w + dxv[i]])) return 0;
        return val >= fmaxf(prev[c], next[c]);
    } else {
        for (int s = 0; s < 3; s++)
            for (int i = 0; i < 8; i++)
                if (!(val <= sl[s][c + (ptrdiff_t)dyv[i] * w + dxv[i]])) return 0;
        return val <= fminf(prev[c], next[c]);
    }
}

typedef struct {
    int scale, x, y;
    float off_s, off_x, off_y;
} interp_t;

/* interpolate_extremum (src/lib.rs:525-603) */
static int interpolate(const float* dog, int w, int h, int scale, int x, int y, interp_t* out) {
    const size_t P = (size_t)w * h;
    for (int it = 0; it < 5; it++) {
        const float* prev = dog + (size_t)(scale - 1) * P;
        const float* curr = dog + (size_t)scale * P;
        const float* next = dog + (size_t)(scale + 1) * P;
#define AT(a, yy, xx) (a)[(size_t)(yy) * w + (xx)]
        const float g1 = (AT(next, y, x) - AT(prev, y, x)) / 2.f;
        const float g2 = (AT(curr, y + 1, x) - AT(curr, y - 1, x)) / 2.f;
        const float g3 = (AT(curr, y, x + 1) - AT(curr, y, x - 1)) / 2.f;
        const float v2 = AT(curr, y, x) * 2.f;
        const float h11 = AT(next, y, x) + AT(prev, y, x) - v2;
        const float h12 = (AT(next, y + 1, x) - AT(next, y - 1, x) - AT(prev, y + 1, x) + AT(prev, y - 1, x)) / 4.f;
        const float h13 = (AT(next, y, x + 1) - AT(next, y, x - 1) - AT(prev, y, x + 1) + AT(prev, y, x - 1)) / 4.f;
        const float h22 = AT(curr, y + 1, x) + AT(curr, y - 1, x) - v2;
        const float h33 = AT(curr, y, x + 1) + AT(curr, y, x - 1) - v2;
        const float h23 =
            (AT(curr, y + 1, x + 1) - AT(curr, y + 1, x - 1) - AT(curr, y - 1, x + 1) + AT(curr, y - 1, x - 1)) / 4.f;
#undef AT
        const float det =
            h11 * h22 * h33 - h11 * h23 * h23 - h12 * h12 * h33 + 2.f * h12 * h13 * h23 - h13 * h13 * h22;
        const float i11 = (h22 * h33 - h23 * h23) / det;
        const float i12 = (h13 * h23 - h12 * h33) / det;
        const float i13 = (h12 * h23 - h13 * h22) / det;
        const float i22 = (h11 * h33 - h13 * h13) / det;
        const float i23 = (h12 * h13 - h11 * h23) / det;
        const float i33 = (h11 * h22 - h12 * h12) / det;
        const float os = -(i11 * g1 + i12 * g2 + i13 * g3);
        const float ox = -(i13 * g1 + i23 * g2 + i33 * g3);
        const float oy = -(i12 * g1 + i22 * g2 + i23 * g3);
        if (fabsf(os) < 0.5f && fabsf(ox) < 0.5f && fabsf(oy) < 0.5f) {
            out->scale = scale;
            out->x = x;
            out->y = y;
            out->off_s = os;
            out->off_x = ox;
            out->off_y = oy;
            return 1;
        }
        /* saturating `as isize`; clamp so the int64 sum cannot overflow */
        int64_t rx = sat_i64(roundf(ox)), ry = sat_i64(roundf(oy)), rs = sat_i64(roundf(os));
        const int64_t LIM = (int64_t)1 << 40;
        if (rx > LIM || rx < -LIM || ry > LIM || ry < -LIM || rs > LIM || rs < -LIM) return 0;
        const int64_t nx = x + rx, ny = y + ry, ns = scale + rs;
        if (!(ns >= 1 && ns <= SCALES_PER_OCTAVE) || nx < IMAGE_BORDER || nx >= w - IMAGE_BORDER || ny < IMAGE_BORDER ||
            ny >= h - IMAGE_BORDER)
            return 0;
        x = (int)nx;
        y = (int)ny;
        scale = (int)ns;
    }
    return 0;
}

/* extremum_contrast (src/lib.rs:606-626) */
static float contrast_at(const float* dog, int w, int h, const interp_t* p) {
    const size_t P = (size_t)w * h;
    const float* prev = dog + (size_t)(p->scale - 1) * P;
    const float* curr = dog + (size_t)p->scale * P;
    const float* next = dog + (size_t)(p->scale + 1) * P;
    const size_t c = (size_t)p->y * w + p->x;
    const float g1 = (next[c] - prev[c]) / 2.f;
    const float g2 = (curr[c + w] - curr[c - w]) / 2.f;
    const float g3 = (curr[c + 1] - curr[c - 1]) / 2.f;
    const float interp = p->off_s * g1 + p->off_y * g2 + p->off_x * g3;
    return curr[c] + interp / 2.f;
}

/* extremum_is_on_edge (src/lib.rs:630-653) */
static int on_edge(const float* curr, int w, int x, int y) {
    const size_t c = (size_t)y * w + x;
    const float v2 = curr[c] * 2.0f;
    const float h11 = curr[c + w] + curr[c - w] - v2;
    const float d22 = curr[c + 1] + curr[c - 1] - v2;
    const float h12 = (curr[c + w + 1] - curr[c + w - 1] - curr[c - w + 1] + curr[c - w - 1]) / 4.f;
    const float tr = d22 + h11;
    const float det = d22 * h11 - h12 * h12;
    if (det <= 0.f) return 1;
    return (tr * tr * 10.0f) > 121.0f * det;
}

/* gradient_direction_histogram (src/lib.rs:657-757), n_bins = 36 */
void oracle_orientation_hist(const float* img, int w, int h, int x, int y, int radius, float sigma, float* hist) {
    const int n_bins = ORI_BINS;
    const float gws = -1.0f / (2.0f * sigma * sigma);
    const float bin_step = (float)n_bins / (3.14159265358979323846f * 2.f);
    float raw[ORI_BINS + 4];
    for (int i = 0; i < n_bins + 4; i++) raw[i] = 0.0f;
    for (int yp = -radius; yp <= radius; yp++) {
        if (yp <= -y) continue;
        const int64_t yy = (int64_t)y + yp;
        if (yy <= 0 || yy >= h - 1) continue;
        for (int xp = -radius; xp <= radius; xp++) {
            if (xp <= -x) continue;
            const int64_t xx = (int64_t)x + xp;
            if (xx <= 0 || xx >= w - 1) continue;
            const float* r = img + (size_t)yy * w;
            const float dx = r[xx + 1] - r[xx - 1];
            const float dy = img[(size_t)(yy - 1) * w + xx] - img[(size_t)(yy + 1) * w + xx];
            const float wexp = (float)(yp * yp + xp * xp) * gws;
            const float weight = expf(wexp);
            const float mag = sqrtf(dx * dx + dy * dy);
            const float ori = (float)atan2((double)dy, (double)dx);
            const float raw_bin = bin_step * ori;
            int bin = sat_i32(roundf(raw_bin));
            if (bin >= n_bins)
                bin -= n_bins;
            else if (bin < 0)
                bin += n_bins;
            raw[bin + 2] += weight * mag;
        }
    }
    raw[1] = raw[n_bins + 1];
    raw[0] = raw[n_bins];
    raw[n_bins + 2] = raw[2];
    raw[n_bins + 3] = raw[3];
    for (int i = 2; i < n_bins + 2; i++)
        hist[i - 2] =
            (raw[i - 2] + raw[i + 2]) * (1.f / 16.f) + (raw[i - 1] + raw[i + 1]) * (4.f / 16.f) + raw[i] * 6.f / 16.f;
}

typedef struct {
    osk_t* v;
    size_t n, cap;
} kpvec_t;

static void kp_push(kpvec_t* k, const osk_t* kp) {
    if (k->n == k->cap) {
        k->cap = k->cap ? 2 * k->cap : 1024;
        k->v = (osk_t*)realloc(k->v, sizeof(osk_t) * k->cap);
    }
    k->v[k->n++] = *kp;
}

/* find_keypoints (src/lib.rs:281-294) + find_extrema_in_dog_img (:299-435) */
static void find_keypoints(const opyr_t* p, kpvec_t* out) {
    for (int o = 0; o < p->n_octaves; o++) {
        const int w = p->w[o], h = p->h[o];
        const size_t P = (size_t)w * h;
        const float* dog = p->dog[o];
        for (int s_in = 1; s_in <= SCALES_PER_OCTAVE; s_in++) {
            if (h < 2 * IMAGE_BORDER || w < 2 * IMAGE_BORDER) continue;
            const float* prev = dog + (size_t)(s_in - 1) * P;
            const float* curr = dog + (size_t)s_in * P;
            const float* next = dog + (size_t)(s_in + 1) * P;
            for (int y0 = IMAGE_BORDER; y0 < h - IMAGE_BORDER; y0++) {
                for (int x0 = IMAGE_BORDER; x0 < w - IMAGE_BORDER; x0++) {
                    if (!is_extremum(prev, curr, next, w, x0, y0)) continue;
                    interp_t pt;
                    if (!interpolate(dog, w, h, s_in, x0, y0, &pt)) continue;
                    const float contrast = fabsf(contrast_at(dog, w, h, &pt));
                    if (contrast * (float)SCALES_PER_OCTAVE <= 0.04f) continue;
                    if (on_edge(dog + (size_t)pt.scale * P, w, pt.x, pt.y)) continue;
                    const float osf = powi_f32(2.0f, o);
                    const float kp_scale =
                        (float)0.8 * ((g_variant & 128) ? exp2f(((float)pt.scale + pt.off_s) / (float)SCALES_PER_OCTAVE) : powf(2.0f, ((float)pt.scale + pt.off_s) / (float)SCALES_PER_OCTAVE)) * 2.f;
                    const float kp_x = ((float)pt.x + pt.off_x) * osf;
                    const float kp_y = ((float)pt.y + pt.off_y) * osf;
                    const int radius = sat_i32(roundf(3.f * 1.5f * kp_scale));
                    float hist[ORI_BINS];
                    oracle_orientation_hist(p->gauss[o] + (size_t)pt.scale * P, w, h, pt.x, pt.y, radius,
                                            1.5f * kp_scale, hist);
                    float hmax = hist[0];
                    for (int i = 1; i < ORI_BINS; i++)
                        if (hist[i] > hmax) hmax = hist[i];
                    const float thr = hmax * 0.8f;
                    for (int k = 0; k < ORI_BINS; k++) {
                        const int km = k > 0 ? k - 1 : ORI_BINS - 1;
                        const int kq = k < ORI_BINS - 1 ? k + 1 : 0;
                        if (hist[k] > hist[km] && hist[k] > hist[kq] && hist[k] >= thr) {
                            const float interp = (hist[km] - hist[kq]) / (hist[km] - 2.0f * hist[k] + hist[kq]);
                            float bin = (float)k + 0.5f * interp;
                            if (bin < 0.0f)
                                bin = (float)ORI_BINS + bin;
                            else if (bin >= (float)ORI_BINS)
                                bin = bin - (float)ORI_BINS;
                            osk_t kp;
                            kp.x = kp_x;
                            kp.y = kp_y;
                            kp.size = kp_scale * osf;
                            kp.response = contrast;
                            kp.octave = o;
                            kp.scale = pt.scale;
                            kp.angle = 360.0f - (360.0f / (float)ORI_BINS) * bin;
                            kp.s_init = s_in;
                            kp.y_init = y0;
                            kp.x_init = x0;
                            kp.peak = k;
                            kp_push(out, &kp);
                        }
                    }
                }
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* compute_descriptor (src/lib.rs:785-990)                              */
/* ------------------------------------------------------------------ */
void oracle_compute_descriptor(const float* img, int width, int height, float xf, float yf, float scale,
                               float orientation, uint8_t* out) {
    const int n_hist = DESC_HIST, n_bins = DESC_BINS;
    const uint64_t x = sat_usize(roundf(xf));
    const uint64_t y = sat_usize(roundf(yf));
    const float BIN_ANGLE_STEP = (float)DESC_BINS / 360.0f;
    const float hist_width = 3.0f * scale;
    const int radius = sat_i32(roundf(3.0f * scale * sqrtf(2.0f) * (float)(n_hist + 1) * 0.5f));
    const float rad = orientation * (3.14159265358979323846f / 180.0f);
    const float sin_ori = sinf(rad), cos_ori = cosf(rad);
    const float sin_s = sin_ori / hist_width, cos_s = cos_ori / hist_width;
    float hist[6][6][DESC_BINS];
    memset(hist, 0, sizeof(hist));
    for (int yi = -radius; yi <= radius; yi++) {
        for (int xi = -radius; xi <= radius; xi++) {
            const float col_rot = (float)xi * cos_s - (float)yi * sin_s;
            const float row_rot = (float)xi * sin_s + (float)yi * cos_s;
            float row_bin = row_rot + (float)(n_hist / 2);
            float col_bin = col_rot + (float)(n_hist / 2);
            const int32_t ay = (int32_t)y + yi;
            const int32_t ax = (int32_t)x + xi;
            if (!(row_bin > -0.5f && row_bin < (float)n_hist + 0.5f && col_bin > -0.5f &&
                  col_bin < (float)n_hist + 0.5f && ay > 0 && ay < height - 1 && ax > 0 && ax < width - 1))
                continue;
            const float* r = img + (size_t)ay * width;
            const float dx = r[ax + 1] - r[ax - 1];
            const float dy = img[(size_t)(ay - 1) * width + ax] - img[(size_t)(ay + 1) * width + ax];
            const float wsq = col_rot * col_rot + row_rot * row_rot;
            const float weight = expf(wsq * (-2.f / (float)(n_hist * n_hist)));
            const double deg = atan2((double)dy, (double)dx) * (180.0 / 3.14159265358979323846);
            const float ori = (float)fmod(deg + 360.0, 360.0) - orientation;
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
            const uint64_t r1 = sat_usize(row_floor + 1.f), cc1 = sat_usize(col_floor + 1.f);
            const uint64_t r2 = sat_usize(row_floor + 2.f), cc2 = sat_usize(col_floor + 2.f);
            float of = ori_floor;
            if (of < 0.f)
                of = of + (float)n_bins;
            else if (of >= (float)n_bins)
                of = of - (float)n_bins;
            const uint64_t o0 = sat_usize(of);
            const uint64_t o1 = o0 + 1 >= (uint64_t)n_bins ? 0 : o0 + 1;
            hist[r1][cc1][o0] += c000;
            hist[r1][cc1][o1] += c001;
            hist[r1][cc2][o0] += c010;
            hist[r1][cc2][o1] += c011;
            hist[r2][cc1][o0] += c100;
            hist[r2][cc1][o1] += c101;
            hist[r2][cc2][o0] += c110;
            hist[r2][cc2][o1] += c111;
        }
    }
    float flat[DESC_SIZE];
    int i = 0;
    for (int r = 1; r < 5; r++)
        for (int c = 1; c < 5; c++)
            for (int o = 0; o < n_bins; o++) flat[i++] = hist[r][c][o];
    float l2 = 0.0f;
    for (int ch = 0; ch < DESC_SIZE / 4; ch++) {
        float s = 0.0f;
        for (int j = 0; j < 4; j++) s += flat[4 * ch + j] * flat[4 * ch + j];
        l2 = ch == 0 ? s : l2 + s;
    }
    l2 = sqrtf(l2);
    const float cap = l2 * 0.2f;
    for (int j = 0; j < DESC_SIZE; j++) flat[j] = fminf(flat[j], cap);
    float l2c = 0.0f;
    for (int ch = 0; ch < DESC_SIZE / 4; ch++) {
        float s = 0.0f;
        for (int j = 0; j < 4; j++) s += flat[4 * ch + j] * flat[4 * ch + j];
        l2c = ch == 0 ? s : l2c + s;
    }
    l2c = sqrtf(l2c);
    const float norm = 512.0f / fmaxf(l2c, FLT_EPSILON);
    for (int j = 0; j < DESC_SIZE; j++) {
        const int32_t v = sat_i32(roundf(flat[j] * norm));
        out[j] = v > 255 ? 255 : (uint8_t)v;
    }
}

/* ------------------------------------------------------------------ */
/* sift_with_precomputed (src/lib.rs:147-177)                           */
/* ------------------------------------------------------------------ */
typedef struct {
    size_t n;
    okp_t* kps;     /* public KeyPoint (x,y,size x0.5) */
    osk_t* ext;     /* internal SiftKeyPoint + emission key */
    uint8_t* desc;  /* n*128 */
} ores_t;

static int cmp_resp_desc(const void* a, const void* b) {
    const osk_t* ka = (const osk_t*)a;
    const osk_t* kb = (const osk_t*)b;
    if (ka->response > kb->response) return -1;
    if (ka->response < kb->response) return 1;
    return 0;
}

/* features_limit < 0 == None.  With a limit, ties in response keep emission
 * order (the reference's sort_unstable_by leaves tie order unspecified). */
ores_t* oracle_sift_with_precomputed(const opyr_t* p, int64_t features_limit) {
    kpvec_t kv = {0};
    find_keypoints(p, &kv);
    if (features_limit >= 0 && (size_t)features_limit < kv.n) {
        /* stable: decorate with emission index via merge of qsort on index */
        osk_t* tmp = kv.v;
        size_t n = kv.n;
        /* simple stable insertion by merge sort */
        osk_t* buf = (osk_t*)malloc(sizeof(osk_t) * n);
        for (size_t width = 1; width < n; width *= 2) {
            for (size_t lo = 0; lo < n; lo += 2 * width) {
                size_t mid = lo + width < n ? lo + width : n;
                size_t hi = lo + 2 * width < n ? lo + 2 * width : n;
                size_t a = lo, b = mid, k = lo;
                while (a < mid && b < hi) buf[k++] = cmp_resp_desc(&tmp[b], &tmp[a]) < 0 ? tmp[b++] : tmp[a++];
                while (a < mid) buf[k++] = tmp[a++];
                while (b < hi) buf[k++] = tmp[b++];
            }
            memcpy(tmp, buf, sizeof(osk_t) * n);
        }
        free(buf);
        kv.n = (size_t)features_limit;
    }
    ores_t* r = (ores_t*)calloc(1, sizeof(ores_t));
    r->n = kv.n;
    r->ext = kv.v;
    r->kps = (okp_t*)malloc(sizeof(okp_t) * (kv.n ? kv.n : 1));
    r->desc = (uint8_t*)malloc((size_t)DESC_SIZE * (kv.n ? kv.n : 1));
    /* compute_descriptors (src/lib.rs:759-782) */
    for (size_t i = 0; i < kv.n; i++) {
        const osk_t* kp = &kv.v[i];
        const int w = p->w[kp->octave], h = p->h[kp->octave];
        const float* img = p->gauss[kp->octave] + (size_t)kp->scale * w * h;
        const float angle = 360.0f - kp->angle;
        const float osf = powi_f32(2.0f, -kp->octave);
        const float kp_size = kp->size * osf;
        oracle_compute_descriptor(img, w, h, kp->x * osf, kp->y * osf, kp_size, angle, r->desc + i * DESC_SIZE);
        r->kps[i].x = kp->x * 0.5f;
        r->kps[i].y = kp->y * 0.5f;
        r->kps[i].size = kp->size * 0.5f;
        r->kps[i].angle = kp->angle;
        r->kps[i].response = kp->response;
    }
    return r;
}

/* sift_with_processing (src/lib.rs:76-81) */
ores_t* oracle_sift(const uint8_t* img, int w, int h, int stride, int profile, int64_t features_limit) {
    opyr_t* p = oracle_precompute(img, w, h, stride, profile);
    if (!p) return NULL;
    ores_t* r = oracle_sift_with_precomputed(p, features_limit);
    oracle_pyramid_free(p);
    return r;
}

size_t oracle_result_n(const ores_t* r) { return r->n; }
const okp_t* oracle_result_keypoints(const ores_t* r) { return r->kps; }
const osk_t* oracle_result_internal(const ores_t* r) { return r->ext; }
const uint8_t* oracle_result_descriptors(const ores_t* r) { return r->desc; }
void oracle_result_free(ores_t* r) {
    if (!r) return;
    free(r->kps);
    free(r->ext);
    free(r->desc);
    free(r);
}

/* ------------------------------------------------------------------ */
/* Descriptor matching (examples/sift-match.rs:30-35):                  */
/* cv::BFMatcher(NORM_L2, crossCheck).match(query, train).              */
/* distance = sqrt((float) exact integer L2^2) (batchDistL2_8u32f);     */
/* nearest = first minimum (strict <); cross check = mutual nearest     */
/* (cv::batchDistance crosscheck).  train_idx[i] = -1: no match.        */
/* ------------------------------------------------------------------ */
static uint32_t l2sq_u8(const uint8_t* a, const uint8_t* b) {
    uint32_t s = 0;
    for (int k = 0; k < DESC_SIZE; k++) {
        const int d = (int)a[k] - (int)b[k];
        s += (uint32_t)(d * d);
    }
    return s;
}

void oracle_match(const uint8_t* q, int nq, const uint8_t* t, int nt, int cross_check, int* train_idx,
                  float* dist) {
    int* tq = (int*)malloc(sizeof(int) * (size_t)(nt > 0 ? nt : 1));
    for (int j = 0; j < nt; j++) { /* nearest query of each train row */
        uint32_t best = 0xffffffffu;
        int bi = -1;
        for (int i = 0; i < nq; i++) {
            const uint32_t d = l2sq_u8(q + (size_t)i * DESC_SIZE, t + (size_t)j * DESC_SIZE);
            if (d < best) {
                best = d;
                bi = i;
            }
        }
        tq[j] = bi;
    }
    for (int i = 0; i < nq; i++) {
        uint32_t best = 0xffffffffu;
        int bj = -1;
        for (int j = 0; j < nt; j++) {
            const uint32_t d = l2sq_u8(q + (size_t)i * DESC_SIZE, t + (size_t)j * DESC_SIZE);
            if (d < best) {
                best = d;
                bj = j;
            }
        }
        if (bj >= 0 && (!cross_check || tq[bj] == i)) {
            train_idx[i] = bj;
            dist[i] = sqrtf((float)best);
        } else {
            train_idx[i] = -1;
            dist[i] = 0.0f;
        }
    }
    free(tq);
}
