// Gaussian scale space + DoG on MI355X (gfx950).
//
// Reference: precompute_images / create_seed_image / build_gaussian_scale_space
// / build_dog (src/lib.rs:131-279) with the OpenCVProcessing backend
// (src/opencv_processing.rs:38-74): cv::resize INTER_LINEAR for the 2x seed,
// cv::GaussianBlur (separable, BORDER_REFLECT_101) for every blur and
// cv::resize INTER_NEAREST for the octave step.
//
// Kernels (all batched over frames with blockIdx.z):
//   k_upsample2x  u8 frame -> f32 2x bilinear seed (OpenCV half-pixel
//                 coefficients, separately rounded products)
//   k_blur_dog<R> one separable blur G_{s-1} -> G_s staged through LDS:
//                 coalesced tile+halo load, register-blocked row pass
//                 (4 outputs/thread, ds_read_b128), register-blocked column
//                 pass (8 outputs/thread); the epilogue also writes
//                 D_{s-1} = G_s - G_{s-1} and, for s == 3, the next
//                 octave's base image (nearest 1/2: pixel (2x, 2y)).
// The stage is HBM-bound: per octave pixel it must write 6 G + 5 D images
// (44 B); see DESIGN.md for the roofline accounting.
#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {

// ---------------------------------------------------------------------------
// Seed: u8 -> f32 (v / 255, image::ConvertBuffer, src/lib.rs:198) -> 2x
// bilinear (cv::resize INTER_LINEAR, src/lib.rs:201-205).  Coefficient tables
// are built on the host with OpenCV's formulas (resizeGeneric_).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_upsample2x(const uint8_t* __restrict__ frames, size_t frame_pitch,
                                                    size_t row_stride, int sw, int sh, const ResizeTab tab,
                                                    float* __restrict__ dst, size_t dst_img_stride, int dw,
                                                    int dh) {
    const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (dx >= dw || dy >= dh) return;
    const uint8_t* src = frames + (size_t)blockIdx.z * frame_pitch;
    const int sx = tab.xofs[dx];
    const float a0 = tab.xa0[dx], a1 = tab.xa1[dx];
    const bool two = dx < tab.xmax;
    const int sy0 = tab.yofs[dy];
    const int sy1 = sy0 + 1 < sh ? sy0 + 1 : sh - 1;
    const uint8_t* r0 = src + (size_t)sy0 * row_stride;
    const uint8_t* r1 = src + (size_t)sy1 * row_stride;
    const int sx1 = two ? sx + 1 : sx;
    const float p00 = (float)r0[sx] / 255.0f, p01 = (float)r0[sx1] / 255.0f;
    const float p10 = (float)r1[sx] / 255.0f, p11 = (float)r1[sx1] / 255.0f;
    // HResizeLinear: t = S[sx]*a0 + S[sx+1]*a1 (two roundings + add)
    const float h0 = two ? p00 * a0 + p01 * a1 : p00;
    const float h1 = two ? p10 * a0 + p11 * a1 : p10;
    // VResizeLinear: S0*b0 + S1*b1
    dst[(size_t)blockIdx.z * dst_img_stride + (size_t)dy * dw + dx] = h0 * tab.ya0[dy] + h1 * tab.ya1[dy];
}

// ---------------------------------------------------------------------------
// Separable Gaussian blur, OpenCV FilterEngine order:
//   row pass   RowVec_32f:       acc = x[-R]*k[-R]; acc = fma(x[t], k[t], acc) t = -R+1..R
//   column pass SymmColumnVec_32f: acc = c*k0; acc = fma(up_t + down_t, k_t, acc) t = 1..R
// Borders: BORDER_REFLECT_101 on both axes (the column border rows are
// row-filtered reflected source rows, exactly as FilterEngine builds them).
// ---------------------------------------------------------------------------
template <int R>
struct BlurGeom {
    static constexpr int TW = 64;                     // output tile width
    static constexpr int TH = 32;                     // output tile height
    static constexpr int VB = 8;                      // column outputs per thread
    static constexpr int IH = TH + 2 * R;             // input / row-pass rows
    static constexpr int IW = TW + 2 * R;             // input columns used
    static constexpr int NV = (2 * R + 4 + 3) / 4;    // float4 reads per row-pass item
    static constexpr int IWP = TW - 4 + 4 * NV;       // padded input pitch (>= IW, %4 == 0)
    static constexpr int LDS_FLOATS = IH * IWP + IH * TW;
};

template <int R>
__global__ __launch_bounds__(256) void k_blur_dog(const float* __restrict__ src, size_t src_img_stride,
                                                  float* __restrict__ dst, size_t dst_img_stride,
                                                  float* __restrict__ dog, size_t dog_img_stride,
                                                  float* __restrict__ nxt, size_t nxt_img_stride, int wn, int hn,
                                                  int W, int H, const BlurTaps taps) {
    using G = BlurGeom<R>;
    static_assert(G::IWP >= G::IW, "pitch");
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    float* tin = lds;                  // [IH][IWP] G_{s-1} tile + halo
    float* th = lds + G::IH * G::IWP;  // [IH][TW]  row-pass output
    const int tid = threadIdx.x;
    const int x0 = blockIdx.x * G::TW, y0 = blockIdx.y * G::TH;
    const size_t b = blockIdx.z;
    src += b * src_img_stride;

    // 1. tile + halo -> LDS (coalesced along rows, reflect-101 at the borders)
    for (int i = tid; i < G::IH * G::IW; i += 256) {
        const int ly = i / G::IW, lx = i - ly * G::IW;
        const int gy = reflect101(y0 - R + ly, H), gx = reflect101(x0 - R + lx, W);
        tin[ly * G::IWP + lx] = src[(size_t)gy * W + gx];
    }
    __syncthreads();

    // 2. row pass: item = (row, quad of 4 outputs); taps read as float4
    for (int i = tid; i < G::IH * (G::TW / 4); i += 256) {
        const int ly = i / (G::TW / 4), q = i - ly * (G::TW / 4);
        const float4* rp = reinterpret_cast<const float4*>(tin + ly * G::IWP + 4 * q);
        float v[4 * G::NV];
#pragma unroll
        for (int j = 0; j < G::NV; j++) {
            const float4 f = rp[j];
            v[4 * j + 0] = f.x;
            v[4 * j + 1] = f.y;
            v[4 * j + 2] = f.z;
            v[4 * j + 3] = f.w;
        }
        float acc[4];
#pragma unroll
        for (int o = 0; o < 4; o++) acc[o] = v[o] * taps.k[R];
#pragma unroll
        for (int t = 1; t <= 2 * R; t++) {
            const float kt = taps.k[t > R ? t - R : R - t];
#pragma unroll
            for (int o = 0; o < 4; o++) acc[o] = __builtin_fmaf(v[o + t], kt, acc[o]);
        }
        *reinterpret_cast<float4*>(th + ly * G::TW + 4 * q) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
    __syncthreads();

    // 3. column pass: item = (column, VB consecutive outputs)
    for (int i = tid; i < G::TW * (G::TH / G::VB); i += 256) {
        const int lx = i & (G::TW - 1), p = i / G::TW;
        const int gx = x0 + lx;
        float v[G::VB + 2 * R];
#pragma unroll
        for (int j = 0; j < G::VB + 2 * R; j++) v[j] = th[(p * G::VB + j) * G::TW + lx];
        if (gx >= W) continue;
#pragma unroll
        for (int o = 0; o < G::VB; o++) {
            const int ly = p * G::VB + o;
            const int gy = y0 + ly;
            if (gy >= H) break;
            float acc = v[o + R] * taps.k[0];
#pragma unroll
            for (int t = 1; t <= R; t++) acc = __builtin_fmaf(v[o + R + t] + v[o + R - t], taps.k[t], acc);
            const size_t off = (size_t)gy * W + gx;
            dst[b * dst_img_stride + off] = acc;
            if (dog) dog[b * dog_img_stride + off] = acc - tin[(ly + R) * G::IWP + lx + R];
            if (nxt && !(gx & 1) && !(gy & 1) && (gx >> 1) < wn && (gy >> 1) < hn)
                nxt[b * nxt_img_stride + (size_t)(gy >> 1) * wn + (gx >> 1)] = acc;
        }
    }
}

template <int R>
static void launch_blur_r(const BlurLaunch& L, hipStream_t st) {
    using G = BlurGeom<R>;
    dim3 grid((L.W + G::TW - 1) / G::TW, (L.H + G::TH - 1) / G::TH, L.n_img);
    hipLaunchKernelGGL(k_blur_dog<R>, grid, dim3(256), 0, st, L.src, L.src_img_stride, L.dst, L.dst_img_stride, L.dog,
                       L.dog_img_stride, L.nxt, L.nxt_img_stride, L.wn, L.hn, L.W, L.H, L.taps);
}

int launch_blur(int R, const BlurLaunch& L, hipStream_t st) {
    switch (R) {
#define CASE(r) \
    case r:     \
        launch_blur_r<r>(L, st); return 0;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10) CASE(11) CASE(12)
        CASE(13) CASE(14) CASE(15) CASE(16) CASE(17) CASE(18) CASE(19) CASE(20) CASE(21) CASE(22) CASE(23) CASE(24)
#undef CASE
        default:
            return -1;
    }
}

void launch_upsample2x(const uint8_t* frames, size_t frame_pitch, size_t row_stride, int sw, int sh,
                       const ResizeTab& tab, float* dst, size_t dst_img_stride, int n_img, hipStream_t st) {
    const int dw = 2 * sw, dh = 2 * sh;
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, n_img);
    hipLaunchKernelGGL(k_upsample2x, grid, dim3(256), 0, st, frames, frame_pitch, row_stride, sw, sh, tab, dst,
                       dst_img_stride, dw, dh);
}

// ---------------------------------------------------------------------------
// Processing-trait op kernels on a single f32 image (src/lib.rs:86-90):
// generic bilinear / nearest resize used by sift_mi_resize_* (op parity only).
// ---------------------------------------------------------------------------
__global__ void k_resize_linear_f32(const float* __restrict__ src, int sw, int sh, const ResizeTab tab,
                                    float* __restrict__ dst, int dw, int dh) {
    const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (dx >= dw || dy >= dh) return;
    const int sx = tab.xofs[dx];
    const bool two = dx < tab.xmax;
    const int sx1 = two ? sx + 1 : sx;
    const int sy0 = tab.yofs[dy];
    const int sy1 = sy0 + 1 < sh ? sy0 + 1 : sh - 1;
    const float* r0 = src + (size_t)sy0 * sw;
    const float* r1 = src + (size_t)sy1 * sw;
    const float h0 = two ? r0[sx] * tab.xa0[dx] + r0[sx1] * tab.xa1[dx] : r0[sx];
    const float h1 = two ? r1[sx] * tab.xa0[dx] + r1[sx1] * tab.xa1[dx] : r1[sx];
    dst[(size_t)dy * dw + dx] = h0 * tab.ya0[dy] + h1 * tab.ya1[dy];
}

__global__ void k_resize_nearest_f32(const float* __restrict__ src, int sw, const int* __restrict__ xofs,
                                     const int* __restrict__ yofs, float* __restrict__ dst, int dw, int dh) {
    const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (dx >= dw || dy >= dh) return;
    dst[(size_t)dy * dw + dx] = src[(size_t)yofs[dy] * sw + xofs[dx]];
}

void launch_resize_linear_f32(const float* src, int sw, int sh, const ResizeTab& tab, float* dst, int dw, int dh,
                              hipStream_t st) {
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, 1);
    hipLaunchKernelGGL(k_resize_linear_f32, grid, dim3(256), 0, st, src, sw, sh, tab, dst, dw, dh);
}

void launch_resize_nearest_f32(const float* src, int sw, const int* xofs, const int* yofs, float* dst, int dw, int dh,
                               hipStream_t st) {
    dim3 grid((dw + 63) / 64, (dh + 3) / 4, 1);
    hipLaunchKernelGGL(k_resize_nearest_f32, grid, dim3(256), 0, st, src, sw, xofs, yofs, dst, dw, dh);
}

}  // namespace siftmi
