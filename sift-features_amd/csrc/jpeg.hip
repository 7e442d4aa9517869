// Input step before the path: baseline JPEG -> 8-bit
// luma exactly as the reference's inputs are made -- image 0.25.2
// `image::open(..)` / `load_from_memory(..)` (zune-jpeg backend) followed by
// `.grayscale()` (examples/run-sift.rs:8; the test inputs of src/lib.rs:1012).
//
// Entropy decoding (ITU-T T.81 F.2: markers, Huffman, dequantisation) is
// sequential and runs on the host; the reconstruction runs on the GPU:
//   * zune-jpeg's integer IDCT: stb_image's 12-bit fixed-point arithmetic
//     with the row-pass bias 512 + 65536 + (128 << 17), and blocks whose 63
//     AC coefficients are zero becoming (DC >> 3) + 128 (k_jpeg_idct, one
//     thread per 8x8 block);
//   * chroma upsampling in two 3:1 triangle passes, vertical then
//     horizontal, each (3a + b + 2) >> 2, edges clamped on the padded block
//     plane; zune's 6-bit fixed-point YCbCr -> RGB (45/32, 11/32, 23/32,
//     113/64); luma = (2126 R + 7152 G + 722 B) / 10000 (k_jpeg_luma, one
//     thread per pixel).
// This is the arithmetic tests/golden/jpeg_decode.py restates and that
// reproduces the reference's snapshots (tests/golden/make_golden.py, DESIGN.md
// 5): decoding the reference's test JPEGs gives the golden fixtures' images
// bit for bit (tests/test_gpu_jpeg.py).  Baseline / extended sequential
// Huffman only (SOF0/SOF1), 1 or 3 components, sampling factors 1 or 2,
// restart intervals.
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sift_mi.h"
#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {
namespace jpg {

constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                             41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                             30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

#ifndef SIFT_JPEG_FAST_AC
#define SIFT_JPEG_FAST_AC 11
#endif
constexpr int kFastAc = SIFT_JPEG_FAST_AC;

// canonical Huffman decoding tables (T.81 F.2.2.3) plus a 9-bit lookahead
struct Huff {
    bool present = false;
    int maxcode[17], valptr[17], mincode[17];
    uint8_t sym[256];
    uint16_t fast[512];  // (code length << 8) | symbol for codes of <= 9 bits; 0: walk the lengths
    // AC run/size symbol and its extra bits in one kFastAc-bit lookup (code
    // length + size <= kFastAc, size > 0): (coefficient << 16) | (run << 8) | bits used
    int32_t fast_ac[1 << kFastAc];
};

struct Comp {
    int id, h, v, tq, td, ta;
};

struct Header {
    int w = 0, h = 0, nc = 0, restart = 0;
    Comp c[3];
    int32_t q[4][64];  // natural order
    bool qset[4] = {false, false, false, false};
    Huff dc[4], ac[4];
    size_t scan = 0;  // first entropy-coded byte
};

// T.81 bit reader with byte stuffing: 0xFF 0x00 is a data 0xFF; any other
// marker feeds zero bits and is not consumed (tests/golden/jpeg_decode.py _Bits)
class Bits {
    const uint8_t* d;
    size_t n, p;
    uint64_t acc = 0;
    int cnt = 0;

  public:
    Bits(const uint8_t* d_, size_t n_, size_t p_) : d(d_), n(n_), p(p_) {}
    void fill() {
        while (cnt <= 56) {
            if (p + 8 <= n) {  // 8 bytes at once when none of them is 0xFF
                uint64_t v;
                std::memcpy(&v, d + p, 8);
                v = __builtin_bswap64(v);
                const uint64_t x = ~v;  // a 0xFF byte of v is a zero byte of x
                if (((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull) == 0) {
                    const int k = (64 - cnt) >> 3;  // 1..8 whole bytes fit
                    acc = k == 8 ? v : (acc << (8 * k)) | (v >> (64 - 8 * k));
                    p += k;
                    cnt += 8 * k;
                    continue;
                }
            }
            uint32_t b = 0;
            if (p < n) {
                b = d[p];
                if (b == 0xFF) {
                    const uint32_t nx = p + 1 < n ? d[p + 1] : 0;
                    if (nx == 0x00)
                        p += 2;
                    else
                        b = 0;
                } else {
                    p++;
                }
            }
            acc = (acc << 8) | b;
            cnt += 8;
        }
    }
    // at least 32 buffered bits: a Huffman code (<= 16) plus its extra bits (<= 16)
    void refill() {
        if (cnt < 32) fill();
    }
    int peek9() {
        refill();
        return (int)((acc >> (cnt - 9)) & 511u);
    }
    int peek_ac() {  // kFastAc bits, after refill()
        return (int)((acc >> (cnt - kFastAc)) & ((1u << kFastAc) - 1));
    }
    void skip(int k) { cnt -= k; }
    int bits(int k) {
        if (!k) return 0;
        refill();
        cnt -= k;
        return (int)((acc >> cnt) & ((1ull << k) - 1));
    }
    void restart() {  // drop the buffered bits, skip the RSTn marker
        acc = 0;
        cnt = 0;
        while (p + 1 < n && !(d[p] == 0xFF && d[p + 1] >= 0xD0 && d[p + 1] <= 0xD7)) p++;
        p += 2;
    }
};

bool build_huff(const uint8_t* counts, const uint8_t* syms, int nsym, Huff& t) {
    if (nsym > 256) return false;
    std::memcpy(t.sym, syms, nsym);
    std::memset(t.fast, 0, sizeof(t.fast));
    int code = 0, k = 0;
    for (int ln = 1; ln <= 16; ln++) {
        t.maxcode[ln] = -1;
        t.valptr[ln] = 0;
        t.mincode[ln] = 0;
        if (counts[ln - 1]) {
            t.valptr[ln] = k;
            t.mincode[ln] = code;
            for (int i = 0; i < counts[ln - 1]; i++, code++, k++) {
                if (ln <= 9) {
                    const int lo = code << (9 - ln), hi = (code + 1) << (9 - ln);
                    for (int x = lo; x < hi && x < 512; x++) t.fast[x] = (uint16_t)((ln << 8) | t.sym[k]);
                }
            }
            t.maxcode[ln] = code - 1;
        }
        code <<= 1;
    }
    // combined AC lookups: every kFastAc-bit window whose leading code has
    // length ln <= 10 and whose symbol's extra bits also fit
    std::memset(t.fast_ac, 0, sizeof(t.fast_ac));
    for (int x = 0; x < (1 << kFastAc); x++) {
        for (int ln = 1; ln <= kFastAc; ln++) {
            const int c = x >> (kFastAc - ln);
            if (c > t.maxcode[ln]) continue;
            const int rs = t.sym[t.valptr[ln] + c - t.mincode[ln]];
            const int r = rs >> 4, sz = rs & 15;
            if (sz && ln + sz <= kFastAc) {
                const int raw = (x >> (kFastAc - ln - sz)) & ((1 << sz) - 1);
                const int v = (raw < (1 << (sz - 1))) ? raw - (1 << sz) + 1 : raw;  // extend()
                t.fast_ac[x] = (int32_t)((uint32_t)(v & 0xffff) << 16 | (uint32_t)(r << 8) | (uint32_t)(ln + sz));
            }
            break;
        }
    }
    t.present = true;
    return true;
}

int decode_sym(Bits& bs, const Huff& t) {
    const uint16_t f = t.fast[bs.peek9()];
    if (f) {
        bs.skip(f >> 8);
        return f & 0xff;
    }
    int code = bs.bits(1);
    for (int ln = 1; ln <= 16; ln++) {
        if (code <= t.maxcode[ln]) return t.sym[t.valptr[ln] + code - t.mincode[ln]];
        code = (code << 1) | bs.bits(1);
    }
    return -1;
}

inline int extend(int v, int t) { return (t && v < (1 << (t - 1))) ? v - (1 << t) + 1 : v; }

// Markers up to the first SOS (tests/golden/jpeg_decode.py parse).  Returns
// 0, or a status with `err` set.
int parse(const uint8_t* d, size_t n, Header& H, std::string& err) {
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return err = "not a JPEG (no SOI)", SIFT_MI_EINVAL;
    size_t p = 2;
    bool frame = false;
    while (p + 4 <= n) {
        if (d[p] != 0xFF) return err = "JPEG: marker expected", SIFT_MI_EINVAL;
        while (p + 1 < n && d[p + 1] == 0xFF) p++;  // fill bytes
        const int m = d[p + 1];
        p += 2;
        if (m == 0xD9) break;
        if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // no length
        if (p + 2 > n) break;
        const size_t ln = ((size_t)d[p] << 8) | d[p + 1];
        if (ln < 2 || p + ln > n) return err = "JPEG: truncated segment", SIFT_MI_EINVAL;
        const uint8_t* seg = d + p + 2;
        const size_t sl = ln - 2;
        if (m == 0xDB) {  // DQT
            size_t i = 0;
            while (i < sl) {
                const int pq = seg[i] >> 4, tq = seg[i] & 15;
                i++;
                if (tq > 3 || i + (pq ? 128 : 64) > sl) return err = "JPEG: bad DQT", SIFT_MI_EINVAL;
                for (int k = 0; k < 64; k++) {
                    const int v = pq ? ((int)seg[i + 2 * k] << 8) | seg[i + 2 * k + 1] : seg[i + k];
                    H.q[tq][kZigzag[k]] = v;
                }
                i += pq ? 128 : 64;
                H.qset[tq] = true;
            }
        } else if (m == 0xC4) {  // DHT
            size_t i = 0;
            while (i + 17 <= sl) {
                const int tc = seg[i] >> 4, th = seg[i] & 15;
                int nsym = 0;
                for (int k = 0; k < 16; k++) nsym += seg[i + 1 + k];
                if (tc > 1 || th > 3 || i + 17 + nsym > sl) return err = "JPEG: bad DHT", SIFT_MI_EINVAL;
                if (!build_huff(seg + i + 1, seg + i + 17, nsym, tc ? H.ac[th] : H.dc[th]))
                    return err = "JPEG: bad DHT", SIFT_MI_EINVAL;
                i += 17 + nsym;
            }
        } else if (m == 0xC0 || m == 0xC1) {  // baseline / extended sequential Huffman
            if (sl < 6) return err = "JPEG: bad SOF", SIFT_MI_EINVAL;
            H.h = (seg[1] << 8) | seg[2];
            H.w = (seg[3] << 8) | seg[4];
            H.nc = seg[5];
            if (seg[0] != 8) return err = "JPEG: only 8-bit samples", SIFT_MI_EUNSUPPORTED;
            if (!(H.nc == 1 || H.nc == 3) || sl < 6 + 3 * (size_t)H.nc)
                return err = "JPEG: 1 or 3 components only", SIFT_MI_EUNSUPPORTED;
            for (int k = 0; k < H.nc; k++) {
                Comp& c = H.c[k];
                c.id = seg[6 + 3 * k];
                c.h = seg[7 + 3 * k] >> 4;
                c.v = seg[7 + 3 * k] & 15;
                c.tq = seg[8 + 3 * k] & 3;
                c.td = c.ta = 0;
                if (c.h < 1 || c.h > 2 || c.v < 1 || c.v > 2)
                    return err = "JPEG: sampling factors 1 or 2 only", SIFT_MI_EUNSUPPORTED;
            }
            frame = true;
        } else if ((m >= 0xC2 && m <= 0xC3) || (m >= 0xC5 && m <= 0xC7) || (m >= 0xC9 && m <= 0xCB) ||
                   (m >= 0xCD && m <= 0xCF)) {
            return err = "JPEG: only baseline sequential Huffman", SIFT_MI_EUNSUPPORTED;
        } else if (m == 0xDD) {
            if (sl < 2) return err = "JPEG: bad DRI", SIFT_MI_EINVAL;
            H.restart = (seg[0] << 8) | seg[1];
        } else if (m == 0xDA) {  // SOS
            if (!frame) return err = "JPEG: SOS before SOF", SIFT_MI_EINVAL;
            // T.81 B.2.3: Ns, Ns x (Cs, Td/Ta), Ss, Se, Ah/Al
            if (sl < 1 || sl < 1 + 2 * (size_t)seg[0] + 3) return err = "JPEG: truncated SOS", SIFT_MI_EINVAL;
            const int ns = seg[0];
            if (ns != H.nc) return err = "JPEG: one interleaved scan only", SIFT_MI_EUNSUPPORTED;
            for (int k = 0; k < ns; k++) {
                const int cid = seg[1 + 2 * k], tt = seg[2 + 2 * k];
                for (int j = 0; j < H.nc; j++)
                    if (H.c[j].id == cid) {
                        H.c[j].td = (tt >> 4) & 3;
                        H.c[j].ta = tt & 3;
                    }
            }
            H.scan = p + ln;
            if (H.w < 1 || H.h < 1) return err = "JPEG: empty frame", SIFT_MI_EINVAL;
            return 0;
        }
        p += ln;
    }
    return err = "JPEG: no frame / scan", SIFT_MI_EINVAL;
}

// Geometry of the padded block planes (tests/golden/jpeg_decode.py _scan).
struct Geom {
    int hmax, vmax, mcux, mcuy;
    int bw[3], bh[3];       // blocks per row / column of each component's plane
    size_t off[3], total;   // block offsets of the planes in the coefficient array
};

Geom geometry(const Header& H) {
    Geom g{};
    g.hmax = g.vmax = 1;
    for (int k = 0; k < H.nc; k++) {
        g.hmax = std::max(g.hmax, H.c[k].h);
        g.vmax = std::max(g.vmax, H.c[k].v);
    }
    g.mcux = (H.w + 8 * g.hmax - 1) / (8 * g.hmax);
    g.mcuy = (H.h + 8 * g.vmax - 1) / (8 * g.vmax);
    g.total = 0;
    for (int k = 0; k < H.nc; k++) {
        g.bw[k] = g.mcux * H.c[k].h;
        g.bh[k] = g.mcuy * H.c[k].v;
        g.off[k] = g.total;
        g.total += (size_t)g.bw[k] * g.bh[k];
    }
    return g;
}

// Entropy decoding + dequantisation: coef[block][64], natural order.
// Quantised coefficients (natural order, int16: AC magnitudes are < 2^10 by
// construction; a DC predictor leaving the int16 range is rejected), the GPU
// dequantises.  Every block of every plane is coded (MCU order), so `coef` is
// written in full: each block is assembled in a zeroed local array and stored
// whole.
int entropy_decode(const uint8_t* d, size_t n, const Header& H, const Geom& g, int16_t* coef, std::string& err) {
    for (int k = 0; k < H.nc; k++) {
        if (!H.qset[H.c[k].tq]) return err = "JPEG: missing quantisation table", SIFT_MI_EINVAL;
        if (!H.dc[H.c[k].td].present || !H.ac[H.c[k].ta].present)
            return err = "JPEG: missing Huffman table", SIFT_MI_EINVAL;
    }
    Bits bs(d, n, H.scan);
    int pred[3] = {0, 0, 0};
    long long mcu = 0;
    for (int my = 0; my < g.mcuy; my++) {
        for (int mx = 0; mx < g.mcux; mx++) {
            if (H.restart && mcu && mcu % H.restart == 0) {
                bs.restart();
                pred[0] = pred[1] = pred[2] = 0;
            }
            mcu++;
            for (int ci = 0; ci < H.nc; ci++) {
                const Comp& c = H.c[ci];
                const Huff& dct = H.dc[c.td];
                const Huff& act = H.ac[c.ta];
                for (int by = 0; by < c.v; by++) {
                    for (int bx = 0; bx < c.h; bx++) {
                        int16_t* dst =
                            coef + 64 * (g.off[ci] + (size_t)(my * c.v + by) * g.bw[ci] + (size_t)(mx * c.h + bx));
                        int16_t* __restrict__ blk = dst;  // natural order, written in place
                        std::memset(blk, 0, 64 * sizeof(int16_t));
                        const int t = decode_sym(bs, dct);
                        if (t < 0 || t > 16) return err = "JPEG: bad Huffman code", SIFT_MI_EINVAL;
                        pred[ci] += extend(bs.bits(t), t);
                        if (pred[ci] < -32768 || pred[ci] > 32767)
                            return err = "JPEG: DC coefficient out of range", SIFT_MI_EUNSUPPORTED;
                        blk[0] = (int16_t)pred[ci];
                        for (int k = 1; k < 64;) {
                            bs.refill();
                            const int32_t fa = act.fast_ac[bs.peek_ac()];
                            if (fa) {  // run, size and coefficient in one lookup
                                k += (fa >> 8) & 15;
                                bs.skip(fa & 255);
                                if (k > 63) return err = "JPEG: coefficient index out of range", SIFT_MI_EINVAL;
                                blk[kZigzag[k]] = (int16_t)(fa >> 16);
                                k++;
                                continue;
                            }
                            const int rs = decode_sym(bs, act);
                            if (rs < 0) return err = "JPEG: bad Huffman code", SIFT_MI_EINVAL;
                            const int r = rs >> 4, s = rs & 15;
                            if (s == 0) {
                                if (r != 15) break;
                                k += 16;
                                continue;
                            }
                            k += r;
                            if (k > 63) return err = "JPEG: coefficient index out of range", SIFT_MI_EINVAL;
                            blk[kZigzag[k]] = (int16_t)extend(bs.bits(s), s);
                            k++;
                        }
                    }
                }
            }
        }
    }
    return 0;
}

// ---------------------------------------------------------------------------
// GPU reconstruction
// ---------------------------------------------------------------------------
constexpr int f2f(double x) { return (int)(x * 4096 + 0.5); }  // stb_image stbi__f2f (truncation as in C)

struct Idct1 {
    int64_t x0, x1, x2, x3, t0, t1, t2, t3;
};

// stbi__IDCT_1D: the even part in x0..x3, the odd part in t0..t3
__device__ __forceinline__ Idct1 idct1d(int64_t s0, int64_t s1, int64_t s2, int64_t s3, int64_t s4, int64_t s5,
                                        int64_t s6, int64_t s7) {
    Idct1 o;
    int64_t p2 = s2, p3 = s6;
    int64_t p1 = (p2 + p3) * f2f(0.5411961);
    int64_t t2 = p1 + p3 * f2f(-1.847759065);
    int64_t t3 = p1 + p2 * f2f(0.765366865);
    p2 = s0;
    p3 = s4;
    int64_t t0 = (p2 + p3) * 4096;
    int64_t t1 = (p2 - p3) * 4096;
    o.x0 = t0 + t3;
    o.x3 = t0 - t3;
    o.x1 = t1 + t2;
    o.x2 = t1 - t2;
    t0 = s7;
    t1 = s5;
    t2 = s3;
    t3 = s1;
    p3 = t0 + t2;
    int64_t p4 = t1 + t3;
    p1 = t0 + t3;
    p2 = t1 + t2;
    const int64_t p5 = (p3 + p4) * f2f(1.175875602);
    t0 = t0 * f2f(0.298631336);
    t1 = t1 * f2f(2.053119869);
    t2 = t2 * f2f(3.072711026);
    t3 = t3 * f2f(1.501321110);
    p1 = p5 + p1 * f2f(-0.899976223);
    p2 = p5 + p2 * f2f(-2.562915447);
    p3 = p3 * f2f(-1.961570560);
    p4 = p4 * f2f(-0.390180644);
    o.t3 = t3 + p1 + p4;
    o.t2 = t2 + p2 + p3;
    o.t1 = t1 + p2 + p4;
    o.t0 = t0 + p1 + p3;
    return o;
}

__device__ __forceinline__ uint8_t clamp_u8(int64_t v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

struct Planes {
    uint8_t* p[3];  // frame 0's planes; frame f's at + f * frame_bytes
    int pitch[3];   // = bw * 8
    int bw[3];
    size_t off[3];  // first block of each component in a frame's coefficients
    size_t frame_blocks, frame_bytes;
    const int32_t* qtab;  // per frame: 3 x 64 quantisation tables (components' order, natural order)
    int nc;
};

// one thread per 8x8 block: zune-jpeg's IDCT (see the file comment)
__global__ __launch_bounds__(256) void k_jpeg_idct(const int16_t* __restrict__ coef, size_t nblk, const Planes P) {
    constexpr int64_t kRowBias = 512 + 65536 + (128 << 17);
    const size_t b = (size_t)blockIdx.x * 256 + threadIdx.x;  // over all frames
    if (b >= nblk) return;
    const size_t f = b / P.frame_blocks, fb = b - f * P.frame_blocks;
    int ci = 0;
    while (ci + 1 < P.nc && fb >= P.off[ci + 1]) ci++;
    const size_t lb = fb - P.off[ci];
    const int by = (int)(lb / P.bw[ci]), bx = (int)(lb - (size_t)by * P.bw[ci]);
    uint8_t* out = P.p[ci] + f * P.frame_bytes + (size_t)by * 8 * P.pitch[ci] + bx * 8;
    const int32_t* q = P.qtab + (f * 3 + ci) * 64;
    int32_t c[64];  // dequantised (T.81 F.2.1.4: coefficient x table entry)
    const int4* src = reinterpret_cast<const int4*>(coef + b * 64);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int4 v = src[i];
        const int32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            c[8 * i + 2 * j] = (int32_t)(int16_t)(w[j] & 0xffff) * q[8 * i + 2 * j];
            c[8 * i + 2 * j + 1] = (int32_t)(int16_t)((uint32_t)w[j] >> 16) * q[8 * i + 2 * j + 1];
        }
    }
    bool ac0 = true;
#pragma unroll
    for (int i = 1; i < 64; i++) ac0 = ac0 && c[i] == 0;
    if (ac0) {  // zune: DC-only block, (DC >> 3) + 128 without rounding
        const uint8_t v = clamp_u8(((int64_t)c[0] >> 3) + 128);
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++) out[(size_t)y * P.pitch[ci] + x] = v;
        return;
    }
    int64_t ws[8][8];  // [column u][row y]
#pragma unroll
    for (int u = 0; u < 8; u++) {
        bool col0 = true;
#pragma unroll
        for (int v = 1; v < 8; v++) col0 = col0 && c[v * 8 + u] == 0;
        if (col0) {
#pragma unroll
            for (int y = 0; y < 8; y++) ws[u][y] = (int64_t)c[u] * 4;
            continue;
        }
        Idct1 o = idct1d(c[u], c[8 + u], c[16 + u], c[24 + u], c[32 + u], c[40 + u], c[48 + u], c[56 + u]);
        o.x0 += 512;
        o.x1 += 512;
        o.x2 += 512;
        o.x3 += 512;
        ws[u][0] = (o.x0 + o.t3) >> 10;
        ws[u][7] = (o.x0 - o.t3) >> 10;
        ws[u][1] = (o.x1 + o.t2) >> 10;
        ws[u][6] = (o.x1 - o.t2) >> 10;
        ws[u][2] = (o.x2 + o.t1) >> 10;
        ws[u][5] = (o.x2 - o.t1) >> 10;
        ws[u][3] = (o.x3 + o.t0) >> 10;
        ws[u][4] = (o.x3 - o.t0) >> 10;
    }
#pragma unroll
    for (int y = 0; y < 8; y++) {
        Idct1 o = idct1d(ws[0][y], ws[1][y], ws[2][y], ws[3][y], ws[4][y], ws[5][y], ws[6][y], ws[7][y]);
        o.x0 += kRowBias;
        o.x1 += kRowBias;
        o.x2 += kRowBias;
        o.x3 += kRowBias;
        uint8_t* r = out + (size_t)y * P.pitch[ci];
        r[0] = clamp_u8((o.x0 + o.t3) >> 17);
        r[7] = clamp_u8((o.x0 - o.t3) >> 17);
        r[1] = clamp_u8((o.x1 + o.t2) >> 17);
        r[6] = clamp_u8((o.x1 - o.t2) >> 17);
        r[2] = clamp_u8((o.x2 + o.t1) >> 17);
        r[5] = clamp_u8((o.x2 - o.t1) >> 17);
        r[3] = clamp_u8((o.x3 + o.t0) >> 17);
        r[4] = clamp_u8((o.x3 - o.t0) >> 17);
    }
}

struct LumaArgs {
    Planes P;
    int w, h;
    int fh[3], fv[3];  // upsampling factors hmax / h_c, vmax / v_c (1 or 2)
    int ph[3], pw[3];  // padded plane size (rows, columns)
    uint8_t* out;  // frame f at out + f * out_pitch
    size_t out_stride, out_pitch;
};

// full-resolution sample (y, x) of component ci: two-pass 3:1 triangle
// upsampling ((3a + b + 2) >> 2, vertical then horizontal, neighbours
// clamped to the padded plane)
__device__ __forceinline__ int sample(const LumaArgs& A, int ci, int y, int x, size_t fo) {
    const uint8_t* p = A.P.p[ci] + fo;
    const int pitch = A.P.pitch[ci];
    if (A.fv[ci] == 1 && A.fh[ci] == 1) return p[(size_t)y * pitch + x];
    auto vrow = [&](int c) -> int {  // vertical pass at plane column c for output row y
        if (A.fv[ci] == 1) return p[(size_t)y * pitch + c];
        const int r = y >> 1;
        const int rn = (y & 1) ? min(r + 1, A.ph[ci] - 1) : max(r - 1, 0);
        return (3 * (int)p[(size_t)r * pitch + c] + (int)p[(size_t)rn * pitch + c] + 2) >> 2;
    };
    if (A.fh[ci] == 1) return vrow(x);
    const int c = x >> 1;
    const int cn = (x & 1) ? min(c + 1, A.pw[ci] - 1) : max(c - 1, 0);
    return (3 * vrow(c) + vrow(cn) + 2) >> 2;
}

__global__ __launch_bounds__(256) void k_jpeg_luma(const LumaArgs A) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= A.w || y >= A.h) return;
    const size_t fo = (size_t)blockIdx.z * A.P.frame_bytes;  // frame blockIdx.z
    uint8_t v;
    if (A.P.nc == 1) {
        v = A.P.p[0][fo + (size_t)y * A.P.pitch[0] + x];
    } else {
        const int yy = sample(A, 0, y, x, fo), cb = sample(A, 1, y, x, fo) - 128, cr = sample(A, 2, y, x, fo) - 128;
        // zune-jpeg's 6-bit fixed-point YCbCr -> RGB (arithmetic shifts)
        const int r = min(max(yy + ((45 * cr) >> 5), 0), 255);
        const int g = min(max(yy - ((11 * cb + 23 * cr) >> 5), 0), 255);
        const int b = min(max(yy + ((113 * cb) >> 6), 0), 255);
        // image 0.25 grayscale(): (2126 R + 7152 G + 722 B) / 10000
        v = (uint8_t)min((2126 * r + 7152 * g + 722 * b) / 10000, 255);
    }
    A.out[(size_t)blockIdx.z * A.out_pitch + (size_t)y * A.out_stride + x] = v;
}

}  // namespace jpg

int jpeg_dims(const uint8_t* data, size_t len, uint32_t* w, uint32_t* h, std::string& err) {
    jpg::Header H;
    const int rc = jpg::parse(data, len, H, err);
    if (rc) return rc;
    if (w) *w = (uint32_t)H.w;
    if (h) *h = (uint32_t)H.h;
    return 0;
}

namespace jpg {
// device views of n frames' coefficients / planes / output for one geometry
void views(const Header& H, const Geom& g, uint8_t* d_planes, uint8_t* out, size_t out_stride, size_t out_pitch,
           Planes& P, LumaArgs& A) {
    P = Planes{};
    P.nc = H.nc;
    size_t po = 0;
    for (int k = 0; k < H.nc; k++) {
        P.p[k] = d_planes + po;
        P.pitch[k] = g.bw[k] * 8;
        P.bw[k] = g.bw[k];
        P.off[k] = g.off[k];
        po += (size_t)g.bw[k] * g.bh[k] * 64;
    }
    P.frame_blocks = g.total;
    P.frame_bytes = po;
    A = LumaArgs{};
    A.P = P;
    A.w = H.w;
    A.h = H.h;
    for (int k = 0; k < H.nc; k++) {
        A.fh[k] = g.hmax / H.c[k].h;
        A.fv[k] = g.vmax / H.c[k].v;
        A.ph[k] = g.bh[k] * 8;
        A.pw[k] = g.bw[k] * 8;
    }
    A.out = out;
    A.out_stride = out_stride;
    A.out_pitch = out_pitch;
}

void qtables(const Header& H, int32_t* q) {  // 3 x 64, components' order
    for (int k = 0; k < H.nc; k++) std::memcpy(q + 64 * k, H.q[H.c[k].tq], 64 * sizeof(int32_t));
}

int check_support(const Header& H, const Geom& g, std::string& err) {
    for (int k = 0; k < H.nc; k++)  // h2v1, h2v2 and full-size chroma (the restatement's cases)
        if (H.nc == 3 && g.hmax / H.c[k].h == 1 && g.vmax / H.c[k].v == 2)
            return err = "JPEG: vertical-only chroma subsampling", SIFT_MI_EUNSUPPORTED;
    return 0;
}

void launch(const int16_t* d_coef, uint32_t n, const Geom& g, const Header& H, const Planes& P, const LumaArgs& A,
            hipStream_t st) {
    const size_t nblk = g.total * n;
    hipLaunchKernelGGL(k_jpeg_idct, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, st, d_coef, nblk, P);
    hipLaunchKernelGGL(k_jpeg_luma, dim3((H.w + 63) / 64, (H.h + 3) / 4, n), dim3(256), 0, st, A);
}
}  // namespace jpg

int jpeg_decode_luma(const uint8_t* data, size_t len, uint8_t* out, size_t out_stride, bool out_on_device,
                     hipStream_t st, std::string& err) {
    jpg::Header H;
    int rc = jpg::parse(data, len, H, err);
    if (rc) return rc;
    const jpg::Geom g = jpg::geometry(H);
    if ((rc = jpg::check_support(H, g, err))) return rc;
    std::vector<int16_t> coef(g.total * 64);
    rc = jpg::entropy_decode(data, len, H, g, coef.data(), err);
    if (rc) return rc;
    const size_t coef_bytes = coef.size() * sizeof(int16_t);
    jpg::Planes P;
    jpg::LumaArgs A;
    jpg::views(H, g, nullptr, nullptr, 0, 0, P, A);
    const size_t plane_bytes = P.frame_bytes;
    const size_t out_bytes = out_on_device ? 0 : (size_t)H.w * H.h;
    const size_t q_bytes = 3 * 64 * sizeof(int32_t);
    std::vector<int32_t> qt(3 * 64, 0);
    jpg::qtables(H, qt.data());
    // one device allocation: quantisation tables, coefficients, padded planes, (host output staging)
    uint8_t* dev = nullptr;
    if (hipMallocAsync((void**)&dev, q_bytes + coef_bytes + plane_bytes + out_bytes + 64, st) != hipSuccess)
        return err = "JPEG: device allocation failed", SIFT_MI_ENOMEM;
    uint8_t* d_cf = dev + q_bytes;
    uint8_t* d_pl = d_cf + coef_bytes;
    uint8_t* d_out = out_on_device ? out : d_pl + plane_bytes;
    jpg::views(H, g, d_pl, d_out, out_on_device ? out_stride : (size_t)H.w, 0, P, A);
    P.qtab = A.P.qtab = reinterpret_cast<const int32_t*>(dev);
    bool ok = hipMemcpyAsync(dev, qt.data(), q_bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemcpyAsync(d_cf, coef.data(), coef_bytes, hipMemcpyHostToDevice, st) == hipSuccess;
    if (ok) {
        jpg::launch(reinterpret_cast<int16_t*>(d_cf), 1, g, H, P, A, st);
        ok = hipGetLastError() == hipSuccess;
    }
    if (ok && !out_on_device)
        ok = hipMemcpy2DAsync(out, out_stride, d_out, (size_t)H.w, (size_t)H.w, (size_t)H.h, hipMemcpyDeviceToHost,
                              st) == hipSuccess;
    ok = (hipFreeAsync(dev, st) == hipSuccess) && ok;
    // the coefficient upload reads pageable host memory that is freed on return
    ok = (hipStreamSynchronize(st) == hipSuccess) && ok;
    if (!ok) return err = "JPEG: HIP error", SIFT_MI_EHIP;
    return 0;
}

// n equal-geometry JPEGs -> device luma frames (frame i at d_out + i *
// frame_pitch).  Entropy decoding of a chunk of frames runs on `threads` host
// threads into pinned buffers (two, alternating) while the previous chunk's
// upload and reconstruction kernels run on the stream.
void JpegBatchCache::release() {
    for (int k = 0; k < 2; k++) {
        if (pin[k]) (void)hipHostFree(pin[k]);
        if (up[k]) (void)hipEventDestroy(up[k]);
        pin[k] = nullptr;
        up[k] = nullptr;
    }
    if (dev) (void)hipFree(dev);
    dev = nullptr;
    pin_bytes = dev_bytes = 0;
}

// Host threads entropy-decode frames in order (work stealing over the whole
// batch) into two pinned chunk buffers; the calling thread uploads each chunk
// as soon as its frames are in and launches the chunk's reconstruction, so
// decoding chunk k + 1 overlaps the upload and kernels of chunk k.  A buffer
// is handed back to the workers when its upload has completed.
int jpeg_decode_batch(const uint8_t* const* data, const size_t* len, uint32_t n, uint8_t* d_out,
                      size_t frame_pitch, size_t stride, int threads, hipStream_t st, JpegBatchCache& cache,
                      std::string& err) {
    if (n == 0) return 0;
    jpg::Header H0;
    int rc = jpg::parse(data[0], len[0], H0, err);
    if (rc) return rc;
    const jpg::Geom g = jpg::geometry(H0);
    if ((rc = jpg::check_support(H0, g, err))) return rc;
    if (stride < (size_t)H0.w || frame_pitch < stride * H0.h) return err = "JPEG batch: output too small", SIFT_MI_EINVAL;
    std::vector<jpg::Header> hdr(n);
    hdr[0] = H0;
    for (uint32_t i = 1; i < n; i++) {
        if ((rc = jpg::parse(data[i], len[i], hdr[i], err))) return rc;
        const jpg::Header& h = hdr[i];
        bool same = h.w == H0.w && h.h == H0.h && h.nc == H0.nc;
        for (int k = 0; same && k < h.nc; k++) same = h.c[k].h == H0.c[k].h && h.c[k].v == H0.c[k].v;
        if (!same) return err = "JPEG batch: frames differ in size or sampling", SIFT_MI_EINVAL;
    }
    const uint32_t C = std::min<uint32_t>(n, 16);  // frames per chunk
    const uint32_t n_chunks = (n + C - 1) / C;
    const size_t fcoef = g.total * 64;              // int16 per frame
    jpg::Planes P;
    jpg::LumaArgs A;
    jpg::views(H0, g, nullptr, nullptr, 0, 0, P, A);
    const size_t fplane = P.frame_bytes;
    const size_t q_bytes = ((size_t)n * 3 * 64 * sizeof(int32_t) + 255) & ~(size_t)255;
    const size_t pin_bytes = C * fcoef * sizeof(int16_t);
    const size_t dev_bytes = q_bytes + 2 * C * fcoef * sizeof(int16_t) + C * fplane;
    // buffers: grow-only, kept by the context (the previous call has drained:
    // every call synchronises its stream before returning)
    if (cache.pin_bytes < pin_bytes) {
        for (int k = 0; k < 2; k++) {
            if (cache.pin[k]) (void)hipHostFree(cache.pin[k]);
            cache.pin[k] = nullptr;
        }
        cache.pin_bytes = 0;
        for (int k = 0; k < 2; k++)
            if (hipHostMalloc((void**)&cache.pin[k], pin_bytes, hipHostMallocDefault) != hipSuccess) {
                cache.release();
                return err = "JPEG batch: allocation failed", SIFT_MI_ENOMEM;
            }
        cache.pin_bytes = pin_bytes;
    }
    for (int k = 0; k < 2; k++)
        if (!cache.up[k] && hipEventCreateWithFlags(&cache.up[k], hipEventDisableTiming) != hipSuccess) {
            cache.release();
            return err = "JPEG batch: HIP error", SIFT_MI_EHIP;
        }
    if (cache.dev_bytes < dev_bytes) {
        if (cache.dev) (void)hipFree(cache.dev);
        cache.dev = nullptr;
        cache.dev_bytes = 0;
        if (hipMalloc((void**)&cache.dev, dev_bytes) != hipSuccess) {
            cache.release();
            return err = "JPEG batch: allocation failed", SIFT_MI_ENOMEM;
        }
        cache.dev_bytes = dev_bytes;
    }
    int16_t* const* pin = cache.pin;
    uint8_t* dev = cache.dev;
    // every frame's quantisation tables (frames may differ in quality)
    std::vector<int32_t> qt((size_t)n * 3 * 64, 0);
    for (uint32_t i = 0; i < n; i++) jpg::qtables(hdr[i], qt.data() + (size_t)i * 192);
    const int32_t* d_q = reinterpret_cast<const int32_t*>(dev);
    if (hipMemcpyAsync(dev, qt.data(), qt.size() * sizeof(int32_t), hipMemcpyHostToDevice, st) != hipSuccess)
        return err = "JPEG batch: HIP error", SIFT_MI_EHIP;
    uint8_t* d_cf = dev + q_bytes;
    uint8_t* d_pl = d_cf + 2 * C * fcoef * sizeof(int16_t);

    // worker pool over the whole batch
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint32_t> done(n_chunks, 0);
    uint32_t free_upto = 2;  // chunks below this may be decoded (their buffer is free)
    bool stop = false;
    int trc = 0;
    std::string terr;
    std::atomic<uint32_t> next{0};
    auto work = [&]() {
        std::string e;
        for (uint32_t i; (i = next.fetch_add(1)) < n;) {
            const uint32_t ch = i / C;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return ch < free_upto || stop; });
                if (stop) return;
            }
            const int r = jpg::entropy_decode(data[i], len[i], hdr[i], g, pin[ch & 1] + (size_t)(i - ch * C) * fcoef, e);
            {
                std::lock_guard<std::mutex> lk(mu);
                if (r && !trc) trc = r, terr = e, stop = true;
                done[ch]++;
            }
            cv.notify_all();
            if (r) return;
        }
    };
    const int T = std::max(1, std::min<int>(threads, (int)n));
    std::vector<std::thread> pool;
    pool.reserve(T);
    for (int t = 0; t < T; t++) pool.emplace_back(work);
    bool ok = true;
    for (uint32_t ch = 0; ch < n_chunks && ok; ch++) {
        const uint32_t c0 = ch * C, m = std::min(C, n - c0), k = ch & 1;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return done[ch] == m || stop; });
            if (stop) break;
        }
        int16_t* d_coef = reinterpret_cast<int16_t*>(d_cf) + k * C * fcoef;
        jpg::views(H0, g, d_pl, d_out + (size_t)c0 * frame_pitch, stride, frame_pitch, P, A);
        P.qtab = A.P.qtab = d_q + (size_t)c0 * 192;
        ok = hipMemcpyAsync(d_coef, pin[k], m * fcoef * sizeof(int16_t), hipMemcpyHostToDevice, st) == hipSuccess &&
             hipEventRecord(cache.up[k], st) == hipSuccess;
        if (ok) {
            jpg::launch(d_coef, m, g, H0, P, A, st);
            ok = hipGetLastError() == hipSuccess;
        }
        // pinned buffer k is free for chunk ch + 2 once this upload is done
        ok = ok && host_wait_event(cache.up[k]) == hipSuccess;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (ok)
                free_upto = ch + 3;
            else
                stop = true;
        }
        cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        stop = stop || !ok;
    }
    cv.notify_all();
    for (auto& th : pool) th.join();
    const bool synced = hipStreamSynchronize(st) == hipSuccess;
    if (trc) return err = terr, trc;
    if (!ok || !synced) return err = "JPEG batch: HIP error", SIFT_MI_EHIP;
    return 0;
}

}  // namespace siftmi
