// Fused octave kernel: the five incremental blurs of one octave and its DoG in
// one streaming pass (OpenCV profile).
//
// EXPERIMENT RECORD (not built into libsift_mi.so): measured slower than the
// per-blur kernels and superseded by the strip blur kernels
// (pyramid.hip k_blur_strip).  Kept with its harnesses (oct_stamps.hip,
// oct_trace.sh) for the measurements DESIGN.md cites.
//
// Reference: build_gaussian_scale_space / build_dog (src/lib.rs:213-279) with
// OpenCVProcessing::gaussian_blur (src/opencv_processing.rs:38-49):
// G_s = blur(G_{s-1}, sigma_s), s = 1..5, D_{s-1} = G_s - G_{s-1}, and the next
// octave's base = nearest 1/2 of G_3 (src/lib.rs:245-247).
//
// Why: the per-blur kernel (pyramid.hip k_blur) must re-read G_{s-1} from HBM
// for every blur: 12 B per blur per octave pixel, 60 B per octave pixel in
// all.  Here a workgroup owns a vertical strip of TW output columns and a
// segment of rows and streams down it, B rows per step, carrying all five
// blur levels at once: level s consumes the G_{s-1} rows level s-1 produced
// one step earlier (through a double-buffered LDS stage), so only G_0 is read
// and G_1..G_4 (+ G_5 when materialised), D_0..D_4 and the next base are
// written: 4 + 36 (40) B per octave pixel plus the halo re-reads of G_0.
//
// Layout of the work (704 threads = 11 waves: 2 per level + 1 loader):
//  * level s computes its output on the strip's TW columns plus a halo of
//    hp(s) columns each side (what the later levels' row filters need), one
//    column PAIR per lane (packed f32 arithmetic);
//  * row filter (OpenCV RowFilter: fma chain from the leftmost tap) reads the
//    lane's 2R+2 input floats of each new row from LDS (ds_read_b64);
//  * column filter (SymmColumnFilter: centre product, fma of (below + above)
//    pair sums outwards) runs on a register window of the last 2R+B
//    row-filtered rows, B outputs per step, then the window shifts by B;
//  * D_{s-1} needs G_{s-1} at the output rows, R rows behind the input: a
//    per-lane LDS ring of R+B centre values;
//  * the loader wave streams G_0 rows into level 1's (triple-buffered) stage
//    by LDS-DMA, one step ahead.  It is the only wave that waits on global
//    loads: the level waves only store, and the per-step
//    barrier is a raw s_barrier after lgkmcnt(0), so their stores drain while
//    the next step runs.  (With the loads in the level waves, each step's
//    wait for its loads also waited for every store issued after them -- the
//    VM counter retires in order -- and the strip stalled on HBM write
//    latency once per step.)
// Borders (BORDER_REFLECT_101): rows are streamed through the reflection
// (level 1 loads G_0 rows reflect101(y); a symmetric kernel applied to a
// reflect-101-symmetric signal gives a symmetric result bit for bit, since
// the column filter adds mirrored pairs -- a + b == b + a -- so rows outside
// the image carry exactly the reflected rows of every level).  The row filter
// is an ordered chain, so columns outside the image are not computed but
// copied: each in-image output is also written to its mirror positions in the
// next level's stage row (one reflection: needs W > hp(1) + 1).
// Bit-identical to k_blur (same operations in the same order), checked by
// tests/test_gpu_parity.py against the C oracle.
#include "../../sift-features_amd/csrc/sift_common.h"
#include "../../sift-features_amd/csrc/sift_kernels.h"

namespace siftmi {

// launch arguments (formerly in sift_kernels.h)
struct OctaveArgs {
    float* gauss;  // octave G stack of image 0 (plane s at + s * plane)
    size_t g_img_stride, plane;
    float* dog;  // octave D stack of image 0
    size_t dog_img_stride;
    float* nxt;  // next octave base (nearest 1/2 of G_3), may be null
    size_t nxt_img_stride;
    int pitch_n, wn, hn;
    int W, H, pitch;
    int seg_rows;  // rows per workgroup segment
    int write_all;  // materialise G_4 and G_5 too (precompute_images); the batch path keeps them on chip
    BlurTaps taps[6];  // taps[s] for s = 1..5
};

namespace oct {

constexpr int kL = 5;                                  // blurs per octave (s = 1..5)
constexpr int kR[kL + 1] = {0, 5, 6, 8, 10, 13};      // OpenCV radii of sigma_1..5 (cvRound(8 sigma + 1) | 1 taps)
constexpr int sum_r(int a, int b) { return a > b ? 0 : kR[a] + sum_r(a + 1, b); }
constexpr int kV0 = sum_r(1, kL);                      // vertical halo of the whole chain (rows)
// column halo of level s's output (even, so every lane's pair is column-aligned)
constexpr int hp(int s) { return s >= kL ? 0 : ((hp(s + 1) + kR[s + 1] + 1) & ~1); }
constexpr int kWavesPerLevel = 2;
constexpr int kPairs = 64 * kWavesPerLevel;            // lanes per level
// owned columns per strip: a multiple of 32 floats (128-B lines), so with
// strip-aligned x0 every row of every plane is stored as whole lines (partial
// lines shared by two strips cost the write path dearly); level 1's width
// (kTW + 2 hp(1)) must fit its 2 x 64 lanes
constexpr int kTW = (2 * (kPairs - hp(1))) / 32 * 32;
constexpr int kLoaderWave = kWavesPerLevel * kL;       // the last wave streams G_0 rows into LDS
constexpr int kThreads = 64 * (kLoaderWave + 1);
constexpr int width(int s) { return kTW + 2 * hp(s); }  // level s output columns; s = 0: level 1 input
constexpr int dH(int s) { return hp(s - 1) - hp(s); }
constexpr int pad(int s) { return (dH(s) - kR[s]) & 1; }  // makes each lane's row window 8-B aligned
constexpr int pitch(int s) { return (width(s - 1) + pad(s) + 1) & ~1; }
static_assert(kTW > 0 && kTW % 32 == 0 && kTW + 2 * hp(1) <= 2 * kPairs, "strip width");
static_assert(width(0) % 2 == 0 && width(0) / 2 >= 64, "loader: a 64-lane load spans at most two rows");
static_assert(dH(1) >= kR[1] && dH(2) >= kR[2] && dH(3) >= kR[3] && dH(4) >= kR[4] && dH(5) >= kR[5], "halos");

// level processed by wave w (0 = the loader).  A workgroup's waves land on
// the SIMDs cyclically, so waves w, w + 4, w + 8 share one; per step (VALU
// instructions ~ taps): {L1, L2, L4}, {L1, L2, L3}, {L5, L3, loader}, {L5, L4}
__device__ __forceinline__ int level_of_wave(int w) {
    constexpr int lv[2 * kL + 1] = {1, 1, 5, 5, 2, 2, 3, 4, 4, 3, 0};
    return lv[w];
}

template <int B>
struct Plan {
    static constexpr int stage_floats(int s) { return (s == 1 ? 3 : 2) * B * pitch(s); }  // stage_1: loader ring
    static constexpr int stage_off(int s) { return s <= 1 ? 0 : stage_off(s - 1) + stage_floats(s - 1); }
    // centre rings: G_{s-1} at the strip's owned columns, R_s + B rows (the
    // DoG's subtrahend, R_s rows behind level s's input)
    static constexpr int ring_rows(int s) { return kR[s] + B; }
    static constexpr int ring_off(int s) { return s <= 1 ? stage_off(kL + 1) : ring_off(s - 1) + ring_rows(s - 1) * kTW; }
    static constexpr int kLds = ring_off(kL + 1);  // stage_1 .. stage_5 + rings
};

typedef __attribute__((address_space(3))) volatile f2v lds_f2v;

// Diagnostic build only (-DSIFT_OCT_STAMPS, tools/exp/oct_stamps.hip): per
// wave role, the cycles of each step phase summed over the run (read shares,
// not lengths: the stamps' waits forbid overlaps the real kernel has).
#ifdef SIFT_OCT_STAMPS
__device__ unsigned long long g_oct_stamps[kL + 1][5];
#define OCT_STAMP(v)                                                                     \
    do {                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                               \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");      \
        __builtin_amdgcn_sched_barrier(0);                                               \
    } while (0)
#define OCT_STAMP_DECL unsigned long long st_t0 = 0, st_t1 = 0, st_acc[4] = {0, 0, 0, 0}
#define OCT_STAMP_ADD(i) st_acc[i] += st_t1 - st_t0, st_t0 = st_t1
#define OCT_STAMP_FLUSH(lvl)                                                            \
    do {                                                                                 \
        if ((threadIdx.x & 63) == 0) {                                                   \
            for (int q = 0; q < 4; q++) atomicAdd(&g_oct_stamps[lvl][q], st_acc[q]);      \
            atomicAdd(&g_oct_stamps[lvl][4], 1ull);                                      \
        }                                                                                \
    } while (0)
#else
#define OCT_STAMP(v) \
    do {             \
    } while (0)
#define OCT_STAMP_DECL
#define OCT_STAMP_ADD(i)
#define OCT_STAMP_FLUSH(lvl)
#endif

// Step barrier: this wave's LDS writes complete, then s_barrier.  gfx950's
// barrier waits for no memory by itself, and the "memory" clobber keeps the
// compiler's LDS accesses on their side of it.
__device__ __forceinline__ void step_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// reflect-101 index without a loop (E(-p) = E(p), period 2 (len - 1))
__device__ __forceinline__ int refl(int p, int len) {
    if (len == 1) return 0;
    const int per = 2 * (len - 1);
    p = abs(p) % per;
    return p >= len ? per - p : p;
}

// s_waitcnt vmcnt(n) alone (expcnt / lgkmcnt left at their maxima), gfx9 encoding
constexpr int vmcnt_only(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

// The loader wave streams the G_0 rows of step t + 2 straight into LDS
// (global_load_lds_dword: lane i of a 64-float chunk lands at chunk base + i;
// columns reflected per lane at the strip borders) while level 1 filters
// step t's: stage_1 is triple-buffered.  At each step it first waits for step
// t + 1's transfers (issued a whole step earlier), then issues step t + 2's,
// then takes the step barrier -- the wait-then-barrier order publishes the
// landed rows to the level waves.  No registers hold the rows, and this wave
// issues no other VM operation, so its counter counts exactly these.
template <int B>
__device__ __forceinline__ void run_loader(const OctaveArgs& a, float* __restrict__ lds, int x0, int y0, size_t img,
                                           int nsteps, bool interior) {
    constexpr int P1 = pitch(1), PAD1 = pad(1), W0 = width(0), HP0 = hp(0);
    constexpr int CH = (W0 + 63) / 64;  // 64-float chunks per row
    constexpr int TAIL = W0 - 64 * (CH - 1);
    const int lane = threadIdx.x & 63;
    const float* __restrict__ g0 = a.gauss + img * a.g_img_stride;
    const int W = a.W, H = a.H, pg = a.pitch;
    float* const st = lds + Plan<B>::stage_off(1) + PAD1;
    // this lane's column in each chunk (step-invariant)
    int col[CH];
#pragma unroll
    for (int m = 0; m < CH; m++) {
        const int c = x0 - HP0 + 64 * m + (m == CH - 1 ? min(lane, TAIL - 1) : lane);
        col[m] = interior ? c : refl(c, W);
    }
    auto issue = [&](int step, int buf) {
        const int roff = refl(y0 - kV0 + step * B + min(lane, B - 1), H) * pg;  // lane b: row b of the step
        float* const dst = st + buf * B * P1;
#pragma unroll
        for (int b = 0; b < B; b++) {
            const float* row = g0 + __builtin_amdgcn_readlane(roff, b);
#pragma unroll
            for (int m = 0; m < CH; m++) {
                if (m < CH - 1 || lane < TAIL)
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(row + col[m]),
                                                     (__attribute__((address_space(3))) void*)(dst + b * P1 + 64 * m),
                                                     4, 0, 0);
            }
        }
    };
    issue(0, 0);
    __builtin_amdgcn_s_waitcnt(vmcnt_only(0));
    issue(1, 1);
    step_barrier();  // step 0's rows are staged
    int buf = 2;     // stage_1 buffer of step t + 2
    OCT_STAMP_DECL;
    OCT_STAMP(st_t0);
    for (int t = 0; t < nsteps; t++) {
        __builtin_amdgcn_s_waitcnt(vmcnt_only(0));  // step t + 1's rows landed
        OCT_STAMP(st_t1);
        OCT_STAMP_ADD(0);
        issue(t + 2, buf);
        buf = buf == 2 ? 0 : buf + 1;
        OCT_STAMP(st_t1);
        OCT_STAMP_ADD(1);
        step_barrier();
        OCT_STAMP(st_t1);
        OCT_STAMP_ADD(3);
    }
    // no transfer may land in LDS after the workgroup has released it
    __builtin_amdgcn_s_waitcnt(vmcnt_only(0));
    OCT_STAMP_FLUSH(0);
}

template <int S, int B>
__device__ __forceinline__ void run_level(const OctaveArgs& a, float* __restrict__ lds, int x0, int y0, int y1,
                                          size_t img, int nsteps, int p) {
    constexpr int R = kR[S];
    constexpr int HPS = hp(S), WS = width(S), DHS = dH(S), PADS = pad(S), PS = pitch(S);
    constexpr int PADN = S < kL ? pad(S + 1) : 0, PN = S < kL ? pitch(S + 1) : 0;
    constexpr int OFF_IN = Plan<B>::stage_off(S), OFF_OUT = Plan<B>::stage_off(S + 1);
    constexpr int SUMR = sum_r(1, S - 1);
    constexpr int NP = WS / 2;  // pairs of this level
    constexpr int RING = Plan<B>::ring_rows(S);
    constexpr int RING_OFF = Plan<B>::ring_off(S);
    static_assert(B % 2 == 0, "rows are filtered two at a time");
    // lane -> pair, rotated so that the first wave of the level holds the
    // strip's first 64 owned pairs (its stores are whole 512-B row segments)
    const int pr = (p + HPS / 2) & (kPairs - 1);
    const bool active = pr < NP;
    const int pp = active ? pr : NP - 1;
    // G_4 and G_5 only when every Gaussian is materialised (precompute_images):
    // downstream stages read G_1..G_3, and the chain keeps G_4 on chip
    float* __restrict__ gS = (S < 4 || a.write_all) ? a.gauss + img * a.g_img_stride + (size_t)S * a.plane : nullptr;
    float* __restrict__ dS = a.dog + img * a.dog_img_stride + (size_t)(S - 1) * a.plane;
    float* __restrict__ nxt = (S == 3 && a.nxt) ? a.nxt + img * a.nxt_img_stride : nullptr;
    const int W = a.W, pg = a.pitch;
    const int xc = x0 - HPS + 2 * pp;  // image column of the lane's pair
    const bool owned = active && xc >= x0 && xc < x0 + kTW && xc < W;
    const bool pair2 = xc + 1 < W;
    const bool odd_edge = (W & 1) && x0 + kTW >= W;  // (uniform) the strip holds a lone last column
    // a strip whose level-S columns all lie inside the image writes its stage
    // pairs unconditionally; border strips write in-image elements and their
    // reflect-101 mirrors (one reflection)
    const bool border = x0 - HPS < 0 || x0 + kTW + HPS > W;
    int m0 = -1, m1 = -1, n0 = -1, n1 = -1;  // mirror positions of element 0 / 1 (left, right reflection)
    bool in0 = false, in1 = false;
    if constexpr (S < kL) {
        const int base = x0 - HPS;
        if (active) {
            in0 = xc >= 0 && xc < W;
            in1 = xc + 1 >= 0 && xc + 1 < W;
            auto mir = [&](int xe, int& ml, int& mr) {
                if (xe < 0 || xe >= W) return;
                if (xe >= 1) {
                    const int l = -xe - base;
                    if (l >= 0 && l < WS) ml = l;
                }
                if (xe < W - 1) {
                    const int l = 2 * (W - 1) - xe - base;
                    if (l >= 0 && l < WS) mr = l;
                }
            };
            mir(xc, m0, n0);
            mir(xc + 1, m1, n1);
        }
    }
    const float* kt = a.taps[S].k;
    f2v win[2 * R + B];
#pragma unroll
    for (int i = 0; i < 2 * R + B; i++) win[i] = f2v{0.f, 0.f};
    // owned lanes: pairs [HPS / 2, HPS / 2 + kTW / 2)
    float* const ring = lds + RING_OFF + 2 * min(max(pp - HPS / 2, 0), kTW / 2 - 1);
    const bool own_lane = active && pp >= HPS / 2 && pp < HPS / 2 + kTW / 2;
    int wslot = 0;  // ring slot of this step's first input row
    int ibuf = 0;   // input stage buffer of this step: t % 3 for level 1 (the loader's ring), t & 1 otherwise
    const int r1_0 = y0 - kV0;  // first G_0 row fed to level 1
    // the previous step's output rows, stored during this step
    f2v pout[B], pdog[B];
#pragma unroll
    for (int j = 0; j < B; j++) pout[j] = pdog[j] = f2v{0.f, 0.f};
    int prow0 = INT_MIN / 2;
    auto put = [&](int row, f2v g, f2v dv) {
        if (owned && row >= y0 && row < y1) {
            const size_t off = (size_t)row * pg + xc;
            if (!odd_edge || pair2) {
                if (gS) *reinterpret_cast<f2v*>(gS + off) = g;
                *reinterpret_cast<f2v*>(dS + off) = dv;
            } else {
                if (gS) gS[off] = g.x;
                dS[off] = dv.x;
            }
            if constexpr (S == 3) {
                if (nxt && (row & 1) == 0 && (row >> 1) < a.hn && (xc >> 1) < a.wn)
                    nxt[(size_t)(row >> 1) * a.pitch_n + (xc >> 1)] = g.x;
            }
        }
    };
    step_barrier();  // the loader has staged step 0's rows
    OCT_STAMP_DECL;
    OCT_STAMP(st_t0);
    for (int t = 0; t < nsteps; t++) {
        // row filter of this step's B input rows (written by level S-1 / the
        // loader at step t-1), two rows at a time: two independent fma chains
        const float* in = lds + OFF_IN + ibuf * B * PS + PADS + 2 * pp + DHS - R;
#pragma unroll
        for (int b = 0; b < B; b += 2) {
            put(prow0 + b, pout[b], pdog[b]);
            put(prow0 + b + 1, pout[b + 1], pdog[b + 1]);
            const lds_f2v* rp0 = (const lds_f2v*)(in + b * PS);
            const lds_f2v* rp1 = (const lds_f2v*)(in + (b + 1) * PS);
            f2v w0[R + 1], w1[R + 1];
#pragma unroll
            for (int k = 0; k <= R; k++) w0[k] = rp0[k];
#pragma unroll
            for (int k = 0; k <= R; k++) w1[k] = rp1[k];
            // floats (v[i], v[i + 1]) of a lane's window
#define PR(w, i) (((i) & 1) ? f2v{w[(i) >> 1].y, w[((i) >> 1) + 1].x} : w[(i) >> 1])
            const f2v kc = {kt[R], kt[R]};
            f2v acc0 = PR(w0, 0) * kc, acc1 = PR(w1, 0) * kc;
#pragma unroll
            for (int tt = 1; tt <= 2 * R; tt++) {
                const float k = kt[tt > R ? tt - R : R - tt];
                acc0 = __builtin_elementwise_fma(PR(w0, tt), f2v{k, k}, acc0);
                acc1 = __builtin_elementwise_fma(PR(w1, tt), f2v{k, k}, acc1);
            }
            asm volatile("" : "+v"(acc0), "+v"(acc1));  // keep the rows' filter here (not sunk into the column pass)
            win[2 * R + b] = acc0;
            win[2 * R + b + 1] = acc1;
            if (own_lane) {
                const int sl = wslot + b < RING ? wslot + b : wslot + b - RING;
                const int sl1 = sl + 1 < RING ? sl + 1 : sl + 1 - RING;
                *(lds_f2v*)(ring + sl * kTW) = PR(w0, R);
                *(lds_f2v*)(ring + sl1 * kTW) = PR(w1, R);
            }
#undef PR
        }
        OCT_STAMP(st_t1);
        OCT_STAMP_ADD(0);
        // column filter: output rows [r_S(t) - R, + B), all B first (independent chains)
        const int orow0 = r1_0 + (t - S + 1) * B - SUMR - R;
        const f2v k0 = {kt[0], kt[0]};
        f2v out[B];
#pragma unroll
        for (int j = 0; j < B; j++) {
            f2v acc = win[R + j] * k0;
#pragma unroll
            for (int tt = 1; tt <= R; tt++) {
                const f2v k = {kt[tt], kt[tt]};
                acc = __builtin_elementwise_fma(win[R + j + tt] + win[R + j - tt], k, acc);
            }
            out[j] = acc;
        }
        OCT_STAMP(st_t1);
        OCT_STAMP_ADD(1);
        // DoG of this step's rows (their ring slots are rewritten next step);
        // the G / D stores themselves are issued during the next step's row
        // filter (put below): a burst of them at the end of the step stalled
        // the waves on the CU's write path while the VALU idled
#pragma unroll
        for (int j = 0; j < B; j++) {
            int sl = wslot - R + j;  // in [-R, RING + B - R - 2]
            sl = sl < 0 ? sl + RING : (sl >= RING ? sl - RING : sl);
            pout[j] = out[j];
            pdog[j] = out[j] - *(const lds_f2v*)(ring + sl * kTW);
        }
        prow0 = orow0;
        if constexpr (S < kL) {
            float* o = lds + OFF_OUT + ((t + 1) & 1) * B * PN + PADN;
            if (!border) {
#pragma unroll
                for (int j = 0; j < B; j++) {
                    o[j * PN + 2 * pp] = out[j].x;
                    o[j * PN + 2 * pp + 1] = out[j].y;
                }
            } else {
#pragma unroll
                for (int j = 0; j < B; j++) {
                    float* oj = o + j * PN;
                    if (in0) oj[2 * pp] = out[j].x;
                    if (in1) oj[2 * pp + 1] = out[j].y;
                    if (m0 >= 0) oj[m0] = out[j].x;
                    if (n0 >= 0) oj[n0] = out[j].x;
                    if (m1 >= 0) oj[m1] = out[j].y;
                    if (n1 >= 0) oj[n1] = out[j].y;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 2 * R; i++) win[i] = win[i + B];
        wslot = wslot + B < RING ? wslot + B : wslot + B - RING;
        ibuf = S == 1 ? (ibuf == 2 ? 0 : ibuf + 1) : ibuf ^ 1;
        OCT_STAMP(st_t1);
        OCT_STAMP_ADD(2);
        step_barrier();
        OCT_STAMP(st_t1);
        OCT_STAMP_ADD(3);
    }
#pragma unroll
    for (int j = 0; j < B; j++) put(prow0 + j, pout[j], pdog[j]);
    OCT_STAMP_FLUSH(S);
}

template <int B>
__global__ __launch_bounds__(kThreads) void k_octave(const OctaveArgs a) {
    using Pn = Plan<B>;
    __shared__ __attribute__((aligned(16))) float lds[Pn::kLds];
    const TileId tile = xcd_tile();
    const int x0 = tile.x * kTW, y0 = tile.y * a.seg_rows;
    const int y1 = min(y0 + a.seg_rows, a.H);
    const size_t img = tile.z;
    const int nsteps = kL + (2 * kV0 + (y1 - y0) + B - 1) / B;
    constexpr int HP0 = hp(0), W0 = width(0);  // (constexpr: hp is recursive, keep it out of device code)
    const bool interior = x0 - HP0 >= 0 && x0 - HP0 + W0 <= a.W;
    const int wave = threadIdx.x >> 6;
    const int p = (wave & 1) * 64 + (threadIdx.x & 63);
    switch (level_of_wave(wave)) {
        case 0: run_loader<B>(a, lds, x0, y0, img, nsteps, interior); break;
        case 1: run_level<1, B>(a, lds, x0, y0, y1, img, nsteps, p); break;
        case 2: run_level<2, B>(a, lds, x0, y0, y1, img, nsteps, p); break;
        case 3: run_level<3, B>(a, lds, x0, y0, y1, img, nsteps, p); break;
        case 4: run_level<4, B>(a, lds, x0, y0, y1, img, nsteps, p); break;
        default: run_level<5, B>(a, lds, x0, y0, y1, img, nsteps, p); break;
    }
}

}  // namespace oct

int octave_strip_width() { return oct::kTW; }
int octave_min_width() { return oct::hp(1) + 2; }
bool octave_radii_supported(const int* r) {
    for (int s = 1; s <= oct::kL; s++)
        if (r[s] != oct::kR[s]) return false;
    return true;
}

int launch_octave(const OctaveArgs& a, int n_img, hipStream_t st) {
    constexpr int B = 8;
    if (a.W < octave_min_width() || a.seg_rows < 1) return -1;
    dim3 grid((a.W + oct::kTW - 1) / oct::kTW, (a.H + a.seg_rows - 1) / a.seg_rows, n_img);
    hipLaunchKernelGGL(oct::k_octave<B>, grid, dim3(oct::kThreads), 0, st, a);
    return 0;
}

}  // namespace siftmi
