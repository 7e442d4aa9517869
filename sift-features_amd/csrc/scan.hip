// Extremum scan on MI355X: point_is_local_extremum (src/lib.rs:437-506) over
// the DoG of each octave, formed from the Gaussian planes as it is read
// (k_detect_rows), and the same scan fused with the octave's last blur
// (k_blur_detect).  Candidates go to k_refine (detect.hip) as packed emission
// keys (frame, octave, scale, y, x).
//
// Built with -fno-honor-nans (Makefile): the scan is max / min / compare on
// finite values (blurs of u8 / 255 data; no NaN can arise), and with no NaN
// to quiet v_max / v_min need no canonicalising copies of their operands, so
// a DPP lane shift folds into the max / min that consumes it
// (v_max_f32_dpp).  Blur arithmetic is unchanged by the flag (no
// reassociation or contraction: -ffp-contract=off, explicit fmaf), so G_5 and
// the candidates are bit-identical to the strip blur + k_detect_rows.
// (-mno-amdgpu-ieee was tried: the device library's functions then are not
// inlined -- __ockl_get_group_id becomes a call -- and every buffer access
// turns into a readfirstlane waterfall loop.)
#include <algorithm>
#include <type_traits>

#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {

// ---------------------------------------------------------------------------
// k_detect_rows: point_is_local_extremum (src/lib.rs:437-506) over all three
// scale triples of an octave, with no LDS staging.  A wave owns a strip of 64
// columns (62 outputs: lanes 1..62, the edge lanes are halo) and ML.sh rows;
// it walks down the strip, loading one row of the 5 DoG planes per step (one
// coalesced 256-B load per plane), forming the 3-wide row max / min with DPP
// wave shifts and keeping the last 3 rows in registers.  Every DoG byte is
// read ~1.1x, there are no barriers, and the loads of the next row are in
// flight while a row is tested.  (A 64x16-tile kernel staging the 5 planes
// in LDS ran 1.8x longer: latency-bound, 62% of wave cycles waiting.)
// Extrema are appended as packed emission keys for k_refine.
// ---------------------------------------------------------------------------
constexpr int DR_SH = 32;       // rows per strip (fewer for launches that cannot fill the chip)
constexpr int DR_COLS = 62;     // output columns per wave
constexpr int DR_LCAP = 256;    // per-block LDS candidate list

// Lane shifts with bound_ctrl (lane 0 / 63 read 0: halo lanes, never
// outputs) and no `old` operand, so no register has to be initialised for
// them and the shift folds into the v_max / v_min that reads it.
__device__ __forceinline__ float dpp_from_left(float v) {  // lane i <- lane i - 1 (wave_shr:1)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane i <- lane i + 1 (wave_shl:1)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

// point_is_local_extremum (src/lib.rs:437-506) for scales 1..3 of row y at
// this lane's column, from the DoG rows y - 1 (prv), y (mid) and y + 1 (cur)
// of the five planes.  Bit s - 1 of the result: scale s is a candidate.
// The reference tests val > threshold (= 0, src/lib.rs:460) and val >= the
// max of its 8 neighbours in plane s and of the 9 values in planes s - 1 and
// s + 1 (val < 0: <= the mins).  Here every plane's full 3x3 max / min (the
// centre included) is formed once -- vertical max3 / min3, then the two lane
// neighbours through DPP shifts -- and val >= max(P_{s-1}, P_s, P_{s+1}):
// P_s includes val itself, so val >= P_s is exactly val >= its 8 neighbours.
// (Comparisons only; no NaN can occur, so the order of max / min operands
// does not matter.)
__device__ __forceinline__ uint32_t extremum3(const float (&prv)[kDogPerOctave], const float (&mid)[kDogPerOctave],
                                              const float (&cur)[kDogPerOctave], bool yin) {
    const float threshold = floorf(0.5f * kContrastThreshold / (float)kScalesPerOctave);  // 0
    float pmx[kDogPerOctave], pmn[kDogPerOctave];
#pragma unroll
    for (int p = 0; p < kDogPerOctave; p++) {
        const float vx = fmaxf(fmaxf(prv[p], mid[p]), cur[p]);
        const float vn = fminf(fminf(prv[p], mid[p]), cur[p]);
        // max(x - 1, x) then max of that and its right neighbour's: two
        // v_max_f32_dpp, no shifted copies
        const float tx = fmaxf(dpp_from_left(vx), vx), tn = fminf(dpp_from_left(vn), vn);
        pmx[p] = fmaxf(dpp_from_right(tx), tx);
        pmn[p] = fminf(dpp_from_right(tn), tn);
    }
    uint32_t ok3 = 0;
#pragma unroll
    for (int s_in = 1; s_in <= kScalesPerOctave; s_in++) {
        const float val = mid[s_in];
        const float mx = fmaxf(fmaxf(pmx[s_in - 1], pmx[s_in]), pmx[s_in + 1]);
        const float mn = fminf(fminf(pmn[s_in - 1], pmn[s_in]), pmn[s_in + 1]);
        const bool ok = yin && fabsf(val) > threshold && (val > 0.0f ? val >= mx : val <= mn);
        ok3 |= (uint32_t)ok << (s_in - 1);
    }
    return ok3;
}

// 73 VGPRs, 6 waves per SIMD; forcing 7 spills in the row loop (+30% time)
#ifndef SIFT_DETECT_WPE
#define SIFT_DETECT_WPE 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_DETECT_WPE))) void k_detect_rows(const DetectLaunch ML) {
    __shared__ uint64_t lcand[DR_LCAP];
    __shared__ uint32_t lcount, gbase;
    // this block's octave (block-uniform: a scan of <= 16 block offsets)
    int oi = 0;
    while (oi + 1 < ML.n_oct && blockIdx.x >= ML.block0[oi + 1]) oi++;
    const DetectOctave& L = ML.oct[oi];
    const int W = L.W, H = L.H, pitch = L.pitch;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int SH = ML.sh;
    const int nsx = (W + DR_COLS - 1) / DR_COLS, nsy = (L.y_hi - L.y_lo + SH - 1) / SH;
    const uint32_t g = (blockIdx.x - ML.block0[oi]) * 4 + wave;  // strip index: frame-major, then row band, then column
    const uint32_t per = (uint32_t)(nsx * nsy);
    const int b = (int)(g / per);
    const uint32_t rem = g - (uint32_t)b * per;
    const int sy = (int)(rem / nsx), sx = (int)(rem % nsx);
    if (tid == 0) lcount = 0;
    __syncthreads();
    if (b < ML.n_img) {
        const float* gb = L.gauss + (size_t)b * L.img_stride;
        const size_t P = (size_t)pitch * H;
        const int x = sx * DR_COLS - 1 + lane;  // this lane's column
        const int xc = min(max(x, 0), W - 1);
        const bool xout = lane >= 1 && lane <= DR_COLS && x >= kImageBorder && x < W - kImageBorder;
        const int y0 = L.y_lo + sy * SH, y1 = min(y0 + SH, L.y_hi);
        // DoG rows y - 1 (prv) and y (mid) at this lane's column
        float prv[kDogPerOctave], mid[kDogPerOctave], nv[kImagesPerOctave];
        // one row of G_0..G_5; the loads of row y + 2 stay in flight as raw
        // Gaussians and become D values (to_dog) when the row is consumed
        auto load_row = [&](int yy, float (&g)[kImagesPerOctave]) {
            const gfloat* rp = as_global(gb) + (size_t)min(max(yy, 0), H - 1) * pitch + xc;
#pragma unroll
            for (int p = 0; p < kImagesPerOctave; p++) g[p] = rp[(size_t)p * P];
        };
        auto to_dog = [&](const float (&g)[kImagesPerOctave], float (&v)[kDogPerOctave]) {
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) v[p] = g[p + 1] - g[p];
        };
        load_row(y0 - 1, nv);
        to_dog(nv, prv);
        load_row(y0, nv);
        to_dog(nv, mid);
        // Two rows in flight (rows y + 1 and y + 2 while row y is tested) in
        // two alternating buffers -- the loop is unrolled by two so neither
        // buffer is copied while its loads are outstanding.
        float nv2[kImagesPerOctave];
        load_row(y0 + 1, nv);
        load_row(y0 + 2, nv2);
        auto step = [&](int y, float (&buf)[kImagesPerOctave]) {
            // row y + 1 arrived in buf; row y + 3 goes in flight into it
            float cur[kDogPerOctave];
            to_dog(buf, cur);
            if (y + 2 < y1) load_row(y + 3, buf);
            const bool yin = xout && y >= kImageBorder && y < H - kImageBorder;
            uint32_t ok3 = extremum3(prv, mid, cur, yin);
            if (__ballot(ok3 != 0)) {  // wave-uniform: rare
                while (ok3) {
                    const int bit = __builtin_ctz(ok3);
                    ok3 &= ok3 - 1;
                    const uint64_t key = make_key((uint32_t)(ML.img_base + b), (uint32_t)L.octave,
                                                  (uint32_t)(bit + 1), (uint32_t)y, (uint32_t)x);
                    const uint32_t li = atomicAdd(&lcount, 1u);
                    if (li < DR_LCAP) {
                        lcand[li] = key;
                    } else {
                        const uint32_t slot = atomicAdd(ML.counter, 1u);
                        if (slot < ML.cap) ML.cand[slot] = key;
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {  // y + 1 becomes the centre row
                prv[p] = mid[p];
                mid[p] = cur[p];
            }
        };
        for (int y = y0; y < y1; y += 2) {
            step(y, nv);
            if (y + 1 < y1) step(y + 1, nv2);
        }
    }
    // one global atomic per block, then a coalesced copy of the block's list
    __syncthreads();
    const uint32_t nl = lcount < DR_LCAP ? lcount : DR_LCAP;
    if (nl == 0) return;
    if (tid == 0) gbase = atomicAdd(ML.counter, nl);
    __syncthreads();
    for (uint32_t i = tid; i < nl; i += 256)
        if (gbase + i < ML.cap) ML.cand[gbase + i] = lcand[i];
}

void launch_detect(DetectLaunch& L, hipStream_t st) {
    // drop empty octaves, then lay the octaves' blocks end to end
    int k = 0;
    for (int i = 0; i < L.n_oct; i++) {
        const DetectOctave& d = L.oct[i];
        if (d.y_lo < 0 || d.y_hi > d.H || d.y_hi <= d.y_lo) continue;
        L.oct[k++] = d;
    }
    L.n_oct = k;
    // A wave walks its strip row after row (~1 us per row at low occupancy):
    // a launch too small to fill the chip twice over at 32-row strips (one
    // frame's octaves) takes shorter ones, down to 4 rows, until it has ~8 k
    // waves
    auto total = [&](int sh) {
        uint32_t nb = 0;
        for (int i = 0; i < k; i++) {
            const DetectOctave& d = L.oct[i];
            const uint32_t strips =
                (uint32_t)((d.W + DR_COLS - 1) / DR_COLS) * ((d.y_hi - d.y_lo + sh - 1) / sh) * L.n_img;
            nb += (strips + 3) / 4;
        }
        return nb;
    };
    int sh = DR_SH;
    while (sh > 4 && total(sh) * 4 < 8192) sh /= 2;
    L.sh = sh;
    uint32_t nb = 0;
    for (int i = 0; i < k; i++) {
        const DetectOctave& d = L.oct[i];
        L.block0[i] = nb;
        const uint32_t strips =
            (uint32_t)((d.W + DR_COLS - 1) / DR_COLS) * ((d.y_hi - d.y_lo + sh - 1) / sh) * L.n_img;
        nb += (strips + 3) / 4;
    }
    L.block0[k] = nb;
    if (nb == 0) return;
    hipLaunchKernelGGL(k_detect_rows, dim3(nb), dim3(256), 0, st, L);
}

// ---------------------------------------------------------------------------
// k_blur_detect: the octave's last blur (G_4 -> G_5, radius R) and the
// extremum scan of its three scales (point_is_local_extremum,
// src/lib.rs:437-506) in one pass.  G_5 is produced on chip, so the scan
// reads G_0..G_4 (G_4 from the blur's own LDS rows) and never reads G_4 /
// G_5 back from HBM: ~26 B per octave pixel for blur 5 and detection
// together instead of ~35 (blur 5: 8 + halo, k_detect_rows: 24 + halo).
//
// A wave owns k_detect_rows' strip geometry: 64 columns x = xb - 1 + lane
// (62 outputs, the edge lanes are halo) by a segment of rows [ya, yb), and
// walks down it one row of G_4 at a time:
//   * the G_4 row's 64 + 2R columns [xb - 1 - R, xb + 63 + R) go to an LDS
//     ring (BD_RING rows per wave; loaded two rows ahead), and each lane's
//     row-filter output at its column is the FMA chain from the leftmost tap
//     of OpenCV's RowFilter (imageproc: the unfused chain) over 2R + 1 ring
//     values -- the same operations as the strip kernels (pyramid.hip);
//   * the last 2R + 1 row-filter outputs are a register window, whose column
//     filter (centre product + fma of the pair sums / imageproc's unfused
//     chain) is G_5 at row r = q - R: stored (rows [ya, yb), lanes 1..62);
//   * row r's D_0..D_4 are formed from G_0..G_3 (loaded two rows ahead),
//     G_4 (its ring row, still resident) and G_5, and the 3x3x3 test of row
//     r - 1 runs on the rolling row max / min exactly as k_detect_rows.
// Rows and columns outside the image are reflect-101 (clamp-to-edge) like the
// strip blur; only rows inside the image are stored or tested, so G_5 and the
// candidates are those of launch_blur + k_detect_rows bit for bit.
// ---------------------------------------------------------------------------
constexpr int BD_RING = 16;  // raw G_4 rows per wave (the rows r .. r + R and the next)
constexpr int BD_RP = 100;   // ring row pitch (floats): 64 + 2R columns, R <= 18
#ifndef BD_UNROLL
#define BD_UNROLL 1  // row groups per steady-state loop iteration
#endif

template <int P>
__device__ __forceinline__ int bd_index(int p, int n) {
    if (P == kProfileOpenCV) p = p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p);
    return p < 0 ? 0 : (p >= n ? n - 1 : p);
}

// 1-D block id remapped so each XCD walks a contiguous range (neighbouring
// strips of one row segment share their G_4 halo columns in that XCD's L2)
__device__ __forceinline__ uint32_t xcd_block_1d() { return xcd_remap(blockIdx.x, gridDim.x); }

template <int R, int P>
#ifndef SIFT_BD_WPE
// waves per SIMD the register budget must allow (1: unconstrained, 104 VGPRs
// = 4 waves).  5 (96 VGPRs, 13 dwords spilled): 4159 / 4176 vs 3213 / 3083 us
// on octave 0 of 64 frames (profiles/r05_ubd31.log)
#define SIFT_BD_WPE 1
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_BD_WPE))) void k_blur_detect(
    const BlurDetectLaunch L) {
    static_assert(64 + 2 * R <= BD_RP && R + 3 <= BD_RING, "ring geometry");
    __shared__ float ring[4][BD_RING * BD_RP];
    __shared__ uint64_t lcand[DR_LCAP];
    __shared__ uint32_t lcount, gbase;
    // the wave index through readfirstlane: everything derived from it (the
    // strip, its rows, the buffer row offsets) is then known to be uniform
    // and lives in SGPRs -- a soffset the compiler cannot prove uniform turns
    // every buffer access into a readfirstlane waterfall loop
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W = L.W, H = L.H, pitch = L.pitch;
    const uint32_t g = xcd_block_1d() * 4 + wave;  // strip index: frame-major, then row segment, then column
    const uint32_t per = (uint32_t)(L.nsx * L.nsy);
    const int b = (int)(g / per);
    const uint32_t rem = g - (uint32_t)b * per;
    const int sy = (int)(rem / (uint32_t)L.nsx), sx = (int)(rem % (uint32_t)L.nsx);
    if (tid == 0) lcount = 0;
    __syncthreads();
    if (b < L.n_img) {
        const size_t P_ = (size_t)pitch * H;
        const uint32_t pb = (uint32_t)P_ * 4u;  // plane bytes (< 2^31: launch_blur_detect)
        const float* gb = L.gauss + (size_t)b * L.img_stride;
        const __amdgpu_buffer_rsrc_t rg0 = uniform_rsrc(gb, pb), rg1 = uniform_rsrc(gb + P_, pb),
                                     rg2 = uniform_rsrc(gb + 2 * P_, pb), rg3 = uniform_rsrc(gb + 3 * P_, pb),
                                     rg4 = uniform_rsrc(gb + 4 * P_, pb), rg5 = uniform_rsrc(gb + 5 * P_, pb);
        const int xb = sx * DR_COLS;
        const int x = xb - 1 + lane;  // this lane's column
        const int xc = min(max(x, 0), W - 1);
        const bool xout = lane >= 1 && lane <= DR_COLS && x >= kImageBorder && x < W - kImageBorder;
        const bool xst = lane >= 1 && lane <= DR_COLS && x < W;
        const int ya = sy * L.seg, yb = min(ya + L.seg, H);
        // G_4 ring columns [xb - 1 - R, xb + 63 + R): lane -> column ca, and
        // lanes < 2R also ca + 64
        const int ca = xb - 1 - R + lane;
        const int va = bd_index<P>(ca, W) * 4, vb = bd_index<P>(ca + 64, W) * 4, vx = xc * 4;
        float* rg = ring[wave];
        auto ld4 = [&](int q, float& a, float& c) {  // G_4 row q (reflected) into registers
            const int so = bd_index<P>(q, H) * pitch * 4;
            // both loads on every lane (vb is clamped into the row): an
            // exec-masked load sits behind a skip branch, which makes the
            // compiler's load-counter waits conservative
            a = buffer_load_f32(rg4, va, so);
            c = buffer_load_f32(rg4, vb, so);
        };
        auto ld03 = [&](int r, float (&d)[4]) {  // G_0..G_3 at (row r clamped, column xc)
            const int so = min(max(r, 0), H - 1) * pitch * 4;
            d[0] = buffer_load_f32(rg0, vx, so);
            d[1] = buffer_load_f32(rg1, vx, so);
            d[2] = buffer_load_f32(rg2, vx, so);
            d[3] = buffer_load_f32(rg3, vx, so);
        };
        // row filter of G_4 row q at this lane's column (q's ring row)
        auto rowpass = [&](int q) -> float {
            const float* p = rg + (q & (BD_RING - 1)) * BD_RP + lane;
            float v[2 * R + 1];
#pragma unroll
            for (int t = 0; t <= 2 * R; t++) v[t] = p[t];
            float acc = v[0] * L.taps.k[R];
#pragma unroll
            for (int t = 1; t <= 2 * R; t++) {
                const float kt = L.taps.k[t > R ? t - R : R - t];
                acc = P == kProfileOpenCV ? __builtin_fmaf(v[t], kt, acc) : acc + v[t] * kt;
            }
            return acc;
        };
        float win[2 * R + 1];  // row-filter outputs of rows r - R .. r + R
        // detection state: the DoG rows r - 2 (prv) and r - 1 (mid)
        float prv[kDogPerOctave] = {}, mid[kDogPerOctave] = {};
        const int q0 = ya - 1 - R, q1 = yb + R;  // G_4 rows filtered: [q0, q1]
        // Row data of one G_4 row q: its ring columns (a, c) and G_0..G_3 of
        // row r = q - R at this lane's column (the window-filling rows r <
        // ya - 1 load rows ya - 1 / ya instead; rows past the end re-load
        // the last one).  Four buffers: the two rows of a half-iteration are
        // processed from one pair while the next two rows' loads, issued at the
        // top of the half, are in flight into the other pair.  Every half
        // issues the same memory operations (a G_5 row outside the segment is
        // stored to an offset the buffer drops), so the compiler's load-counter
        // waits are static: each waits for loads issued a half-iteration
        // earlier, never for the ones just issued.
        struct RowBuf {
            float a, c, d[4];
        };
        auto load = [&](int q, RowBuf& B, int par) {
            const int qq = min(q, q1), r = qq - R;
            ld4(qq, B.a, B.c);
            ld03(r >= ya - 1 ? min(r, yb) : ya - 1 + par, B.d);
        };
        auto shift = [&]() {
#pragma unroll
            for (int j = 0; j < 2 * R; j++) win[j] = win[j + 1];
        };
        // G_4 row q from B into the ring, row-filtered into win[2R]; once the
        // window holds rows r - R .. r + R (r = q - R >= ya - 1): G_5 of row r,
        // row r's DoG values, the test of row r - 1.  Steps past q1 only
        // issue their (dropped) store.
        // FULL: a steady-state row (q <= q1, and row r - 1 >= ya is tested):
        // no uniform branches, so the rolling state needs no reconciling
        // copies between paths -- only the segment's first 2R + 2 rows and
        // its last few take the guarded form.
        auto step = [&](int q, const RowBuf& B, auto full_tag) {
            constexpr bool FULL = decltype(full_tag)::value;
            const bool on = FULL || q <= q1;  // uniform
            const int r = q - R;
            float g5 = 0.0f;
            if (on) {
                float* wp = rg + (q & (BD_RING - 1)) * BD_RP;
                wp[lane] = B.a;
                if (lane < 2 * R) wp[64 + lane] = B.c;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                win[2 * R] = rowpass(q);
                if constexpr (P == kProfileOpenCV) {
                    g5 = win[R] * L.taps.k[0];
#pragma unroll
                    for (int t = 1; t <= R; t++) g5 = __builtin_fmaf(win[R + t] + win[R - t], L.taps.k[t], g5);
                } else {
                    g5 = win[0] * L.taps.k[R];
#pragma unroll
                    for (int t = 1; t <= 2 * R; t++) g5 = g5 + win[t] * L.taps.k[t > R ? t - R : R - t];
                }
            }
            // (a FULL row has r >= ya + 1; its last one may be r = yb, the
            // next segment's row: dropped like every row past the segment)
            const uint32_t bad = ((FULL || (on && r >= ya)) && r < yb && xst) ? 0u : 0xfffffff0u;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, g5), rg5,
                                                  ((uint32_t)(r * pitch * 4) + (uint32_t)vx) | bad, 0, 2 /* nt */);
            if (!FULL && !(on && r >= ya - 1)) {  // uniform
                shift();
                return;
            }
            // row r's DoG values (G_4 from the ring: row r is resident)
            const float g4 = rg[(r & (BD_RING - 1)) * BD_RP + lane + R];
            float cur[kDogPerOctave];
            cur[0] = B.d[1] - B.d[0];
            cur[1] = B.d[2] - B.d[1];
            cur[2] = B.d[3] - B.d[2];
            cur[3] = g4 - B.d[3];
            cur[4] = g5 - g4;
            const int y = r - 1;  // tested row: rows r - 2, r - 1, r are in
            if (FULL || y >= ya) {  // uniform
                const bool yin = xout && y >= kImageBorder && y < H - kImageBorder;
                uint32_t ok3 = extremum3(prv, mid, cur, yin);
                if (__ballot(ok3 != 0)) {  // wave-uniform: rare
                    while (ok3) {
                        const int bit = __builtin_ctz(ok3);
                        ok3 &= ok3 - 1;
                        const uint64_t key = make_key((uint32_t)(L.img_base + b), (uint32_t)L.octave,
                                                      (uint32_t)(bit + 1), (uint32_t)y, (uint32_t)x);
                        const uint32_t li = atomicAdd(&lcount, 1u);
                        if (li < DR_LCAP) {
                            lcand[li] = key;
                        } else {
                            const uint32_t slot = atomicAdd(L.counter, 1u);
                            if (slot < L.cap) L.cand[slot] = key;
                        }
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                prv[p] = mid[p];
                mid[p] = cur[p];
            }
            shift();
        };
        // rows q, q + 1 from (A0, A1) while q + 2, q + 3 load into (B0, B1),
        // then the other way round (even / odd rows: par 0 / 1)
        RowBuf A0, A1, B0, B1;
        constexpr int GROUP = 4;
        auto group = [&](int q, auto full_tag) {
            load(q + 2, B0, 0);
            load(q + 3, B1, 1);
            __builtin_amdgcn_sched_barrier(0);
            step(q, A0, full_tag);
            step(q + 1, A1, full_tag);
            __builtin_amdgcn_sched_barrier(0);
            load(q + 4, A0, 0);
            load(q + 5, A1, 1);
            __builtin_amdgcn_sched_barrier(0);
            step(q + 2, B0, full_tag);
            step(q + 3, B1, full_tag);
            __builtin_amdgcn_sched_barrier(0);
        };
        load(q0, A0, 0);
        load(q0 + 1, A1, 1);
        // window fill: rows q0 .. ya + R (2R + 2 rows), then the steady rows
        // a group at a time, the last rows guarded again (a guarded step is
        // exact at any row, so the fill may run past ya + R)
        int q = q0;
        for (; q < ya + R + 1; q += GROUP) group(q, std::false_type{});
        for (; q + GROUP * BD_UNROLL - 1 <= q1; q += GROUP * BD_UNROLL) {
#pragma unroll
            for (int u = 0; u < BD_UNROLL; u++) group(q + GROUP * u, std::true_type{});
        }
        for (; q <= q1; q += GROUP) group(q, std::false_type{});
    }
    // one global atomic per block, then a coalesced copy of the block's list
    __syncthreads();
    const uint32_t nl = lcount < DR_LCAP ? lcount : DR_LCAP;
    if (nl == 0) return;
    if (tid == 0) gbase = atomicAdd(L.counter, nl);
    __syncthreads();
    for (uint32_t i = tid; i < nl; i += 256)
        if (gbase + i < L.cap) L.cand[gbase + i] = lcand[i];
}

// ---------------------------------------------------------------------------
// k_blur_detect_pair: k_blur_detect with two column strips per lane.  Lane l
// owns columns x0 = xb - 1 + l and x1 = x0 + 62, so a wave covers 124 output
// columns (two 62-column halves, lanes 0 / 63 the halo of each).  The blur's
// arithmetic runs on the pair {x0, x1} as packed f32 (v_pk_fma_f32 /
// v_pk_mul_f32 / v_pk_add_f32: two lanes' worth per instruction, each half
// the same IEEE operation sequence as the single-column kernel, so G_5 is
// bit-identical); the ring row's taps for the pair are ring[t] and
// ring[t + 62], one ds_read2_b32 into a register pair.  The DoG differences
// are packed too; the extremum scan runs on each half (max / min have no
// packed form).  The test is branch-free: each scale's verdict is a lane mask
// (val == the 27-value max or min on its side of 0, val != 0), and the
// per-lane key bits are formed only when some lane of the wave has one.
// ---------------------------------------------------------------------------
typedef float bd_f2 __attribute__((ext_vector_type(2)));
constexpr int BD2_COLS = 2 * DR_COLS;  // output columns per wave
// The G_4 ring holds a row as 90 column pairs {c, c + 62} (8-byte slots, the
// taps of the two halves side by side): slot j of a lane's tap t is j = lane
// + t, read with one ds_read_b64 straight into the register pair the packed
// FMA takes.
constexpr int BD2_SLOTS = DR_COLS + 2 + 2 * 13;  // 90: lanes 0..63 plus the 2R taps (R <= 13)

// The scan of one half: three lane masks, scale s of row y - 1 at this
// lane's column a candidate (rows prv, mid, cur of the five DoG planes).
struct ScanMasks {
    bool s1, s2, s3;
};
__device__ __forceinline__ ScanMasks extremum3_masks(const float (&prv)[kDogPerOctave], const float (&mid)[kDogPerOctave],
                                                     const float (&cur)[kDogPerOctave], bool yin) {
    float pmx[kDogPerOctave], pmn[kDogPerOctave];
#pragma unroll
    for (int p = 0; p < kDogPerOctave; p++) {
        const float vx = fmaxf(fmaxf(prv[p], mid[p]), cur[p]);
        const float vn = fminf(fminf(prv[p], mid[p]), cur[p]);
        const float tx = fmaxf(dpp_from_left(vx), vx), tn = fminf(dpp_from_left(vn), vn);
        pmx[p] = fmaxf(dpp_from_right(tx), tx);
        pmn[p] = fminf(dpp_from_right(tn), tn);
    }
    bool ok[kScalesPerOctave];
#pragma unroll
    for (int s_in = 1; s_in <= kScalesPerOctave; s_in++) {
        // threshold 0 (src/lib.rs:460): val != 0, then val >= the max (val > 0)
        // or <= the min (val < 0).  The max / min include val, so >= / <= is
        // equality with the side's extreme.
        const float val = mid[s_in];
        const float mx = fmaxf(fmaxf(pmx[s_in - 1], pmx[s_in]), pmx[s_in + 1]);
        const float mn = fminf(fminf(pmn[s_in - 1], pmn[s_in]), pmn[s_in + 1]);
        const float ext = val > 0.0f ? mx : mn;
        ok[s_in - 1] = yin & (val != 0.0f) & (val == ext);
    }
    return ScanMasks{ok[0], ok[1], ok[2]};
}

#ifndef SIFT_BD2_WPE
#define SIFT_BD2_WPE 1
#endif
template <int R, int P, int NB, int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SIFT_BD2_WPE))) void k_blur_detect_pair(
    const BlurDetectLaunch L) {
    static_assert(R <= 13 && R + 3 <= BD_RING, "ring geometry");
    __shared__ bd_f2 ring[4][BD_RING * BD2_SLOTS];
    __shared__ uint64_t lcand[DR_LCAP];
    __shared__ uint32_t lcount, gbase;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int W = L.W, H = L.H, pitch = L.pitch;
    const uint32_t g = xcd_block_1d() * 4 + wave;  // strip index: frame-major, then row segment, then column
    const uint32_t per = (uint32_t)(L.nsx * L.nsy);
    const int b = (int)(g / per);
    const uint32_t rem = g - (uint32_t)b * per;
    const int sy = (int)(rem / (uint32_t)L.nsx), sx = (int)(rem % (uint32_t)L.nsx);
    if (tid == 0) lcount = 0;
    __syncthreads();
    if (b < L.n_img) {
        const size_t P_ = (size_t)pitch * H;
        const int pb = (int)((uint32_t)P_ * 4u);  // plane bytes (6 planes < 2^31: launch_blur_detect)
        // one resource over the frame's six planes; the plane is a scalar offset
        const __amdgpu_buffer_rsrc_t rgs = uniform_rsrc(L.gauss + (size_t)b * L.img_stride, (uint32_t)(6 * pb));
        const int xb = sx * BD2_COLS;
        const int x0 = xb - 1 + lane, x1 = x0 + DR_COLS;  // this lane's two columns
        const int vx0 = min(max(x0, 0), W - 1) * 4, vx1 = min(max(x1, 0), W - 1) * 4;
        const bool edge = lane >= 1 && lane <= DR_COLS;
        const bool xout0 = edge && x0 >= kImageBorder && x0 < W - kImageBorder;
        const bool xout1 = edge && x1 >= kImageBorder && x1 < W - kImageBorder;
        const uint32_t xbad0 = (edge && x0 < W) ? 0u : 0xfffffff0u, xbad1 = (edge && x1 < W) ? 0u : 0xfffffff0u;
        const int ya = sy * L.seg, yb = min(ya + L.seg, H);
        // ring slot j = {column xb - 1 - R + j, the same + 62}: lane l fills
        // slot l and (l < 26) slot l + 64
        const int ca = xb - 1 - R + lane;
        const int va = bd_index<P>(ca, W) * 4, vb = bd_index<P>(ca + DR_COLS, W) * 4,
                  vc = bd_index<P>(ca + 64, W) * 4, vd = bd_index<P>(ca + 64 + DR_COLS, W) * 4;
        const bool second = lane < BD2_SLOTS - 64;
        bd_f2* rg = ring[wave];
        struct RowBuf {
            bd_f2 s0, s1;  // ring slots lane, lane + 64
            bd_f2 d[4];    // G_0..G_3 at the two columns
        };
        const int q0 = ya - 1 - R, q1 = yb + R;  // G_4 rows filtered: [q0, q1]
        auto load = [&](int q, RowBuf& B, int par) {
            const int qq = min(q, q1), r = qq - R;
            const int so = bd_index<P>(qq, H) * pitch * 4 + 4 * pb;
            B.s0 = bd_f2{buffer_load_f32(rgs, va, so), buffer_load_f32(rgs, vb, so)};
            B.s1 = bd_f2{buffer_load_f32(rgs, vc, so), buffer_load_f32(rgs, vd, so)};
            const int rr = r >= ya - 1 ? min(r, yb) : ya - 1 + par;
            const int sd = min(max(rr, 0), H - 1) * pitch * 4;
#pragma unroll
            for (int p = 0; p < 4; p++)
                B.d[p] = bd_f2{buffer_load_f32(rgs, vx0, sd + p * pb), buffer_load_f32(rgs, vx1, sd + p * pb)};
        };
        // row filter of G_4 row q at this lane's two columns
        auto rowpass = [&](int q) -> bd_f2 {
            const bd_f2* p = rg + (q & (BD_RING - 1)) * BD2_SLOTS + lane;
            bd_f2 v[2 * R + 1];
#pragma unroll
            for (int t = 0; t <= 2 * R; t++) v[t] = p[t];
            bd_f2 acc = v[0] * L.taps.k[R];
#pragma unroll
            for (int t = 1; t <= 2 * R; t++) {
                const float kt = L.taps.k[t > R ? t - R : R - t];
                if constexpr (P == kProfileOpenCV)
                    acc = __builtin_elementwise_fma(v[t], (bd_f2)kt, acc);
                else
                    acc = acc + v[t] * kt;
            }
            return acc;
        };
        bd_f2 win[2 * R + 1];
        float prv0[kDogPerOctave] = {}, mid0[kDogPerOctave] = {}, prv1[kDogPerOctave] = {}, mid1[kDogPerOctave] = {};
        auto shift = [&]() {
#pragma unroll
            for (int j = 0; j < 2 * R; j++) win[j] = win[j + 1];
        };
        auto emit = [&](const ScanMasks& m, int y, int x) {
            uint32_t ok3 = (uint32_t)m.s1 | ((uint32_t)m.s2 << 1) | ((uint32_t)m.s3 << 2);
            while (ok3) {
                const int bit = __builtin_ctz(ok3);
                ok3 &= ok3 - 1;
                const uint64_t key = make_key((uint32_t)(L.img_base + b), (uint32_t)L.octave, (uint32_t)(bit + 1),
                                              (uint32_t)y, (uint32_t)x);
                const uint32_t li = atomicAdd(&lcount, 1u);
                if (li < DR_LCAP) {
                    lcand[li] = key;
                } else {
                    const uint32_t slot = atomicAdd(L.counter, 1u);
                    if (slot < L.cap) L.cand[slot] = key;
                }
            }
        };
        auto step = [&](int q, const RowBuf& B, auto full_tag) {
            constexpr bool FULL = decltype(full_tag)::value;
            const bool on = FULL || q <= q1;  // uniform: G_4 row q is row-filtered
            const int r = q - R;              // the G_5 row this step forms
            bd_f2 g5 = bd_f2{0.0f, 0.0f};
            if (on) {
                bd_f2* wp = rg + (q & (BD_RING - 1)) * BD2_SLOTS;
                wp[lane] = B.s0;
                if (second) wp[64 + lane] = B.s1;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                win[2 * R] = rowpass(q);
                if constexpr (P == kProfileOpenCV) {
                    g5 = win[R] * L.taps.k[0];
#pragma unroll
                    for (int t = 1; t <= R; t++)
                        g5 = __builtin_elementwise_fma(win[R + t] + win[R - t], (bd_f2)L.taps.k[t], g5);
                } else {
                    g5 = win[0] * L.taps.k[R];
#pragma unroll
                    for (int t = 1; t <= 2 * R; t++) g5 = g5 + win[t] * L.taps.k[t > R ? t - R : R - t];
                }
            }
            const uint32_t rbad = ((FULL || (on && r >= ya)) && r < yb) ? 0u : 0xfffffff0u;
            const int so5 = r * pitch * 4 + 5 * pb;
            // (the halves through scalars: a __builtin_bit_cast of g5.y, an
            // element of a vector lvalue, reads element 0 in this clang)
            const float g5x = g5.x, g5y = g5.y;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g5x), rgs, (uint32_t)vx0 | rbad | xbad0, so5,
                                                  2 /* nt */);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g5y), rgs, (uint32_t)vx1 | rbad | xbad1, so5,
                                                  2 /* nt */);
            if (!FULL && !(on && r >= ya - 1)) {  // uniform
                shift();
                return;
            }
            // row r's DoG values (G_4 from the ring: row r is resident)
            const bd_f2 g4 = rg[(r & (BD_RING - 1)) * BD2_SLOTS + lane + R];
            bd_f2 cur[kDogPerOctave];
            cur[0] = B.d[1] - B.d[0];
            cur[1] = B.d[2] - B.d[1];
            cur[2] = B.d[3] - B.d[2];
            cur[3] = g4 - B.d[3];
            cur[4] = g5 - g4;
            float c0[kDogPerOctave], c1[kDogPerOctave];
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                c0[p] = cur[p].x;
                c1[p] = cur[p].y;
            }
            const int y = r - 1;  // tested row: rows r - 2, r - 1, r are in
            if (FULL || y >= ya) {  // uniform
                const bool yin = y >= kImageBorder && y < H - kImageBorder;
                const ScanMasks m0 = extremum3_masks(prv0, mid0, c0, yin && xout0);
                const ScanMasks m1 = extremum3_masks(prv1, mid1, c1, yin && xout1);
                if (__builtin_amdgcn_ballot_w64(m0.s1 | m0.s2 | m0.s3 | m1.s1 | m1.s2 | m1.s3)) {  // rare
                    emit(m0, y, x0);
                    emit(m1, y, x1);
                }
            }
#pragma unroll
            for (int p = 0; p < kDogPerOctave; p++) {
                prv0[p] = mid0[p];
                mid0[p] = c0[p];
                prv1[p] = mid1[p];
                mid1[p] = c1[p];
            }
            shift();
        };
        // NB buffer pairs: rows q, q + 1 are processed from one pair while
        // the next NB - 1 pairs' loads (rows up to q + 2 NB - 1) are in flight
        RowBuf buf[NB][2];
        constexpr int GROUP = 2 * NB;
        auto group = [&](int q, auto full_tag) {
#pragma unroll
            for (int k = 0; k < NB; k++) {
                load(q + 2 * k + 2 * (NB - 1), buf[(k + NB - 1) % NB][0], 0);
                load(q + 2 * k + 2 * (NB - 1) + 1, buf[(k + NB - 1) % NB][1], 1);
                __builtin_amdgcn_sched_barrier(0);
                step(q + 2 * k, buf[k][0], full_tag);
                step(q + 2 * k + 1, buf[k][1], full_tag);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
#pragma unroll
        for (int k = 0; k < NB - 1; k++) {
            load(q0 + 2 * k, buf[k][0], 0);
            load(q0 + 2 * k + 1, buf[k][1], 1);
        }
        int q = q0;
        for (; q < ya + R + 1; q += GROUP) group(q, std::false_type{});
        if constexpr (NB == 2 && U == 3) {
            // three groups per iteration: the rolling DoG rows (a 3-cycle)
            // and the buffer pairs (a 2-cycle) return to their registers
            for (; q + 3 * GROUP - 1 <= q1; q += 3 * GROUP) {
                group(q, std::true_type{});
                group(q + GROUP, std::true_type{});
                group(q + 2 * GROUP, std::true_type{});
            }
        }
        for (; q + GROUP - 1 <= q1; q += GROUP) group(q, std::true_type{});
        for (; q <= q1; q += GROUP) group(q, std::false_type{});
    }
    __syncthreads();
    const uint32_t nl = lcount < DR_LCAP ? lcount : DR_LCAP;
    if (nl == 0) return;
    if (tid == 0) gbase = atomicAdd(L.counter, nl);
    __syncthreads();
    for (uint32_t i = tid; i < nl; i += 256)
        if (gbase + i < L.cap) L.cand[gbase + i] = lcand[i];
}

// PathOpts::fused_detect: 0 keeps blur 5 and detection apart, 2 fuses every
// octave it can at 32-row segments (test paths)
// Whether L runs as k_blur_detect_pair (its one buffer resource spans the
// frame's six planes: < 2^31 bytes; larger octaves -- octave 0 of an 8192^2
// frame -- take the one-column kernel, whose resources are per plane).
static bool blur_detect_pair(const BlurDetectLaunch& L, const PathOpts& o) {
    return o.bd_pair && (uint64_t)L.H * (uint64_t)L.pitch * 4 * 6 < (1ull << 31);
}

// The segment length the fused pass would use for L (0: it does not apply).
static int blur_detect_segment(int R, const BlurDetectLaunch& L, const PathOpts& o) {
    if (o.fused_detect == 0) return 0;
    const bool ok = L.W > R + 1 && L.H > R + 1 && L.W >= 2 * kImageBorder && L.H >= 2 * kImageBorder &&
                    (uint64_t)L.H * (uint64_t)L.pitch * 4 < (1ull << 31) && L.n_img > 0;
    if (!ok) return 0;
    const bool pair = blur_detect_pair(L, o);
    const bool ocv = L.profile == kProfileOpenCV;
    if (!((ocv && R == 13) || (!ocv && R == 7))) return 0;
    if (o.fused_detect == 2) return 32;  // many segment boundaries on test-sized frames
    // row segments: a segment re-filters 2R + 2 halo rows, so long ones, but
    // enough waves to fill the chip (>= ~16 k).  A wave walks its segment row
    // after row, so an octave too small for that at >= 64-row segments (one
    // 1080p frame's octaves, a batch's small octaves) is left to launch_blur +
    // k_detect_rows: there the fused pass is a chain of latency-bound row
    // steps (one frame's octave 4: 54 us against 10 us for its blur 5)
    // The octave's rows split into nsy equal segments, not nsy - 1 full ones
    // and a remainder (octave 0 of 64 1080p frames: 3240 vs 3290 us; 384- or
    // 512-row segments, fewer and longer: 3290-3320 us)
    const int cols = pair ? BD2_COLS : DR_COLS;
    const long nsx = (L.W + cols - 1) / cols;
    const long want = pair ? o.bd_waves : 16384;
    for (int s : {256, 128, 64}) {
        const int nsy = (L.H + s - 1) / s;
        if (nsx * nsy * L.n_img >= want) return (L.H + nsy - 1) / nsy;
    }
    return 0;
}

bool blur_detect_applies(int R, const BlurDetectLaunch& L, const PathOpts& o) {
    return blur_detect_segment(R, L, o) > 0;
}

int launch_blur_detect(int R, BlurDetectLaunch& L, hipStream_t st, const PathOpts& o) {
    const int seg = blur_detect_segment(R, L, o);
    if (!seg) return -1;
    const bool pair = blur_detect_pair(L, o);
    const int cols = pair ? BD2_COLS : DR_COLS;
    L.nsx = (L.W + cols - 1) / cols;
    L.seg = seg;
    L.nsy = (L.H + seg - 1) / seg;
    const long waves = (long)L.nsx * L.nsy * L.n_img;
    const dim3 grid((uint32_t)((waves + 3) / 4));
    if (pair && o.bd_pair == 2) {
        if (L.profile == kProfileOpenCV)
            hipLaunchKernelGGL((k_blur_detect_pair<13, kProfileOpenCV, 2, 1>), grid, dim3(256), 0, st, L);
        else
            hipLaunchKernelGGL((k_blur_detect_pair<7, kProfileImageproc, 2, 1>), grid, dim3(256), 0, st, L);
    } else if (pair) {
        if (L.profile == kProfileOpenCV)
            hipLaunchKernelGGL((k_blur_detect_pair<13, kProfileOpenCV, 2, 3>), grid, dim3(256), 0, st, L);
        else
            hipLaunchKernelGGL((k_blur_detect_pair<7, kProfileImageproc, 2, 3>), grid, dim3(256), 0, st, L);
    } else if (L.profile == kProfileOpenCV)
        hipLaunchKernelGGL((k_blur_detect<13, kProfileOpenCV>), grid, dim3(256), 0, st, L);
    else
        hipLaunchKernelGGL((k_blur_detect<7, kProfileImageproc>), grid, dim3(256), 0, st, L);
    return 0;
}

}  // namespace siftmi
