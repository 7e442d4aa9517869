// Keypoint ordering on MI355X.
//
// The reference emits keypoints lazily in (octave, initial scale, initial
// row, initial column, orientation peak) order (src/lib.rs:281-294,
// :324-332, :397-431).  The detection kernels append with atomics, so the
// order is restored with one LSD radix sort of the 64-bit emission keys
// (hipcub / rocPRIM onesweep).  With a features_limit the frames whose count
// exceeds the limit are re-sorted by response, descending (src/lib.rs:156-161,
// stable w.r.t. emission order for ties) and truncated.
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>

#include "launch_ext.h"
#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {

// onesweep: rocprim's Onesweep radix sort for every size above one block
// (merge_sort_limit 0); otherwise the library default, which takes a block
// radix sort of 1024-key tiles plus merge passes up to 1 M keys
size_t sort_pairs_u64(void* temp, size_t temp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                      uint32_t* vout, uint32_t n, int end_bit, hipStream_t st, bool onesweep) {
    size_t bytes = temp_bytes;
    hipError_t e;
    if (onesweep) {
        using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                               rocprim::default_config, 0>;
        e = rocprim::radix_sort_pairs<Cfg>(temp, bytes, kin, kout, vin, vout, n, 0u, (unsigned)end_bit, st);
    } else {
        e = hipcub::DeviceRadixSort::SortPairs(temp, bytes, kin, kout, vin, vout, (int)n, 0, end_bit, st);
    }
    return e == hipSuccess ? bytes : 0;
}

// Per-chunk counters in one launch (instead of three memsets): cnt[0..3] = 0,
// the m frame starts = ~0 (no keypoint), the descriptor work queues = 0.
__global__ void k_chunk_init(uint32_t* __restrict__ cnt, int m, int work_words) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 4) cnt[i] = 0;
    if (i < m) cnt[4 + i] = 0xffffffffu;
    if (i < work_words) cnt[4 + 2 * m + i] = 0;
}

void launch_chunk_init(uint32_t* cnt, int m, int work_words, hipStream_t st) {
    const int n = std::max(std::max(4, m), work_words);
    hipLaunchKernelGGL(k_chunk_init, dim3((n + 255) / 256), dim3(256), 0, st, cnt, m, work_words);
}

__global__ void k_make_sort_keys(const KpRec* __restrict__ kp, const uint32_t* __restrict__ n_dev, uint32_t bound,
                                 uint64_t pad, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= bound) return;
    const uint32_t n = min(*n_dev, bound);
    keys[i] = i < n ? kp[i].key : pad;
    vals[i] = i;
}

void launch_make_sort_keys(const KpRec* kp, const uint32_t* n, uint32_t bound, uint64_t pad, uint64_t* keys,
                           uint32_t* vals, hipStream_t st) {
    if (!bound) return;
    hipLaunchKernelGGL(k_make_sort_keys, dim3((bound + 255) / 256), dim3(256), 0, st, kp, n, bound, pad, keys, vals);
}

__global__ void k_frame_starts(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ n_dev, uint32_t bound,
                               uint32_t* __restrict__ starts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = min(*n_dev, bound);
    if (i >= n) return;
    const uint32_t f = (uint32_t)(keys[i] >> kKeyImgShift);
    if (i == 0 || (uint32_t)(keys[i - 1] >> kKeyImgShift) != f) starts[f] = i;
}

void launch_frame_starts(const uint64_t* sorted_keys, const uint32_t* n, uint32_t bound, uint32_t* starts,
                         hipStream_t st) {
    if (!bound) return;
    hipLaunchKernelGGL(k_frame_starts, dim3((bound + 255) / 256), dim3(256), 0, st, sorted_keys, n, bound, starts);
}

// One workgroup; frame f = thread (n_img <= kLimitPlanFrames).  cnt[f] =
// next non-empty start - start[f] (starts are in sorted order, so that is
// the end of frame f's segment), then exclusive prefix sums of the counts
// and of the output counts over the block.
constexpr int kLimitPlanFrames = 256;
__global__ __launch_bounds__(kLimitPlanFrames) void k_limit_plan(const uint32_t* __restrict__ starts,
                                                                 const uint32_t* __restrict__ n_kp, uint32_t bound,
                                                                 int n_img, int64_t limit,
                                                                 uint32_t* __restrict__ out_cnt,
                                                                 uint32_t* __restrict__ seg_off,
                                                                 uint32_t* __restrict__ out_off,
                                                                 uint8_t* __restrict__ use_resp,
                                                                 uint32_t* __restrict__ n_out) {
    __shared__ uint32_t st[kLimitPlanFrames + 1];
    __shared__ uint32_t wsum[2][kLimitPlanFrames / 64];
    const int f = threadIdx.x, lane = f & 63, wv = f >> 6;
    const uint32_t n = min(*n_kp, bound);
    const uint32_t s = f < n_img ? starts[f] : 0xffffffffu;
    // end of frame f: the smallest start among later frames (suffix min), else n
    st[f] = s;
    __syncthreads();
    uint32_t nxt = 0xffffffffu;
    for (int g = n_img - 1; g > f; g--) nxt = min(nxt, st[g]);
    const uint32_t end = nxt == 0xffffffffu ? n : nxt;
    const uint32_t cnt = s == 0xffffffffu ? 0u : end - s;
    const bool trunc = limit >= 0 && (uint64_t)limit < cnt;
    const uint32_t oc = trunc ? (uint32_t)limit : cnt;
    // inclusive scans within each wave, then the waves' totals
    uint32_t seg = cnt, out = oc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t a = __shfl_up(seg, o), b = __shfl_up(out, o);
        if (lane >= o) {
            seg += a;
            out += b;
        }
    }
    if (lane == 63) {
        wsum[0][wv] = seg;
        wsum[1][wv] = out;
    }
    __syncthreads();
    for (int w = 0; w < wv; w++) {
        seg += wsum[0][w];
        out += wsum[1][w];
    }
    if (f < n_img) {
        out_cnt[f] = oc;
        seg_off[f] = seg - cnt;
        out_off[f] = out - oc;
        use_resp[f] = trunc ? 1 : 0;
    }
    if (f == kLimitPlanFrames - 1) *n_out = out;
}

void launch_limit_plan(const uint32_t* starts, const uint32_t* n_kp, uint32_t bound, int n_img, int64_t limit,
                       uint32_t* out_cnt, uint32_t* seg_off, uint32_t* out_off, uint8_t* use_resp, uint32_t* n_out,
                       hipStream_t st) {
    klaunch(k_limit_plan, dim3(1), dim3(kLimitPlanFrames), st, starts, n_kp, bound, n_img, limit, out_cnt, seg_off,
            out_off, use_resp, n_out);
}

// key = (frame << 32) | ~bits(response)  (response >= 0, so bit order == value order)
__global__ void k_make_resp_keys(const KpRec* __restrict__ kp, const uint32_t* __restrict__ order,
                                 const uint32_t* __restrict__ n_dev, uint32_t bound, int img_base, uint64_t pad,
                                 uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= bound) return;
    const uint32_t n = min(*n_dev, bound);
    if (i >= n) {
        keys[i] = pad;
        vals[i] = 0;
        return;
    }
    const KpRec k = kp[order[i]];
    const uint32_t bits = __float_as_uint(k.response);
    keys[i] = ((uint64_t)(uint32_t)(k.img - img_base) << 32) | (uint64_t)(~bits);
    vals[i] = order[i];
}

void launch_make_resp_keys(const KpRec* kp, const uint32_t* order, const uint32_t* n, uint32_t bound, int img_base,
                           uint64_t pad, uint64_t* keys, uint32_t* vals, hipStream_t st) {
    if (!bound) return;
    hipLaunchKernelGGL(k_make_resp_keys, dim3((bound + 255) / 256), dim3(256), 0, st, kp, order, n, bound, img_base,
                       pad, keys, vals);
}

__global__ void k_select(const uint32_t* __restrict__ emis, const uint32_t* __restrict__ resp,
                         const uint32_t* __restrict__ seg_off, const uint32_t* __restrict__ out_off,
                         const uint8_t* __restrict__ use_resp, int n_img, const uint32_t* __restrict__ n_out_dev,
                         uint32_t bound, uint32_t* __restrict__ fin) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n_out = min(*n_out_dev, bound);
    if (i >= n_out) return;
    int lo = 0, hi = n_img - 1;  // frame f with out_off[f] <= i < out_off[f+1]
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (out_off[mid] <= i)
            lo = mid;
        else
            hi = mid - 1;
    }
    const uint32_t j = seg_off[lo] + (i - out_off[lo]);
    fin[i] = use_resp[lo] ? resp[j] : emis[j];
}

void launch_select(const uint32_t* emis_order, const uint32_t* resp_order, const uint32_t* seg_off,
                   const uint32_t* out_off, const uint8_t* use_resp, int n_img, const uint32_t* n_out, uint32_t bound,
                   uint32_t* final_idx, hipStream_t st) {
    if (!bound) return;
    hipLaunchKernelGGL(k_select, dim3((bound + 255) / 256), dim3(256), 0, st, emis_order, resp_order, seg_off, out_off,
                       use_resp, n_img, n_out, bound, final_idx);
}

// Outputs of a call whose descriptors were computed in keypoint index order
// (one-frame calls: k_describe runs beside the ordering stage): row j of the
// outputs is keypoint order[j] -- its descriptor (16 bytes per thread), its
// KeyPoint (src/lib.rs:163-176: x, y, size * DELTA_MIN) and its emission key.
// Block 0 also copies the chunk's counters (cnt_words words) to the host's
// pinned buffer, written back to host memory before the kernel ends (system
// fence): no copy command after the kernel (~4 us plus its dispatch).
__global__ void k_gather_out(const KpRec* __restrict__ kp, const uint32_t* __restrict__ order,
                             const uint32_t* __restrict__ n_out, uint32_t bound, const uint4* __restrict__ desc_in,
                             uint4* __restrict__ desc_out, OutKp* __restrict__ out_kp, uint64_t* __restrict__ out_key,
                             uint64_t key_base, const uint32_t* __restrict__ cnt, uint32_t* __restrict__ h_cnt,
                             int cnt_words) {
    constexpr uint32_t kParts = kDescSize / 16;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (h_cnt && blockIdx.x == 0) {
        for (int w = threadIdx.x; w < cnt_words; w += blockDim.x) h_cnt[w] = cnt[w];
        __threadfence_system();
    }
    const uint32_t j = t / kParts, part = t % kParts;
    const uint32_t n = min(*n_out, bound);
    if (j >= n) return;
    const uint32_t i = order[j];
    desc_out[(size_t)j * kParts + part] = desc_in[(size_t)i * kParts + part];
    if (part == 0) {
        const KpRec r = kp[i];
        OutKp k;
        k.x = r.x * 0.5f;
        k.y = r.y * 0.5f;
        k.size = r.size * 0.5f;
        k.angle = r.angle;
        k.response = r.response;
        out_kp[j] = k;
        out_key[j] = r.key + key_base;
    }
}

void launch_gather_out(const KpRec* kp, const uint32_t* order, const uint32_t* n_out, uint32_t bound,
                       const uint8_t* desc_in, uint8_t* desc_out, OutKp* out_kp, uint64_t* out_key, uint64_t key_base,
                       const uint32_t* cnt, uint32_t* h_cnt, int cnt_words, hipStream_t st) {
    if (!bound) return;
    const uint64_t threads = (uint64_t)bound * (kDescSize / 16);
    klaunch(k_gather_out, dim3((unsigned)((threads + 255) / 256)), dim3(256), st, kp, order, n_out, bound,
            reinterpret_cast<const uint4*>(desc_in), reinterpret_cast<uint4*>(desc_out), out_kp, out_key, key_base, cnt,
            h_cnt, cnt_words);
}

}  // namespace siftmi
