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

#include "sift_common.h"
#include "sift_kernels.h"

namespace siftmi {

size_t sort_pairs_u64(void* temp, size_t temp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                      uint32_t* vout, uint32_t n, int end_bit, hipStream_t st) {
    size_t bytes = temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(temp, bytes, kin, kout, vin, vout, (int)n, 0, end_bit, st) != hipSuccess)
        return 0;
    return bytes;
}

__global__ void k_make_sort_keys(const KpRec* __restrict__ kp, uint32_t n, uint64_t* __restrict__ keys,
                                 uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = kp[i].key;
    vals[i] = i;
}

void launch_make_sort_keys(const KpRec* kp, uint32_t n, uint64_t* keys, uint32_t* vals, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_make_sort_keys, dim3((n + 255) / 256), dim3(256), 0, st, kp, n, keys, vals);
}

__global__ void k_frame_starts(const uint64_t* __restrict__ keys, uint32_t n, uint32_t* __restrict__ starts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t f = (uint32_t)(keys[i] >> kKeyImgShift);
    if (i == 0 || (uint32_t)(keys[i - 1] >> kKeyImgShift) != f) starts[f] = i;
}

void launch_frame_starts(const uint64_t* sorted_keys, uint32_t n, uint32_t* starts, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_frame_starts, dim3((n + 255) / 256), dim3(256), 0, st, sorted_keys, n, starts);
}

// key = (frame << 32) | ~bits(response)  (response >= 0, so bit order == value order)
__global__ void k_make_resp_keys(const KpRec* __restrict__ kp, const uint32_t* __restrict__ order, uint32_t n,
                                 int img_base, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const KpRec k = kp[order[i]];
    const uint32_t bits = __float_as_uint(k.response);
    keys[i] = ((uint64_t)(uint32_t)(k.img - img_base) << 32) | (uint64_t)(~bits);
    vals[i] = order[i];
}

void launch_make_resp_keys(const KpRec* kp, const uint32_t* order, uint32_t n, int img_base, uint64_t* keys,
                           uint32_t* vals, hipStream_t st) {
    if (!n) return;
    hipLaunchKernelGGL(k_make_resp_keys, dim3((n + 255) / 256), dim3(256), 0, st, kp, order, n, img_base, keys, vals);
}

__global__ void k_select(const uint32_t* __restrict__ emis, const uint32_t* __restrict__ resp,
                         const uint32_t* __restrict__ seg_off, const uint32_t* __restrict__ out_off,
                         const uint8_t* __restrict__ use_resp, int n_img, uint32_t n_out, uint32_t* __restrict__ fin) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
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
                   const uint32_t* out_off, const uint8_t* use_resp, int n_img, uint32_t n_out, uint32_t* final_idx,
                   hipStream_t st) {
    if (!n_out) return;
    hipLaunchKernelGGL(k_select, dim3((n_out + 255) / 256), dim3(256), 0, st, emis_order, resp_order, seg_off, out_off,
                       use_resp, n_img, n_out, final_idx);
}

}  // namespace siftmi
