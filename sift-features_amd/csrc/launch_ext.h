// Kernel launch with an optional completion event (shared by the stage
// launchers).  The next kernel a launcher enqueues from this host thread
// after set_launch_done_event(e) signals e on completion -- hipExtLaunchKernel's
// stop event, no marker packet of its own: a marker between two kernels costs
// ~7 us of the stream's timeline.
#pragma once
#include <hip/hip_ext.h>

#include <tuple>

namespace siftmi {

inline thread_local hipEvent_t t_done = nullptr;

template <class F, class... A>
inline void klaunch(F kernel, dim3 grid, dim3 block, hipStream_t st, A... args) {
    if (t_done) {
        hipEvent_t e = t_done;
        t_done = nullptr;
        // hipExtLaunchKernelGGL's packing, with its status checked: on failure
        // the kernel goes out plainly and e is recorded after it
        auto tup_ = std::tuple<A...>{args...};
        auto tup = validateArgsCountType(kernel, tup_);
        void* kargs[sizeof...(A) > 0 ? sizeof...(A) : 1];
        pArgs<0>(tup, kargs);
        if (hipExtLaunchKernel(reinterpret_cast<void*>(kernel), grid, block, kargs, 0, st, nullptr, e, 0) !=
            hipSuccess) {
            (void)hipGetLastError();
            hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
            (void)hipEventRecord(e, st);
        }
    } else {
        hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
    }
}

}  // namespace siftmi
