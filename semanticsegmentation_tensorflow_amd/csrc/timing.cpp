// Timing events for per-launch kernel timing (Session.timer, bench.py's
// roofline): HIP events created with hipEventDisableSystemFence.  A plain
// timing event (hipEventDefault, torch.cuda.Event(enable_timing=True)) ends
// its interval with a system-scope release -- an L2 write-back + invalidate --
// which is both counted in the bracketed interval and slows the next kernel:
// measured +23 us (+15 %) per conv_halo2 launch in the C2 step against the
// kernel durations of a rocprofv3 trace of the same steps.  Host code (HIP
// runtime API only, no kernels).
#include <hip/hip_runtime.h>

#include "../../include/segkern.h"

extern "C" int seg_timing_event_create(void** ev) {
    if (!ev) return SEG_EINVAL;
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return SEG_ELAUNCH;
    *ev = (void*)e;
    return SEG_OK;
}

extern "C" int seg_timing_event_record(void* ev, void* stream) {
    if (!ev) return SEG_EINVAL;
    return hipEventRecord((hipEvent_t)ev, (hipStream_t)stream) == hipSuccess ? SEG_OK : SEG_ELAUNCH;
}

// Milliseconds from start to end; waits for end to complete.
extern "C" int seg_timing_event_elapsed_ms(float* ms, void* start, void* end) {
    if (!ms || !start || !end) return SEG_EINVAL;
    if (hipEventSynchronize((hipEvent_t)end) != hipSuccess) return SEG_ELAUNCH;
    return hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end) == hipSuccess ? SEG_OK : SEG_ELAUNCH;
}

extern "C" int seg_timing_event_destroy(void* ev) {
    if (!ev) return SEG_OK;
    return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? SEG_OK : SEG_ELAUNCH;
}
