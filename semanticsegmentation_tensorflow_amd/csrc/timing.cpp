// Host-side HIP runtime helpers (no kernels).
//
// Timing events for per-launch kernel timing (Session.timer, bench.py's
// roofline): HIP events created with hipEventDisableSystemFence.  A plain
// timing event (hipEventDefault, torch.cuda.Event(enable_timing=True)) ends
// its interval with a system-scope release -- an L2 write-back + invalidate --
// which is both counted in the bracketed interval and slows the next kernel:
// measured +23 us (+15 %) per conv_halo2 launch in the C2 step against the
// kernel durations of a rocprofv3 trace of the same steps.  Host code (HIP
// runtime API only, no kernels).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

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

// A stream whose kernels run only on the CUs set in `mask` (nwords 32-bit
// words, bit i = CU i in the runtime's order): the Session's stream for the
// fused conv6 / conv7 filter-gradient + Adam launches, so that HBM-bound
// update cannot hold every CU while the input-gradient chain waits (its
// 256 x 256 conv tiles need a whole CU's LDS).
extern "C" int seg_stream_create_cu_mask(void** stream, const unsigned* mask, int nwords) {
    if (!stream || !mask || nwords <= 0) return SEG_EINVAL;
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) return SEG_ELAUNCH;
    *stream = (void*)s;
    return SEG_OK;
}

extern "C" int seg_stream_destroy(void* stream) {
    if (!stream) return SEG_OK;
    return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? SEG_OK : SEG_ELAUNCH;
}
