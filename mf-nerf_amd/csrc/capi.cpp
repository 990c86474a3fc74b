// capi.cpp -- error plumbing and versioning of the C ABI (include/mfnerf.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mfnerf.h"

static thread_local char g_err[512] = "";

void mfn_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int mfn_check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        mfn_set_error("%s: HIP error %d (%s)", what, (int)e, hipGetErrorString(e));
        return MFN_ERR_LAUNCH;
    }
    return MFN_OK;
}

// Zero-fill as a KERNEL, never hipMemsetAsync, for every buffer a captured graph clears: a memset
// node in a replayed graph was seen not to run (round 4, test_engine_refresh_end_to_end in the full
// GPU suite: the occupancy refresh's scratch kept the previous refresh's sigmas at ~735 k cells),
// and a kernel node is what every other step of the graphs already relies on.
__global__ void mfn_zero_kernel(uint32_t* __restrict__ p, int64_t n_words) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += stride) p[i] = 0u;
}

void mfn_zero_async(void* p, int64_t bytes, hipStream_t stream) {
    if (bytes <= 0) return;
    const int64_t words = bytes / 4;  // callers clear whole 32-bit words
    const int64_t want = (words + 255) / 256;
    hipLaunchKernelGGL(mfn_zero_kernel, dim3((unsigned)(want < 2048 ? (want < 1 ? 1 : want) : 2048)), dim3(256), 0,
                       stream, (uint32_t*)p, words);
}

extern "C" {

const char* mfnerf_last_error(void) { return g_err; }

int mfnerf_abi_version(void) { return 2; }

}  // extern "C"
