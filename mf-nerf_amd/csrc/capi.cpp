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

extern "C" {

const char* mfnerf_last_error(void) { return g_err; }

int mfnerf_abi_version(void) { return 2; }

}  // extern "C"
