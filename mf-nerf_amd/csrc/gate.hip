// gate.hip -- a soft cross-stream gate INSIDE captured graphs (performance only, never correctness).
// The training step replays the next batch's draw + march on a side stream so that it runs beside
// this step's table-gradient scatter, not beside the chain (encode -> field -> compositing -> field
// backward), whose CUs it would take.  With host events that start point costs a graph boundary on
// the main stream (the event must be recorded between the chain and the scatter graphs); events
// cannot be recorded inside a captured graph here.  Instead the side stream's graph starts with a
// one-thread wait on a device counter that the chain graph's last node advances, and the chain and
// the scatter + optimizer tail become one graph.  Data hazards stay covered by host events (the side
// stream also waits for the step's start); the wait only delays, and gives up after timeout_us.
#include "common.hpp"
#include "../../include/mfnerf.h"

namespace {

// gate = {signals, waits, -, timeouts}: the chain adds a signal; a wait takes the next ticket and waits for the
// matching signal, then catches up with signals nobody waited for (a chain replayed without a
// gated march), so a desynchronised pair heals after one early start
// Relaxed atomics throughout (placement only, no data is handed over): an agent-scope release writes
// the XCD's dirty L2 lines back and an acquire invalidates its L2 (one L2 per XCD) -- the polling
// loop's acquire did that every ~0.2 us on one XCD for the whole chain (round 5)
__global__ void gate_signal_kernel(int32_t* gate) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(gate, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void gate_wait_kernel(int32_t* gate, int64_t timeout_ticks, int lane_mask) {
    if (threadIdx.x != 0) return;
    // a lane-dependent (opaque) index keeps the polling load a vector memory load
    int32_t* sig = gate + (threadIdx.x & lane_mask);
    const int target = __hip_atomic_fetch_add(gate + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    const uint64_t t0 = wall_clock64();  // constant-rate clock (100 MHz on gfx9)
    int c = __hip_atomic_load(sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (c < target && (int64_t)(wall_clock64() - t0) < timeout_ticks) {
        __builtin_amdgcn_s_sleep(8);
        c = __hip_atomic_load(sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (c > target) __hip_atomic_fetch_max(gate + 1, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // gate[3] counts the waits that gave up (never reset here): the host reads it to tell a slow step
    // from a gate that never opened (e.g. the side stream sharing a hardware queue with the signaller)
    if (c < target) __hip_atomic_fetch_add(gate + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

extern "C" {

int mfnerf_gate_signal(int32_t* gate, mfnerf_stream_t stream) {
    if (!gate) { mfn_set_error("gate_signal: null pointer"); return MFN_ERR_INVALID; }
    hipLaunchKernelGGL(gate_signal_kernel, dim3(1), dim3(64), 0, stream, gate);
    return mfn_check_launch("gate_signal");
}

int mfnerf_gate_wait(int32_t* gate, int64_t timeout_us, mfnerf_stream_t stream) {
    if (!gate || timeout_us < 0) { mfn_set_error("gate_wait: bad arguments"); return MFN_ERR_INVALID; }
    hipLaunchKernelGGL(gate_wait_kernel, dim3(1), dim3(64), 0, stream, gate, timeout_us * 100, 0);
    return mfn_check_launch("gate_wait");
}

}  // extern "C"
