// queue_fetch.h — work distribution of the persistent queue tracers (trace_queue.hip and the
// fused bounce chain in pathtrace.hip), DESIGN.md §4.1.
#pragma once
#include "rt_device.h"

namespace rtd {

#ifndef RTX_REFILL_MIN
#define RTX_REFILL_MIN 16
#endif
constexpr int kRefillMin = RTX_REFILL_MIN;  // idle lanes that trigger a refill (ablation: -DRTX_REFILL_MIN)
constexpr int kParts = 8;       // fetch counters (one per XCD by blockIdx % 8): spreads the atomics

// Work distribution.  Wave g first takes items [64 g, 64 g + 64) with no atomic: a short queue
// (a sky-dominated frame) costs no atomics at all.  The rest, [64 * waves, n), is cut into
// kParts contiguous parts; a wave tops up a 64-item reserve from its home part (one atomic per
// 64 items), moving on to the next part when its home part is drained.  A same-address
// device-scope atomic serialises at the memory side, so both the static first batch and the
// per-part counters keep the queue of atomics on any one address short.
struct Fetch {
    uint32_t resLo, resHi;  // wave-uniform reserve [resLo, resHi)
    uint32_t dynBase, partLen;
    uint32_t drained;       // bit x: part x has no items left
    int home;
};

// staticFirst = false: no static first batch, every item is fetched (a workgroup dispatched
// late, behind other kernels' waves, then holds back no items)
RT_DEV void fetch_init(Fetch& f, uint32_t n, uint32_t wavesTotal, uint32_t gw, bool staticFirst = true) {
    const uint32_t s0 = staticFirst ? gw * 64u : 0u;
    f.resLo = staticFirst && s0 < n ? s0 : n;
    f.resHi = staticFirst ? (s0 + 64u < n ? s0 + 64u : n) : n;
    f.dynBase = staticFirst ? wavesTotal * 64u : 0u;
    const uint32_t dyn = n > f.dynBase ? n - f.dynBase : 0u;
    f.partLen = (dyn + kParts - 1) / kParts;
    f.drained = dyn == 0u ? (1u << kParts) - 1u : 0u;
    f.home = (int)(blockIdx.x % kParts);
}

// refill an empty reserve from the first part that still has items (wave-uniform call)
RT_DEV void fetch_topup(Fetch& f, uint32_t n, uint32_t* counters, int lane) {
    while (f.resLo == f.resHi && f.drained != (1u << kParts) - 1u) {
        int part = f.home;
        while (f.drained & (1u << part)) part = (part + 1) % kParts;
        uint32_t got = 0u;
        if (lane == 0) got = atomicAdd(&counters[part * 16], 64u);  // counters 64 B apart
        got = __shfl(got, 0);
        const uint32_t lo = f.dynBase + part * f.partLen + got;
        uint32_t hi = f.dynBase + part * f.partLen + (got + 64u < f.partLen ? got + 64u : f.partLen);
        if (hi > n) hi = n;
        if (got >= f.partLen || lo >= hi) {
            f.drained |= 1u << part;
            continue;
        }
        f.resLo = lo;
        f.resHi = hi;
    }
}

}  // namespace rtd
