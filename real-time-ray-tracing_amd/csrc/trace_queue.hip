// trace_queue.hip — persistent tracer of a deferred-ray queue (wavefront path tracing,
// DESIGN.md §4) for gfx950.
//
// The bounce and shadow rays leaving a surface are incoherent: inside one wave64 their
// traversals differ in length by an order of magnitude, and the single-kernel path tracer
// kept every lane of a wave waiting for its longest ray at 2 waves/SIMD.  Here a lean kernel
// (traversal state only) runs at 5 waves/SIMD, and each wave refills its idle lanes from the
// queue (one atomic per 64 rays, see Fetch) so lanes stay busy until the queue is drained
// (Aila & Laine 2009, persistent threads with dynamic fetch).
//
// Each lane runs TraverseBvh (traverse.h:107-253) one iteration per trav_step call, so the
// reference semantics — 16-entry LDS stack with dropped overflow pushes, nearer child first,
// 1024-iteration cap — hold per ray exactly as in the inline traversal.
//
// Exit: a lane becomes `exhausted` once its reserve is empty and every part is drained; the
// wave leaves the loop when no lane holds a ray, which every wave reaches because the fetch
// counters only grow and every ray ends within 1024 iterations.
#include "frame_kernels.h"
#include "queue_fetch.h"
#include "traverse.h"

using namespace rtd;

namespace {

constexpr int kTraceBlock = 256;
constexpr uint32_t kTrace3Short = 1u << 20;  // queue-3 length below which trace3ShortBlocks apply
#ifndef RTX_LEAF_BATCH
#define RTX_LEAF_BATCH 1
#endif
constexpr bool kLeafBatch = RTX_LEAF_BATCH != 0;  // ablation: -DRTX_LEAF_BATCH=0

// kStats: the launch keeps per-pixel statistics (P.statsOut), so the traversal counts visits and tests
template <int kStep, bool kStats>
__global__ __launch_bounds__(kTraceBlock) void k_trace_queue(PathTraceParams P) {
    __shared__ uint2 stk[17 * kTraceBlock];  // 16 entries + the dead slot trav_step stores above the top
    // The tracers' waves issue at the denoise kernels' priority (DN_PRIO), above the next frame's
    // camera waves: in a pipelined frame the context stream binds (bench.py binding_stream), and its
    // queue tracers' time is their longest rays' dependent iterations, which stretch when the SIMD
    // arbiter serves the camera waves first.  Measured (tools/ab.sh, three repeats): frame
    // 0.803-0.811 -> 0.782-0.792 ms, trace<3> 0.287 -> 0.244 ms, trace<4> 0.203 -> 0.166 ms, terrain
    // 3.20-3.24 -> 3.16-3.21 ms; trace<4> alone at 3: 0.785-0.790; both at 2: 0.799-0.802; the resume
    // kernels at 3 on top: no better (profiles/r05_ab/queue_prio/).  (Round 4, with the shade kernel
    // at 2 waves per SIMD and the post stream binding, the same measured slower.)
    __builtin_amdgcn_s_setprio(3);
    const int tid = threadIdx.x;
    const int lane = (int)__lane_id();
    const PtQueue& q = kStep == 3 ? P.ws.q3 : P.ws.q4;
    const uint32_t n = P.ws.counters[kStep == 3 ? kCntQ3 : kCntQ4];
    uint32_t* fetchCounters = P.ws.fetch + (kStep == 3 ? 0 : kParts * 16);
    const SceneView sc = scene_view(P.nodes, P.tlasNodes, P.triPos, P.triNrm);

    // a short queue 3 runs on the first trace3ShortBlocks workgroups only (frame.cpp); the others
    // leave before taking any work, and the static first batches are cut over the ones that stay
    uint32_t blocks = gridDim.x;
    if (kStep == 3 && P.ws.trace3ShortBlocks != 0u && n < kTrace3Short && P.ws.trace3ShortBlocks < blocks)
        blocks = P.ws.trace3ShortBlocks;
    if (blockIdx.x >= blocks) return;
    const uint32_t wavesPerBlock = kTraceBlock / 64;
    Fetch f;
    fetch_init(f, n, blocks * wavesPerBlock, blockIdx.x * wavesPerBlock + (uint32_t)(tid >> 6));

    bool active = false, exhausted = false, occlusion = false;
    uint32_t idx = 0, accV = 0, accT = 0;
    TravRay r;
    TravState s;
    TravRec rec;  // the record the lane's next iteration processes
    r.org = f3(0.0f);
    trav_init(s, sc.root);
#pragma unroll 1
    while (true) {
        const unsigned long long need = __ballot(!active && !exhausted);
        const unsigned long long busy = __ballot(active);
        if (need != 0ull && (__popcll(need) >= kRefillMin || busy == 0ull)) {
            const uint32_t k = (uint32_t)__popcll(need);
            fetch_topup(f, n, fetchCounters, lane);
            const uint32_t avail = f.resHi - f.resLo;
            const bool none = avail == 0u && f.drained == (1u << kParts) - 1u;
            if (!active && !exhausted) {
                const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
                if (rank < avail) {
                    idx = f.resLo + rank;
                    const float4 o = q.rayO[idx], d = q.rayD[idx];
                    trav_setup(sc, f3(o.x, o.y, o.z), f3(d.x, d.y, d.z), r);
                    trav_init(s, sc.root);
                    rec = trav_first_rec(sc);
                    active = true;
                    occlusion = kStep == 4 || (__float_as_uint(d.w) & kQShadowFlag) != 0u;
                } else if (none) {
                    exhausted = true;
                }
            }
            f.resLo += k < avail ? k : avail;
        }
        if (__ballot(active) == 0ull) break;
        // Tail: this wave's reserve is empty and every part drained, so no lane can be refilled.
        // The remaining rays then run in a plain per-lane loop, without the refill ballots and the
        // leaf batching (a wave in the tail has few lanes left, and its iteration latency is the
        // kernel's tail).  Each ray's steps are unchanged.
        const bool tail = f.resLo == f.resHi && f.drained == (1u << kParts) - 1u;
        if (tail || !kLeafBatch ? active : trav_lane_steps(active, s)) {
            bool done;
            do {  // two steps per trip: the loop's refill / exec-mask bookkeeping once per two
                done = trav_step<16, true, kStats>(sc, r, s, rec, stk + tid, kTraceBlock, nullptr) || s.iters >= 1024u ||
                       (occlusion && s.hitIdx >= 0);
                if (!done && (tail || !kLeafBatch || trav_lane_steps(true, s)))
                    done = trav_step<16, true, kStats>(sc, r, s, rec, stk + tid, kTraceBlock, nullptr) || s.iters >= 1024u ||
                           (occlusion && s.hitIdx >= 0);
            } while (tail && !done);
            if (done) {
                P.ws.hitRec[idx] = make_float4(s.t, __uint_as_float((uint32_t)s.hitIdx), s.hitU, s.hitV);
                P.ws.hitErr[idx] = s.hitErrT;
                if (P.ws.itersOut) P.ws.itersOut[idx] = s.iters;
                if (P.statsOut) {
                    const uint32_t p = __float_as_uint(q.rayO[idx].w);
                    atomicAdd(&P.statsOut[p].y, s.visits);
                    atomicAdd(&P.statsOut[p].z, s.tests);
                    atomicMax(&P.ws.counters[kStep == 3 ? kCntMaxIter3 : kCntMaxIter4], s.iters);
                    accV += s.visits;
                    accT += s.tests;
                }
                active = false;
            }
        }
    }
    if (P.statsOut) {  // every lane left the loop together (the wave-uniform break above)
        uint32_t v = accV, t = accT;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            v += __shfl_xor(v, o);
            t += __shfl_xor(t, o);
        }
        if (lane == 0) {
            if (v) atomicAdd(&P.ws.counters[kStep == 3 ? kCntVisQ3 : kCntVisQ4], v);
            if (t) atomicAdd(&P.ws.counters[kStep == 3 ? kCntTstQ3 : kCntTstQ4], t);
        }
    }
}

}  // namespace

extern "C" int rtk_trace_queue_blocks_per_cu() {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_trace_queue<3, false>, kTraceBlock, 0) != hipSuccess) return 0;
    return b;
}

extern "C" hipError_t rtk_launch_trace_queue(const PathTraceParams* p, int step, hipStream_t stream) {
    const uint32_t blocks = step == 3 ? p->ws.traceBlocks : p->ws.trace4Blocks;
    if (blocks < 1) return hipErrorInvalidValue;
    const dim3 grid(blocks);
    const bool stats = p->statsOut != nullptr;
    void (*k)(PathTraceParams) = step == 3 ? (stats ? k_trace_queue<3, true> : k_trace_queue<3, false>)
                                           : (stats ? k_trace_queue<4, true> : k_trace_queue<4, false>);
    hipLaunchKernelGGL(k, grid, dim3(kTraceBlock), 0, stream, *p);
    return hipGetLastError();
}
