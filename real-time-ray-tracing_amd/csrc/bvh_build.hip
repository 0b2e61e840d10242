// bvh_build.hip — per-frame two-level LBVH build for gfx950, one launch.
//
// Replaces the reference's six launches (bvh.cu:7-97):
//   UpdateSceneGeometry -> RadixSort -> BuildLBVH   (per 1024-triangle BLAS batch)
//   UpdateTLAS -> RadixSort -> BuildLBVH             (one TLAS over the batch roots)
// with ONE kernel: a 1024-thread workgroup (16 wave64s) builds a whole batch inside LDS
// (gather -> batch box -> Morton -> 5x6-bit LSD radix sort -> Karras topology -> bottom-up
// boxes), and the last workgroup to finish (agent-scope release/acquire on an arrival
// counter, cdna_hip_programming.md Guideline 16) builds the TLAS with the same LDS
// machinery.  Results are bit-identical to the reference semantics (oracle/bvh.cpp):
//   * Morton codes: same fp32 ops, no contraction, saturating float->uint
//   * sort: stable LSD radix on the low 30 bits (all codes < 2^30; padding keys
//     0xFFFFFFFF sit at the highest positions, so stability keeps them last) == the
//     reference's stable 32-bit sort (radixSort.cuh:19-246)
//   * Karras: the reference's LCP/direction/split rules (buildBVH.cuh:8-134)
//   * boxes: a pure function of the topology; evaluated by atomic bottom-up climbing in LDS
//   * TLAS scene box: the reference's reduction skips thread slots s with s mod 64 >= 32
//     (no +32 merge, updateGeometry.cuh:317-336), i.e. batches b with (b & 255) >= 128.
#include "bvh_kernels.h"
#include "rt_device.h"

using namespace rtd;

namespace {

constexpr int kT = 1024;  // threads per workgroup == triangles per batch (kernel.cuh:579)

struct Lds {
    uint32_t key[2][kT];
    uint16_t idx[2][kT];
    uint32_t hist[64 * 16];   // [digit][wave]
    float leaf[kT][6];        // leaf boxes by original local index (min xyz, max xyz)
    float merged[kT][6];      // merged box of each internal node
    uint16_t childL[kT], childR[kT];  // bit 15 = leaf
    uint16_t parent[kT];
    uint32_t arrive[kT];
    float red[16][6];
    uint32_t isLast;
};

RT_DEV Box load_box(const float* p) {
    Box b;
    b.mn = f3(p[0], p[1], p[2]);
    b.mx = f3(p[3], p[4], p[5]);
    return b;
}
RT_DEV void store_box(float* p, const Box& b) {
    p[0] = b.mn.x; p[1] = b.mn.y; p[2] = b.mn.z;
    p[3] = b.mx.x; p[4] = b.mx.y; p[5] = b.mx.z;
}

RT_DEV uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    x = (x | (x << 16)) & 0x030000FFu; x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;  x = (x | (x << 2)) & 0x09249249u;
    y = (y | (y << 16)) & 0x030000FFu; y = (y | (y << 8)) & 0x0300F00Fu;
    y = (y | (y << 4)) & 0x030C30C3u;  y = (y | (y << 2)) & 0x09249249u;
    z = (z | (z << 16)) & 0x030000FFu; z = (z | (z << 8)) & 0x0300F00Fu;
    z = (z | (z << 4)) & 0x030C30C3u;  z = (z | (z << 2)) & 0x09249249u;
    return x | (y << 1) | (z << 2);
}

RT_DEV uint32_t morton_of(F3 c, const Box& s) {
    F3 u = (c - s.mn) / (s.mx - s.mn);
    return morton3(sat_u32(u.x * 1023.0f), sat_u32(u.y * 1023.0f), sat_u32(u.z * 1023.0f));
}

// wave64 butterfly min/max; min/max are exact, so the order cannot change the bits
RT_DEV Box wave_reduce(Box b) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        b.mn.x = fmn(b.mn.x, __shfl_xor(b.mn.x, off));
        b.mn.y = fmn(b.mn.y, __shfl_xor(b.mn.y, off));
        b.mn.z = fmn(b.mn.z, __shfl_xor(b.mn.z, off));
        b.mx.x = fmx(b.mx.x, __shfl_xor(b.mx.x, off));
        b.mx.y = fmx(b.mx.y, __shfl_xor(b.mx.y, off));
        b.mx.z = fmx(b.mx.z, __shfl_xor(b.mx.z, off));
    }
    return b;
}

// whole-workgroup box reduction (every thread returns the result)
RT_DEV Box block_reduce(Lds& s, Box b) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    b = wave_reduce(b);
    if (lane == 0) store_box(s.red[w], b);
    __syncthreads();
    Box r = load_box(s.red[0]);
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        Box o = load_box(s.red[k]);
        r.mn = min3(r.mn, o.mn);
        r.mx = max3(r.mx, o.mx);
    }
    return r;
}

// Stable LSD radix sort of s.key[0]/s.idx[0] (1024 entries) on bits 0..29, 6 bits per pass.
// Within a wave, lanes with equal digits are ranked by a 6-ballot match mask; waves are
// ranked through a [digit][wave] histogram scanned by wave 0.  Result in s.key[1]/s.idx[1].
RT_DEV void radix_sort(Lds& s) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int src = 0;
#pragma unroll 1
    for (int pass = 0; pass < 5; ++pass) {
        const int dst = src ^ 1;
        const uint32_t k = s.key[src][t];
        const uint16_t ix = s.idx[src][t];
        const uint32_t d = (k >> (6 * pass)) & 63u;
        s.hist[lane * 16 + w] = 0u;
        uint64_t m = ~0ull;
#pragma unroll
        for (int b = 0; b < 6; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            m &= bit ? bal : ~bal;
        }
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (rank == 0) s.hist[d * 16 + w] = (uint32_t)__popcll(m);
        __syncthreads();
        if (w == 0) {
            uint32_t run[16];
            uint32_t sum = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) { run[j] = sum; sum += s.hist[lane * 16 + j]; }
            uint32_t incl = sum;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                uint32_t v = __shfl_up(incl, off);
                if (lane >= off) incl += v;
            }
            const uint32_t base = incl - sum;
#pragma unroll
            for (int j = 0; j < 16; ++j) s.hist[lane * 16 + j] = base + run[j];
        }
        __syncthreads();
        const uint32_t pos = s.hist[d * 16 + w] + rank;
        s.key[dst][pos] = k;
        s.idx[dst][pos] = ix;
        __syncthreads();
        src = dst;
    }
}

RT_DEV int lcp(const uint32_t* key, int n, uint32_t m0, int j) {
    if (j < 0 || j >= n) return 0;
    const uint32_t x = m0 ^ key[j];
    return x == 0u ? 32 : __builtin_clz(x);
}

// Karras 2012 topology over s.key[1][0..n) (buildBVH.cuh:60-134), children into LDS.
RT_DEV void karras(Lds& s, int n) {
    const int i = threadIdx.x;
    if (i >= n - 1) return;
    const uint32_t* key = s.key[1];
    const uint32_t m0 = key[i];
    const int dl = lcp(key, n, m0, i - 1);
    const int dr = lcp(key, n, m0, i + 1);
    const int d = (dr - dl) >= 0 ? 1 : -1;
    const int deltaMin = lcp(key, n, m0, i - d);
    int lmax = 2;
    while (lcp(key, n, m0, i + lmax * d) > deltaMin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (lcp(key, n, m0, i + (l + t) * d) > deltaMin) l += t;
    const int j = i + l * d;
    const int deltaNode = lcp(key, n, m0, j);
    int sp = 0, div = 2;
    while (true) {  // the reference's extra t == 1 probes are no-ops (SURVEY §0 #8b)
        const int t = (l + div - 1) / div;
        if (lcp(key, n, m0, i + (sp + t) * d) > deltaNode) sp += t;
        if (t <= 1) break;
        div *= 2;
    }
    const int gamma = i + sp * d + (d < 0 ? d : 0);
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    if (lo == gamma) {
        s.childL[i] = (uint16_t)(0x8000u | s.idx[1][gamma]);
    } else {
        s.childL[i] = (uint16_t)gamma;
        s.parent[gamma] = (uint16_t)i;
    }
    if (hi == gamma + 1) {
        s.childR[i] = (uint16_t)(0x8000u | s.idx[1][gamma + 1]);
    } else {
        s.childR[i] = (uint16_t)(gamma + 1);
        s.parent[gamma + 1] = (uint16_t)i;
    }
}

RT_DEV void store_node(Node* dst, const Box& l, const Box& r, uint16_t cl, uint16_t cr) {
    Node nd;
    nd.q0 = make_float4(l.mn.x, l.mn.y, l.mn.z, l.mx.x);
    nd.q1 = make_float4(l.mx.y, l.mx.z, r.mn.x, r.mn.y);
    nd.q2 = make_float4(r.mn.z, r.mx.x, r.mx.y, r.mx.z);
    nd.q3 = make_uint4(cl & 0x7FFFu, cr & 0x7FFFu, cl >> 15, cr >> 15);
    *dst = nd;
}

// Bottom-up boxes: nodes whose children are both leaves start climbing; a parent with two
// internal children is finished by the second arrival (LDS counter, acq_rel workgroup
// scope); a parent with one leaf child is finished by its only internal child.
RT_DEV void refit(Lds& s, int n, Node* nodes) {
    const int i = threadIdx.x;
    if (n == 1) {
        if (i == 0) {
            Box zero; zero.mn = f3(0.0f); zero.mx = f3(0.0f);
            store_node(nodes, load_box(s.leaf[0]), zero, 0x8000u, 0x8000u);
        }
        return;
    }
    if (i >= n - 1) return;
    if (!((s.childL[i] & 0x8000u) && (s.childR[i] & 0x8000u))) return;
    int cur = i;
    for (int guard = 0; guard < kT; ++guard) {  // a valid tree ends at the root in < n steps
        const uint16_t cl = s.childL[cur], cr = s.childR[cur];
        const Box l = (cl & 0x8000u) ? load_box(s.leaf[cl & 0x7FFFu]) : load_box(s.merged[cl]);
        const Box r = (cr & 0x8000u) ? load_box(s.leaf[cr & 0x7FFFu]) : load_box(s.merged[cr]);
        store_box(s.merged[cur], box_merge(l, r));
        store_node(nodes + cur, l, r, cl, cr);
        if (cur == 0) break;
        const int p = s.parent[cur];
        const bool twoInternal = !(s.childL[p] & 0x8000u) && !(s.childR[p] & 0x8000u);
        if (twoInternal) {
            const uint32_t old = __hip_atomic_fetch_add(&s.arrive[p], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == 0u) break;
        }
        cur = p;
    }
}

// Sort keys already in s.key[0]/s.idx[0] and build the tree of n leaves into `nodes`.
RT_DEV void sort_and_build(Lds& s, int n, uint32_t* mortonOut, uint32_t* reorderOut, Node* nodes) {
    __syncthreads();
    radix_sort(s);
    const int t = threadIdx.x;
    mortonOut[t] = s.key[1][t];
    reorderOut[t] = s.idx[1][t];
    karras(s, n);
    __syncthreads();
#if !(defined(RTX_BVH_ABL) && RTX_BVH_ABL == 3)
    refit(s, n, nodes);  // (ablation 3: no refit; timing only)
#endif
}

// The TLAS of a scene of at most 64 batches, built by wave 0 of the last workgroup alone: the
// same results as the 1024-thread path (UpdateTLAS + RadixSort + BuildLBVH over B keys) without
// its ~20 workgroup barriers.  The stable sort is a rank count (keys below, plus equal keys of
// lower index: a stable sort's position); the 1024 - B padding keys (0xFFFFFFFF) keep their
// order after the real ones, as the radix sort leaves them.  LDS written by one lane and read by
// another is ordered by wavefront-scope fences.
RT_DEV void tlas_wave(Lds& s, const BvhBuildParams& P, uint32_t B) {
    const int lane = threadIdx.x;  // 0..63
    const Node* nodes = (const Node*)P.nodes;
    s.arrive[lane] = 0u;
    Box rb = box_empty();
    F3 rc = f3(0.0f);
    if ((uint32_t)lane < B) {
        const Node nd = nodes[(size_t)lane * kT];
        Box l, r;
        l.mn = f3(nd.q0.x, nd.q0.y, nd.q0.z); l.mx = f3(nd.q0.w, nd.q1.x, nd.q1.y);
        r.mn = f3(nd.q1.z, nd.q1.w, nd.q2.x); r.mx = f3(nd.q2.y, nd.q2.z, nd.q2.w);
        rb = box_merge(l, r);
        rc = (rb.mx + rb.mn) / 2.0f;
        store_box(P.tlasAabbs + 6 * (size_t)lane, rb);
    }
    store_box(s.leaf[lane], rb);
    // the quirk reduction keeps slots with (s & 255) < 128: every slot below 64
    const Box quirk = wave_reduce(rb);
    const uint32_t key = (uint32_t)lane < B ? morton_of(rc, quirk) : 0xFFFFFFFFu;
    if (lane == 0) store_box(P.tlasSceneAabb, quirk);
    uint32_t rank = 0;
#pragma unroll 8
    for (int j = 0; j < 64; ++j) {
        const uint32_t kj = __shfl(key, j);
        rank += (kj < key || (kj == key && j < lane)) ? 1u : 0u;
    }
    s.key[1][rank] = key;
    s.idx[1][rank] = (uint16_t)lane;
    for (int t = lane; t < kT; t += 64) {
        P.tlasMorton[t] = t < 64 ? 0u : 0xFFFFFFFFu;  // rows < 64 rewritten below
        P.tlasReorder[t] = (uint32_t)t;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    P.tlasMorton[lane] = s.key[1][lane];
    P.tlasReorder[lane] = s.idx[1][lane];
    karras(s, (int)B);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    refit(s, (int)B, (Node*)P.tlasNodes);
    if (lane == 0) __hip_atomic_store(P.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// t through a VALU move the compiler cannot see through, so an LDS slot address derived from it is
// recomputed where it is used instead of being kept (and spilled) from an earlier use
RT_DEV int opaque_lane(int t) {
    int r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}

__global__ __launch_bounds__(kT, 8) void k_build_bvh(BvhBuildParams P) {  // 8 waves/SIMD = 2 workgroups per CU: <= 64 VGPRs
    __shared__ Lds s;
    const int t = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint32_t B = P.batchCount;
    const uint32_t start = b * kT;
    const uint32_t cnt = (b + 1 < B) ? (uint32_t)kT : P.triCount - (B - 1) * kT;  // init.cu:129-130
    const uint32_t active = (((cnt - 1) >> 2) + 1) << 2;  // triangles of threads with tid*4 <= cnt-1

    // ---- gather triangles, leaf boxes, centroids (updateGeometry.cuh:104-184)
    Box bx = box_empty();
    F3 center = f3(0.0f);
    if ((uint32_t)t < active) {
        const uint32_t g = start + t;
        const uint32_t i0 = P.indices[3 * g], i1 = P.indices[3 * g + 1], i2 = P.indices[3 * g + 2];
        const F3 v1 = f3(P.vertices[3 * i0], P.vertices[3 * i0 + 1], P.vertices[3 * i0 + 2]);
        const F3 v2 = f3(P.vertices[3 * i1], P.vertices[3 * i1 + 1], P.vertices[3 * i1 + 2]);
        const F3 v3 = f3(P.vertices[3 * i2], P.vertices[3 * i2 + 1], P.vertices[3 * i2 + 2]);
        P.triPos[3 * g + 0] = make_float4(v1.x, v1.y, v1.z, 0.0f);
        P.triPos[3 * g + 1] = make_float4(v2.x, v2.y, v2.z, 0.0f);
        P.triPos[3 * g + 2] = make_float4(v3.x, v3.y, v3.z, 0.0f);
        P.triNrm[3 * g + 0] = make_float4(P.normals[3 * i0], P.normals[3 * i0 + 1], P.normals[3 * i0 + 2], 0.0f);
        P.triNrm[3 * g + 1] = make_float4(P.normals[3 * i1], P.normals[3 * i1 + 1], P.normals[3 * i1 + 2], 0.0f);
        P.triNrm[3 * g + 2] = make_float4(P.normals[3 * i2], P.normals[3 * i2 + 1], P.normals[3 * i2 + 2], 0.0f);
        F3 mn = min3(v1, min3(v2, v3));
        F3 mx = max3(v1, max3(v2, v3));
        const F3 diff = max3(mx - mn, kMachineEps * mx);
        mx = mn + diff;
        bx.mn = mn;
        bx.mx = mx;
        store_box(P.aabbs + 6 * (size_t)g, bx);
        center = (v1 + v2 + v3) / 3.0f;
    }
    store_box(s.leaf[t], bx);

    // ---- batch box (updateGeometry.cuh:186-248) and Morton codes (:250-261)
    const Box scene = block_reduce(s, bx);
    s.key[0][t] = ((uint32_t)t < active) ? morton_of(center, scene) : 0xFFFFFFFFu;
    s.idx[0][t] = (uint16_t)t;
    if (t == 0) store_box(P.batchSceneAabbs + 6 * (size_t)b, scene);

    Node* const nodes = (Node*)P.nodes;
    // the refit's arrival counters, zeroed here (the sort's barriers order it before the refit)
    // rather than at entry: the slot address would otherwise stay live across the gather, and at
    // the 64-VGPR bound it was spilled to scratch
    s.arrive[opaque_lane(t)] = 0u;
    sort_and_build(s, (int)cnt, P.morton + start, P.reorder + start, nodes + start);

    // ---- arrival: the last workgroup builds the TLAS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t old = __hip_atomic_fetch_add(P.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t last = (old == B - 1) ? 1u : 0u;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        s.isLast = last;
    }
    __syncthreads();
    if (!s.isLast) return;
    if (B <= 64u) {  // small TLAS: wave 0 alone
        if (t < 64) tlas_wave(s, P, B);
        return;
    }
#if defined(RTX_BVH_ABL) && RTX_BVH_ABL == 1
    if (t == 0) __hip_atomic_store(P.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;  // timing ablation: no TLAS
#endif

    // ---- TLAS (UpdateTLAS, updateGeometry.cuh:264-364; then sort + Karras over B keys)
    s.arrive[opaque_lane(t)] = 0u;
    Box rb = box_empty();
    F3 rc = f3(0.0f);
    if ((uint32_t)t < B) {
        const Node nd = nodes[(size_t)t * kT];
        Box l, r;
        l.mn = f3(nd.q0.x, nd.q0.y, nd.q0.z); l.mx = f3(nd.q0.w, nd.q1.x, nd.q1.y);
        r.mn = f3(nd.q1.z, nd.q1.w, nd.q2.x); r.mx = f3(nd.q2.y, nd.q2.z, nd.q2.w);
        rb = box_merge(l, r);
        rc = (rb.mx + rb.mn) / 2.0f;
        store_box(P.tlasAabbs + 6 * (size_t)t, rb);
    }
    store_box(s.leaf[t], rb);
    const Box contrib = ((uint32_t)t < B && (t & 255) < 128) ? rb : box_empty();
    const Box quirk = block_reduce(s, contrib);
    s.key[0][t] = ((uint32_t)t < B) ? morton_of(rc, quirk) : 0xFFFFFFFFu;
    s.idx[0][t] = (uint16_t)t;
    if (t == 0) store_box(P.tlasSceneAabb, quirk);
    sort_and_build(s, (int)B, P.tlasMorton, P.tlasReorder, (Node*)P.tlasNodes);
    __syncthreads();
    if (t == 0) __hip_atomic_store(P.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

extern "C" hipError_t rtk_launch_build_bvh(const BvhBuildParams* p, hipStream_t stream) {
    hipLaunchKernelGGL(k_build_bvh, dim3(p->batchCount), dim3(kT), 0, stream, *p);
    return hipGetLastError();
}
