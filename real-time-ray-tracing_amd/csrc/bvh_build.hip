// bvh_build.hip — per-frame two-level LBVH build for gfx950, one launch.
//
// Replaces the reference's six launches (bvh.cu:7-97):
//   UpdateSceneGeometry -> RadixSort -> BuildLBVH   (per 1024-triangle BLAS batch)
//   UpdateTLAS -> RadixSort -> BuildLBVH             (one TLAS over the batch roots)
// with ONE kernel: a workgroup builds a whole batch inside LDS (gather -> batch box -> Morton ->
// 5x6-bit LSD radix sort -> Karras topology -> bottom-up boxes), and one more workgroup builds the
// TLAS with the same LDS machinery beside them, from the batches' root boxes, which each batch
// publishes right after its gather (agent-coherent stores, then a count on a launch counter the TLAS
// workgroup polls; tlas_builder).  Results are bit-identical to the reference semantics
// (oracle/bvh.cpp):
//   * Morton codes: same fp32 ops, no contraction, saturating float->uint
//   * sort: stable LSD radix on the low 30 bits (all codes < 2^30; padding keys
//     0xFFFFFFFF sit at the highest positions, so stability keeps them last) == the
//     reference's stable 32-bit sort (radixSort.cuh:19-246)
//   * Karras: the reference's LCP/direction/split rules (buildBVH.cuh:8-134)
//   * boxes: a pure function of the topology; evaluated by atomic bottom-up climbing in LDS
//   * TLAS scene box: the reference's reduction skips thread slots s with s mod 64 >= 32
//     (no +32 merge, updateGeometry.cuh:317-336), i.e. batches b with (b & 255) >= 128.
//
// Two workgroup shapes (kThr threads, kPer = 1024 / kThr batch elements per thread):
//   kThr 1024  16 waves, one element per thread, leaf boxes in LDS (63 KB): two workgroups fill a
//              CU's 32 wave slots — the default scene's 60 batches, one per CU;
//   kThr 512   8 waves, two elements per thread, leaf boxes read back from the AABB array, 38 KB of
//              LDS: four workgroups per CU, so 937 batches (the 958,720-triangle scene, BASELINE
//              config 4) run in one round on 256 CUs instead of two rounds of 512.
// The launcher takes 512 when the batches would not fit 2 per CU.
#include "bvh_kernels.h"
#include "rt_device.h"

using namespace rtd;

namespace {

constexpr int kBatch = 1024;  // triangles per batch (kernel.cuh:579)

typedef uint32_t __attribute__((may_alias)) U32Alias;

template <int kThr>
struct Lds {
    static constexpr bool kLeafLds = kThr == kBatch;
    // region A: the sort's second key / index buffers and its histogram ([digit][64-element
    // virtual wave]); after the sort, the node info of the Karras topology and the refit:
    // per internal node [0] left child, [1] right child (bit 15 = leaf), [2] parent,
    // [3] arrivals — one 8-byte word, so the refit reads children and parent in one ds_read_b64
    union {
        struct {
            uint32_t key0[kBatch];
            uint16_t idx0[kBatch];
            uint16_t hist[64 * 16];
        } srt;
        uint16_t info[kBatch][4];
    } a;
    uint32_t key1[kBatch];  // sorted keys (the sort ends in buffer 1)
    uint16_t idx1[kBatch];
    float merged[kBatch][6];  // merged box of each internal node (rows 0..2 hold the gather's centroids
                              // until the refit; block_reduce's partials use the sort histogram's area)
    float leaf[kLeafLds ? kBatch : 1][6];  // leaf boxes by original local index (kThr 1024)
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

// A TLAS leaf box through the cross-workgroup hand-off of rt_device.h (xwg_*: agent-coherent stores
// and loads, no release fence — on gfx950 an agent-scope release writes back the producer XCD's
// whole L2, which doubled every batch's gather).
RT_DEV void store_box_agent(float* p, const Box& b) {
    const float v[6] = {b.mn.x, b.mn.y, b.mn.z, b.mx.x, b.mx.y, b.mx.z};
#pragma unroll
    for (int k = 0; k < 6; ++k) xwg_store((uint32_t*)p + k, __float_as_uint(v[k]));
}
RT_DEV Box load_box_agent(const float* p) {
    float v[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = __uint_as_float(xwg_load((const uint32_t*)p + k));
    Box b;
    b.mn = f3(v[0], v[1], v[2]);
    b.mx = f3(v[3], v[4], v[5]);
    return b;
}

// row i of an [n][3] float array: through a 64-bit row pointer (kRows: one dwordx3 load) or with
// 32-bit element indices (three dword loads)
template <bool kRows>
RT_DEV F3 vtx_row(const float* a, uint32_t i) {
    if (kRows) {
        const float* r = a + 3 * (size_t)i;
        return f3(r[0], r[1], r[2]);
    }
    return f3(a[3 * i], a[3 * i + 1], a[3 * i + 2]);
}

// leaf box k: from LDS (kThr 1024) or from the AABB array this launch wrote (leafG)
template <int kThr>
RT_DEV Box leaf_box(const Lds<kThr>& s, const float* leafG, uint32_t k) {
    if (Lds<kThr>::kLeafLds) return load_box(s.leaf[k]);
    return load_box(leafG + 6 * (size_t)k);
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

// t through a VALU move the compiler cannot see through, so an address derived from it is
// recomputed where it is used instead of being kept (and spilled) from an earlier use
RT_DEV int opaque_lane(int t) {
    int r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}

RT_DEV float xor_lane(float v, int lane, int off) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute((lane ^ off) << 2, __float_as_int(v)));
}

// wave64 butterfly min/max; min/max are exact, so the order cannot change the bits.  The lane
// index is opaque per call: the kernel reduces twice (batch box, TLAS box), and shared shuffle
// addresses kept live between the two were spilled at the 64-VGPR bound.
RT_DEV Box wave_reduce(Box b) {
    const int lane = opaque_lane((int)__lane_id());
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        b.mn.x = fmn(b.mn.x, xor_lane(b.mn.x, lane, off));
        b.mn.y = fmn(b.mn.y, xor_lane(b.mn.y, lane, off));
        b.mn.z = fmn(b.mn.z, xor_lane(b.mn.z, lane, off));
        b.mx.x = fmx(b.mx.x, xor_lane(b.mx.x, lane, off));
        b.mx.y = fmx(b.mx.y, xor_lane(b.mx.y, lane, off));
        b.mx.z = fmx(b.mx.z, xor_lane(b.mx.z, lane, off));
    }
    return b;
}

// whole-workgroup box reduction (every thread returns the result); the per-wave partials go to
// the sort histogram's area of region A, which the sort only clears after its first barrier (and
// the key0 / idx0 writes after a reduction do not reach)
template <int kThr>
RT_DEV Box block_reduce(Lds<kThr>& s, Box b) {
    constexpr int kW = kThr / 64;
    static_assert(kW * 6 * 4 <= (int)sizeof(s.a.srt.hist), "reduction partials fit the histogram area");
    float* red = (float*)s.a.srt.hist;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    b = wave_reduce(b);
    if (lane == 0) store_box(red + 6 * w, b);
    __syncthreads();
    Box r = load_box(red);
#pragma unroll
    for (int k = 1; k < kW; ++k) {
        Box o = load_box(red + 6 * k);
        r.mn = min3(r.mn, o.mn);
        r.mx = max3(r.mx, o.mx);
    }
    return r;
}

// Stable LSD radix sort of the 1024 entries key0/idx0 on bits 0..29, 6 bits per pass; result in
// key1/idx1.  Element e sits in 64-element virtual wave e / 64: thread t of wave w holds elements
// t + j * kThr (virtual waves w + j * kW).  Within a virtual wave, elements with equal digits are
// ranked by a 6-ballot match mask; virtual waves are ranked through a [digit][16] histogram
// scanned by wave 0.
template <int kThr>
RT_DEV void radix_sort(Lds<kThr>& s) {
    constexpr int kW = kThr / 64, kPer = kBatch / kThr;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint16_t* hist = s.a.srt.hist;
#pragma unroll 1
    for (int pass = 0; pass < 5; ++pass) {
        const bool fromA = (pass & 1) == 0;  // passes 0, 2, 4 read buffer 0 (region A)
        const uint32_t* ksrc = fromA ? s.a.srt.key0 : s.key1;
        const uint16_t* isrc = fromA ? s.a.srt.idx0 : s.idx1;
        uint32_t* kdst = fromA ? s.key1 : s.a.srt.key0;
        uint16_t* idst = fromA ? s.idx1 : s.a.srt.idx0;
        uint32_t k[kPer], d[kPer], rank[kPer];
        uint16_t ix[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            k[j] = ksrc[t + j * kThr];
            ix[j] = isrc[t + j * kThr];
            d[j] = (k[j] >> (6 * pass)) & 63u;
            hist[lane * 16 + w + j * kW] = 0u;  // this wave's columns, zeroed before its counts
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            // lanes whose digit equals this lane's: the AND over the six bits of (bit ? ballot : ~ballot),
            // with ~ballot = ballot ^ ~0 — per bit one sign-extended inverted bit s (0 where the bit is
            // set, ~0 where clear), the ballot of s == 0, and m &= ballot ^ s as one v_bitop3 per half
            // (LUT 0x60: src0 & (src1 ^ src2))
            const uint32_t nd = ~d[j];
            uint32_t mlo = 0u, mhi = 0u;
#pragma unroll
            for (int b = 0; b < 6; ++b) {
                const uint32_t sb = (uint32_t)((int32_t)(nd << (31 - b)) >> 31);
                const uint64_t bal = __ballot(sb == 0u);
                if (b == 0) {
                    mlo = (uint32_t)bal ^ sb;
                    mhi = (uint32_t)(bal >> 32) ^ sb;
                } else {
                    mlo = __builtin_amdgcn_bitop3_b32(mlo, (uint32_t)bal, sb, 0x60);
                    mhi = __builtin_amdgcn_bitop3_b32(mhi, (uint32_t)(bal >> 32), sb, 0x60);
                }
            }
            const uint64_t m = ((uint64_t)mhi << 32) | mlo;
            rank[j] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (rank[j] == 0) hist[d[j] * 16 + w + j * kW] = (uint16_t)__popcll(m);
        }
        __syncthreads();
        if (w == 0) {
            uint32_t run[16];
            uint32_t sum = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) { run[j] = sum; sum += hist[lane * 16 + j]; }
            uint32_t incl = sum;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                uint32_t v = __shfl_up(incl, off);
                if (lane >= off) incl += v;
            }
            const uint32_t base = incl - sum;
#pragma unroll
            for (int j = 0; j < 16; ++j) hist[lane * 16 + j] = (uint16_t)(base + run[j]);
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const uint32_t pos = hist[d[j] * 16 + w + j * kW] + rank[j];
            kdst[pos] = k[j];
            idst[pos] = ix[j];
        }
        __syncthreads();
    }
}

// delta(i, j) of the reference (buildBVH.cuh:8-20): the common prefix length of key i (m0) and key j,
// 32 for equal keys, 0 for j outside [0, n).  Branch-free: the read is clamped into the array and
// the out-of-range result selected afterwards.
RT_DEV int lcp(const uint32_t* key, int n, uint32_t m0, int j) {
    const int jc = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
    const uint32_t x = m0 ^ key[jc];
    const int c = x == 0u ? 32 : __builtin_clz(x);
    return (uint32_t)j < (uint32_t)n ? c : 0;
}

// Karras 2012 topology over key1[0..n) (buildBVH.cuh:60-134) of internal node i, into the info
// words; also clears node i's arrival count for the refit.  The probes i + k * d (d = +-1) are
// 24-bit multiplies (v_mul_i32_i24, full rate; |k| < 2048) and the split search's ceil(l / div),
// div = 2, 4, 8 ..., a shift: the reference's arithmetic on these operand ranges.
template <int kThr>
RT_DEV void karras_node(Lds<kThr>& s, int n, int i) {
    const uint32_t* key = s.key1;
    const uint32_t m0 = key[i];
    const int dl = lcp(key, n, m0, i - 1);
    const int dr = lcp(key, n, m0, i + 1);
    const int d = (dr - dl) >= 0 ? 1 : -1;
    const int deltaMin = lcp(key, n, m0, i - d);
    int lmax = 2;
    while (lcp(key, n, m0, i + __mul24(lmax, d)) > deltaMin) lmax *= 2;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (lcp(key, n, m0, i + __mul24(l + t, d)) > deltaMin) l += t;
    const int j = i + __mul24(l, d);
    const int deltaNode = lcp(key, n, m0, j);
    int sp = 0, sh = 1;  // div = 2^sh
    while (true) {  // the reference's extra t == 1 probes are no-ops (SURVEY §0 #8b)
        const int t = (l + (1 << sh) - 1) >> sh;  // (l + div - 1) / div, l >= 0
        if (lcp(key, n, m0, i + __mul24(sp + t, d)) > deltaNode) sp += t;
        if (t <= 1) break;
        ++sh;
    }
    const int gamma = i + __mul24(sp, d) + (d < 0 ? d : 0);
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    if (lo == gamma) {
        s.a.info[i][0] = (uint16_t)(0x8000u | s.idx1[gamma]);
    } else {
        s.a.info[i][0] = (uint16_t)gamma;
        s.a.info[gamma][2] = (uint16_t)i;
    }
    if (hi == gamma + 1) {
        s.a.info[i][1] = (uint16_t)(0x8000u | s.idx1[gamma + 1]);
    } else {
        s.a.info[i][1] = (uint16_t)(gamma + 1);
        s.a.info[gamma + 1][2] = (uint16_t)i;
    }
    s.a.info[i][3] = 0u;
}

template <int kThr>
RT_DEV void karras(Lds<kThr>& s, int n) {
#pragma unroll 1
    for (int i = threadIdx.x; i < n - 1; i += kThr) karras_node(s, n, i);
}

// Traversal words of one tree's child references (traverse.h, the record arena): an internal
// child c is the node at nodeBase + c, a leaf c the record at leafBase + c * leafMul (a BLAS: the
// triangle record; the TLAS: batch c's BLAS root), each with its (leaf, BLAS) kind bits.
struct WordCtx {
    uint32_t nodeKind, nodeBase, leafKind, leafBase, leafMul;
};
RT_DEV uint32_t child_word(const WordCtx& w, uint32_t c) {
    const uint32_t i = c & 0x7FFFu;
    return (c & 0x8000u) ? (w.leafKind | (w.leafBase + i * w.leafMul)) : (w.nodeKind | (w.nodeBase + i));
}

// the reference's BVHNode boxes in q0..q2; q3: the children's traversal words and the reference's
// child references (left | right << 16, bit 15 of each = leaf), for rt_download's reference layout
RT_DEV void store_node(Node* dst, const Box& l, const Box& r, uint32_t cl, uint32_t cr, const WordCtx& w) {
    Node nd;
    nd.q0 = make_float4(l.mn.x, l.mn.y, l.mn.z, l.mx.x);
    nd.q1 = make_float4(l.mx.y, l.mx.z, r.mn.x, r.mn.y);
    nd.q2 = make_float4(r.mn.z, r.mx.x, r.mx.y, r.mx.z);
    nd.q3 = make_uint4(child_word(w, cl), child_word(w, cr), (cl & 0xFFFFu) | ((cr & 0xFFFFu) << 16), 0u);
    *dst = nd;
}

template <int kThr>
RT_DEV uint64_t info_of(const Lds<kThr>& s, int k) {
    return *(const volatile unsigned long long*)&s.a.info[k][0];
}

// Bottom-up boxes: nodes whose children are both leaves start climbing; a parent with two
// internal children is finished by the second arrival (LDS counter, acq_rel workgroup scope); a
// parent with one leaf child is finished by its only internal child.
//
// A climbing lane carries the box it just merged to the parent: per step it reads the parent's
// info word (children + grandparent), bumps the arrival count (two internal children only), and
// reads the one sibling box it does not hold.  The boxes are the reference's
// AABBCompact(left, right) / GetMerged values; only the second arrival at a parent reads the
// first one's box from LDS (published before its count update).
struct Climb {
    Box l, r;
    uint64_t inf;
    uint32_t cl, cr;
    int cur;
    bool on;
};

template <int kThr>
RT_DEV void climb_start(const Lds<kThr>& s, const float* leafG, int n, int i, Climb& c) {
    c.on = false;
    c.cur = i;
    if (i >= n - 1) return;
    c.inf = info_of(s, i);
    c.cl = (uint32_t)c.inf & 0xFFFFu;
    c.cr = (uint32_t)(c.inf >> 16) & 0xFFFFu;
    if (!((c.cl & 0x8000u) && (c.cr & 0x8000u))) return;
    c.l = leaf_box(s, leafG, c.cl & 0x7FFFu);
    c.r = leaf_box(s, leafG, c.cr & 0x7FFFu);
    c.on = true;
}

// kDefer: the merged box of every node goes to LDS and refit() stores the nodes afterwards, in
// order; otherwise each climb step stores its node.  On gfx9 vmcnt counts stores too, so a step's
// wait for its sibling-box load also waited for the 64-B node store it had just issued (the refit
// phase of the 958,720-triangle build: 38 k of its 143 k clocks).
template <int kThr, bool kDefer>
RT_DEV void climb_step(Lds<kThr>& s, const float* leafG, Node* nodes, const WordCtx& w, Climb& c) {
    const Box m = box_merge(c.l, c.r);
    if (kDefer) store_box(s.merged[c.cur], m);
    else store_node(nodes + c.cur, c.l, c.r, c.cl, c.cr, w);
    if (c.cur == 0) {
        c.on = false;
        return;
    }
    const int p = (int)(c.inf >> 32) & 0xFFFF;
    const uint64_t pinf = info_of(s, p);
    const uint32_t pl = (uint32_t)pinf & 0xFFFFu, pr = (uint32_t)(pinf >> 16) & 0xFFFFu;
    const bool curLeft = pl == (uint32_t)c.cur;  // cur is internal: its reference has no leaf bit
    const uint32_t sib = curLeft ? pr : pl;
    Box sb;
    if (sib & 0x8000u) {
        sb = leaf_box(s, leafG, sib & 0x7FFFu);
    } else {  // two internal children: the second arrival finishes the parent
        if (!kDefer) store_box(s.merged[c.cur], m);
        const uint32_t old = __hip_atomic_fetch_add((U32Alias*)&s.a.info[p][2], 0x10000u, __ATOMIC_ACQ_REL,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((old >> 16) == 0u) {
            c.on = false;
            return;
        }
        sb = load_box(s.merged[sib]);
    }
    c.l = curLeft ? m : sb;
    c.r = curLeft ? sb : m;
    c.cl = pl;
    c.cr = pr;
    c.inf = pinf;
    c.cur = p;
}

// The climbs of this thread's internal nodes (kPer of them, one after the other).  kDefer (every
// thread of the workgroup calls): the nodes are stored after the climbs, node i by thread i mod kThr,
// from the children's boxes — leaf boxes and the merged boxes the climbs left in LDS — so the stores
// are coalesced and no climb step waits for one.  Without kDefer (the one-wave TLAS) the steps store.
template <int kThr, bool kDefer>
RT_DEV void refit(Lds<kThr>& s, const float* leafG, int n, Node* nodes, const WordCtx& w) {
    constexpr int kPer = kBatch / kThr;
    const int t = threadIdx.x;
    if (n == 1) {
        if (t == 0) {
            Box zero; zero.mn = f3(0.0f); zero.mx = f3(0.0f);
            store_node(nodes, leaf_box(s, leafG, 0u), zero, 0x8000u, 0x8000u, w);
        }
        return;
    }
#pragma unroll 1
    for (int j = 0; j < kPer; ++j) {
        Climb c;
        climb_start(s, leafG, n, t + j * kThr, c);
        for (int guard = 0; guard < kBatch && c.on; ++guard)  // a valid tree ends at the root in < n steps
            climb_step<kThr, kDefer>(s, leafG, nodes, w, c);
    }
    if (!kDefer) return;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int i = t + j * kThr;
        if (i >= n - 1) continue;
        const uint64_t inf = info_of(s, i);
        const uint32_t cl = (uint32_t)inf & 0xFFFFu, cr = (uint32_t)(inf >> 16) & 0xFFFFu;
        const Box l = (cl & 0x8000u) ? leaf_box(s, leafG, cl & 0x7FFFu) : load_box(s.merged[cl]);
        const Box r = (cr & 0x8000u) ? leaf_box(s, leafG, cr & 0x7FFFu) : load_box(s.merged[cr]);
        store_node(nodes + i, l, r, cl, cr, w);
    }
}

// Timing-only builds (-DRTX_BVH_STAMPS, tools/lbvh_stamps.py): s_memtime at the phase boundaries of
// each workgroup (slots 1..6) and s_memrealtime at its start and end (0, 7), kept by thread 0 and
// written over the last 8 Morton keys of its batch at the end
#ifdef RTX_BVH_STAMPS
#define BVH_STAMP(k) do { if (threadIdx.x == 0) g_stamp[k] = (uint32_t)__builtin_readcyclecounter(); } while (0)
#define BVH_RSTAMP(k) do { if (threadIdx.x == 0) g_stamp[k] = (uint32_t)__builtin_amdgcn_s_memrealtime(); } while (0)
__shared__ uint32_t g_stamp[8];
#else
#define BVH_STAMP(k) do { } while (0)
#define BVH_RSTAMP(k) do { } while (0)
#endif

// A batch's TLAS leaf box, published to the TLAS workgroup (tlas_builder): agent-coherent stores,
// complete before the count that announces them (xwg_arrive).  Thread 0 of the batch's workgroup.
// P.skipPublish names a batch that publishes nothing: fault injection for the TLAS wait's timeout
// path ([debug] bvhSkipPublish, tests only; 0xFFFFFFFF otherwise).
RT_DEV void publish_root(const BvhBuildParams& P, uint32_t b, const Box& root) {
    if (b == P.skipPublish) return;
    store_box_agent(P.tlasAabbs + 6 * (size_t)b, root);
    xwg_arrive(P.counter);
}

// Sort the keys in key0/idx0 and build the tree of n leaves into `nodes`.  pub: publish batch b's
// root box from the sorted order (the first n sorted elements are the leaves).
template <int kThr>
RT_DEV void sort_and_build(Lds<kThr>& s, const float* leafG, int n, uint32_t* mortonOut, uint32_t* reorderOut,
                           Node* nodes, const WordCtx& w, const BvhBuildParams* pub = nullptr, uint32_t b = 0) {
    __syncthreads();
    radix_sort(s);
    BVH_STAMP(3);
    if (pub) {
        __syncthreads();  // idx1 complete; the partials below reuse the histogram area
        Box own = box_empty();
#pragma unroll
        for (int j = 0; j < kBatch / kThr; ++j) {
            const int e = threadIdx.x + j * kThr;
            if (e < n) {
                const Box lb = leaf_box(s, leafG, s.idx1[e]);
                own.mn = min3(own.mn, lb.mn);
                own.mx = max3(own.mx, lb.mx);
            }
        }
        Box root = block_reduce(s, own);
        if (n == 1) {  // a one-leaf BLAS's root is (element 0's box, zero box), as refit() stores it
            Box zero;
            zero.mn = f3(0.0f);
            zero.mx = f3(0.0f);
            root = box_merge(leaf_box(s, leafG, 0u), zero);
        }
        if (threadIdx.x == 0) publish_root(*pub, b, root);
        __syncthreads();  // the partials are read before Karras reuses the area
    }
#pragma unroll
    for (int j = 0; j < kBatch / kThr; ++j) {
        const int e = threadIdx.x + j * kThr;
        mortonOut[e] = s.key1[e];
        reorderOut[e] = s.idx1[e];
    }
    karras(s, n);
    __syncthreads();
    BVH_STAMP(4);
    refit<kThr, true>(s, leafG, n, nodes, w);
}

// the TLAS's child words: internal nodes after the B*1024 BLAS slots, leaves at their BLAS roots
RT_DEV WordCtx tlas_words(uint32_t B) { return WordCtx{0u, B * (uint32_t)kBatch, kLeafBit, 0u, (uint32_t)kBatch}; }

// The TLAS of a scene of at most 64 batches, built by wave 0 of the TLAS workgroup alone: the
// same results as the workgroup path (UpdateTLAS + RadixSort + BuildLBVH over B keys) without
// its ~20 workgroup barriers.  The stable sort is a rank count (keys below, plus equal keys of
// lower index: a stable sort's position); the 1024 - B padding keys (0xFFFFFFFF) keep their
// order after the real ones, as the radix sort leaves them.  LDS written by one lane and read by
// another is ordered by wavefront-scope fences.
template <int kThr>
RT_DEV void tlas_wave(Lds<kThr>& s, const BvhBuildParams& P, uint32_t B) {
    const int lane = threadIdx.x;  // 0..63
    Box rb = box_empty();
    F3 rc = f3(0.0f);
    if ((uint32_t)lane < B) {  // the published box, stored back for the refit's plain reads
        rb = load_box_agent(P.tlasAabbs + 6 * (size_t)lane);
        rc = (rb.mx + rb.mn) / 2.0f;
        store_box(P.tlasAabbs + 6 * (size_t)lane, rb);
    }
    if (Lds<kThr>::kLeafLds) store_box(s.leaf[lane], rb);
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
    s.key1[rank] = key;
    s.idx1[rank] = (uint16_t)lane;
    for (int t = lane; t < kBatch; t += 64) {
        P.tlasMorton[t] = t < 64 ? 0u : 0xFFFFFFFFu;  // rows < 64 rewritten below
        P.tlasReorder[t] = (uint32_t)t;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    P.tlasMorton[lane] = s.key1[lane];
    P.tlasReorder[lane] = s.idx1[lane];
    karras(s, (int)B);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    refit<kThr, false>(s, P.tlasAabbs, (int)B, (Node*)P.tlasNodes, tlas_words(B));
}

}  // namespace

// Up to this many batches the TLAS is built by one wave (tlas_wave), beyond by the whole workgroup.
constexpr uint32_t kTlasWaveMax = 64;

// The TLAS (UpdateTLAS, updateGeometry.cuh:264-364; then sort + Karras over B keys), built by
// workgroup B of the launch.  Each batch's workgroup publishes its TLAS leaf box (its BLAS root's
// merged box, computed from the leaf boxes right after the gather) and then counts itself in the
// launch counter; this workgroup, dispatched after every batch's, waits for all B of them, so the
// TLAS is built while the batches sort, Karras-link and refit.
//
// The wait is bounded by the wall clock (P.waitTicks of s_memrealtime, 1 s by default): a batch
// that never publishes must not leave a wave spinning until the GPU is reset.  On a timeout the TLAS
// is still built (from the boxes that are there: the grid drains normally), and the number of
// missing batches goes to the host's status word, which rt_sync / rt_build_bvh report as
// RT_ERR_DEVICE and answer by re-arming the counters.  The counter is re-armed here by subtracting
// B, not by storing 0: a late publisher's count then still lands, and the counter is back at 0 when
// the launch ends whatever the timing.
//
// The count is compared signed: after a timeout the counter sits below zero (wrapped) until the
// host re-arms it, and a build already queued behind the faulty one must not read that wrapped
// count as complete — it waits, times out and reports in turn (its sequence number goes to the
// second status word), instead of reading leaf boxes its batches are still publishing.
RT_DEV bool tlas_short(uint32_t seen, uint32_t B) { return (int32_t)(seen - B) < 0; }
RT_DEV void tlas_wait(const BvhBuildParams& P, uint32_t B) {
    if (threadIdx.x == 0) {
        uint32_t seen = xwg_load(P.counter);
        if (tlas_short(seen, B)) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (tlas_short(seen = xwg_load(P.counter), B) && __builtin_amdgcn_s_memrealtime() - t0 < P.waitTicks)
                __builtin_amdgcn_s_sleep(2);
        }
        if (tlas_short(seen, B)) {
            report_status(P.status, kStatusTlasTimeoutBuild, P.buildSeq);
            report_status(P.status, kStatusTlasTimeout, B - seen);
        }
        xwg_acquire();
    }
    __syncthreads();  // the boxes are read below with agent-coherent loads only
}
RT_DEV void tlas_rearm(const BvhBuildParams& P, uint32_t B) {
    __hip_atomic_fetch_sub(P.counter, B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int kThr>
RT_DEV void tlas_builder(Lds<kThr>& s, const BvhBuildParams& P, uint32_t B) {
    constexpr int kPer = kBatch / kThr;
    const int t = threadIdx.x;
    tlas_wait(P, B);
    if (B <= kTlasWaveMax) {  // wave 0 alone
        if (t < 64) tlas_wave(s, P, B);
#ifdef RTX_BVH_STAMPS
        if (t == 0) *(uint32_t*)P.tlasSceneAabb = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
        if (t == 0) tlas_rearm(P, B);
        return;
    }
    Box rq = box_empty();  // this thread's contribution to the quirk reduction
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t e = (uint32_t)(t + j * kThr);
        Box rb = box_empty();
        if (e < B) {
            // read coherently, then stored back by this workgroup so that its plain re-reads (Morton
            // keys, the 512-thread refit) see its own stores whatever this XCD's L2 held
            rb = load_box_agent(P.tlasAabbs + 6 * (size_t)e);
            store_box(P.tlasAabbs + 6 * (size_t)e, rb);
            if ((e & 255u) < 128u) {
                rq.mn = min3(rq.mn, rb.mn);
                rq.mx = max3(rq.mx, rb.mx);
            }
        }
        if (Lds<kThr>::kLeafLds) store_box(s.leaf[e], rb);
    }
    const Box quirk = block_reduce(s, rq);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t e = (uint32_t)(t + j * kThr);
        uint32_t key = 0xFFFFFFFFu;
        if (e < B) {  // the leaf centre from the box just loaded (not held across the reduction)
            const Box lb = leaf_box(s, P.tlasAabbs, e);
            key = morton_of((lb.mx + lb.mn) / 2.0f, quirk);
        }
        s.a.srt.key0[e] = key;
        s.a.srt.idx0[e] = (uint16_t)e;
    }
    if (t == 0) store_box(P.tlasSceneAabb, quirk);
    sort_and_build(s, (const float*)P.tlasAabbs, (int)B, P.tlasMorton, P.tlasReorder, (Node*)P.tlasNodes,
                   tlas_words(B));
    __syncthreads();
#ifdef RTX_BVH_STAMPS
    if (t == 0) *(uint32_t*)P.tlasSceneAabb = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
    if (t == 0) tlas_rearm(P, B);
}

// kThr 1024: 8 waves/SIMD = 2 workgroups per CU; kThr 512: 4 workgroups per CU.  Either way <= 64
// VGPRs.
template <int kThr>
__global__ __launch_bounds__(kThr, 8) void k_build_bvh(BvhBuildParams P) {
    constexpr int kPer = kBatch / kThr;
    __shared__ Lds<kThr> s;
    const int t = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint32_t B = P.batchCount;
    if (b == B) {  // the extra workgroup: the TLAS, beside the batches' BLAS builds
        tlas_builder(s, P, B);
        return;
    }
    BVH_RSTAMP(0);
    BVH_STAMP(1);
    const uint32_t start = b * kBatch;
    const uint32_t cnt = (b + 1 < B) ? (uint32_t)kBatch : P.triCount - (B - 1) * kBatch;  // init.cu:129-130
    const uint32_t active = (((cnt - 1) >> 2) + 1) << 2;  // triangles of threads with tid*4 <= cnt-1
    const float* leafG = P.aabbs + 6 * (size_t)start;

    // ---- gather triangles, leaf boxes, centroids (updateGeometry.cuh:104-184); the centroids wait
    // for the batch box in `merged` (free until the refit)
    Box own = box_empty();
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t e = (uint32_t)(t + j * kThr);
        Box bx = box_empty();
        F3 center = f3(0.0f);
        if (e < active) {
            const uint32_t g = start + e;
            // kThr 1024: 64-bit row pointers, so each row's three words are provably consecutive and
            // load as one dwordx3 (60,800 tris 0.0355 -> 0.0339 ms); the 512-thread shape keeps the
            // single-dword loads, measured faster for the 958,720-triangle scene (0.0887 vs 0.0896)
            constexpr bool kRows = kThr == 1024;
            const uint32_t* ip = P.indices + 3 * (size_t)g;
            const uint32_t i0 = kRows ? ip[0] : P.indices[3 * g], i1 = kRows ? ip[1] : P.indices[3 * g + 1],
                           i2 = kRows ? ip[2] : P.indices[3 * g + 2];
            const F3 v1 = vtx_row<kRows>(P.vertices, i0), v2 = vtx_row<kRows>(P.vertices, i1),
                     v3 = vtx_row<kRows>(P.vertices, i2);
            P.triPos[4 * g + 0] = make_float4(v1.x, v1.y, v1.z, 0.0f);  // the triangle's arena record
            P.triPos[4 * g + 1] = make_float4(v2.x, v2.y, v2.z, 0.0f);
            P.triPos[4 * g + 2] = make_float4(v3.x, v3.y, v3.z, 0.0f);
            const F3 n1 = vtx_row<kRows>(P.normals, i0), n2 = vtx_row<kRows>(P.normals, i1),
                     n3 = vtx_row<kRows>(P.normals, i2);
            P.triNrm[3 * g + 0] = make_float4(n1.x, n1.y, n1.z, 0.0f);
            P.triNrm[3 * g + 1] = make_float4(n2.x, n2.y, n2.z, 0.0f);
            P.triNrm[3 * g + 2] = make_float4(n3.x, n3.y, n3.z, 0.0f);
            F3 mn = min3(v1, min3(v2, v3));
            F3 mx = max3(v1, max3(v2, v3));
            const F3 diff = max3(mx - mn, kMachineEps * mx);
            mx = mn + diff;
            bx.mn = mn;
            bx.mx = mx;
            store_box(P.aabbs + 6 * (size_t)g, bx);
            center = (v1 + v2 + v3) / 3.0f;
        }
        if (Lds<kThr>::kLeafLds) store_box(s.leaf[e], bx);
        s.merged[e][0] = center.x;
        s.merged[e][1] = center.y;
        s.merged[e][2] = center.z;
        own.mn = min3(own.mn, bx.mn);  // exact min / max: the grouping cannot change the bits
        own.mx = max3(own.mx, bx.mx);
    }

    // ---- batch box (updateGeometry.cuh:186-248) and Morton codes (:250-261)
    const Box scene = block_reduce(s, own);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const uint32_t e = (uint32_t)(t + j * kThr);
        const F3 center = f3(s.merged[e][0], s.merged[e][1], s.merged[e][2]);
        s.a.srt.key0[e] = (e < active) ? morton_of(center, scene) : 0xFFFFFFFFu;
        s.a.srt.idx0[e] = (uint16_t)e;
    }
    if (t == 0) store_box(P.batchSceneAabbs + 6 * (size_t)b, scene);
    // The TLAS leaf box of this batch (its BLAS root's merged box, box_merge of the root's two child
    // boxes), published as soon as it is known, so that the TLAS workgroup runs beside the batches'
    // sort / Karras / refit.  The refit's boxes are exact min / max merges of the leaf boxes, and
    // the BLAS's cnt leaves are the first cnt elements in sorted order: when every gathered element
    // is a leaf (cnt == active) that is the batch box above; otherwise (a last batch whose padding
    // triangles sort among the real ones) it is known after the sort (sort_and_build).
    const bool pubNow = cnt == active;
    if (pubNow && t == 0) publish_root(P, b, scene);

    Node* const nodes = (Node*)P.nodes;
    const WordCtx blasWords{kBlasBit, start, kLeafBit | kBlasBit, B * (uint32_t)kBatch + B + start, 1u};
    BVH_STAMP(2);
    sort_and_build(s, leafG, (int)cnt, P.morton + start, P.reorder + start, nodes + start, blasWords,
                   pubNow ? nullptr : &P, b);
    __syncthreads();
    BVH_STAMP(5);

#ifdef RTX_BVH_STAMPS
    if (t == 0) {
        g_stamp[6] = (uint32_t)__builtin_readcyclecounter();
        g_stamp[7] = (uint32_t)__builtin_amdgcn_s_memrealtime();
        for (int k = 0; k < 8; ++k) P.morton[start + 1016 + k] = g_stamp[k];
    }
#endif
}

// Batches that fit two 1024-thread workgroups per CU take that shape; more take the 512-thread one,
// four per CU ([render] bvhThreads forces one: tests and A/B).  p->cus is the device's CU count,
// queried once by rt_init for the context's device.
extern "C" hipError_t rtk_launch_build_bvh(const BvhBuildParams* p, hipStream_t stream) {
    const int want = (int)p->threads;
    const bool narrow = want == 512 || (want != 1024 && p->batchCount > 2 * p->cus);
    const unsigned grid = p->batchCount + 1u;  // one workgroup per batch, then the TLAS's
    if (narrow) hipLaunchKernelGGL(k_build_bvh<512>, dim3(grid), dim3(512), 0, stream, *p);
    else hipLaunchKernelGGL(k_build_bvh<1024>, dim3(grid), dim3(1024), 0, stream, *p);
    return hipGetLastError();
}
