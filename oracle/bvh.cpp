// ORACLE (test infrastructure only; see ocommon.h) — two-level LBVH build.
//
// Restates, per BLAS batch of 1024 triangles:
//   UpdateSceneGeometry<256,4>  updateGeometry.cuh:63-262
//   RadixSort<256,4>            radixSort.cuh:19-246   (== stable sort by 32-bit key)
//   BuildLBVH<256,4>            buildBVH.cuh:16-271    (Karras 2012, no tie-break)
// and for the TLAS over the BLAS roots:
//   UpdateTLAS<256,4,1024>      updateGeometry.cuh:264-364 (incl. the missing +32 merge)
// sequenced as BuildBvhLevel1/2 (bvh.cu:7-97).  The per-frame memsets of morton/tlasMorton
// to 0xFFFFFFFF (kernel.cu:279-280) are part of the contract.
#include <algorithm>
#include <thread>
#include <vector>

#include "oracle.h"
#include "ocommon.h"

namespace orc {

// MortonCode3D, updateGeometry.cuh:13-27
uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    x = (x | (x << 16)) & 0x030000FFu; x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;  x = (x | (x << 2)) & 0x09249249u;
    y = (y | (y << 16)) & 0x030000FFu; y = (y | (y << 8)) & 0x0300F00Fu;
    y = (y | (y << 4)) & 0x030C30C3u;  y = (y | (y << 2)) & 0x09249249u;
    z = (z | (z << 16)) & 0x030000FFu; z = (z | (z << 8)) & 0x0300F00Fu;
    z = (z | (z << 4)) & 0x030C30C3u;  z = (z | (z << 2)) & 0x09249249u;
    return x | (y << 1) | (z << 2);
}

static uint32_t morton_of(F3 c, const AABB& scene) {
    F3 u = (c - scene.min) / (scene.max - scene.min);
    return morton3(sat_u32(u.x * 1023.0f), sat_u32(u.y * 1023.0f), sat_u32(u.z * 1023.0f));
}

static int clz32(uint32_t v) { return v == 0 ? 32 : __builtin_clz(v); }

// LCP, buildBVH.cuh:8-14
static int lcp(const uint32_t* m, int n, uint32_t m0, int j) {
    if (j < 0 || j >= n) return 0;
    return clz32(m0 ^ m[j]);
}

// Karras topology + bottom-up boxes for one batch (buildBVH.cuh:60-267).  Boxes are a pure
// function of the tree, so the refit is evaluated in post-order instead of by racing threads.
static void build_lbvh(Node* nodes, const AABB* leafBoxes, const uint32_t* morton, const uint32_t* reorder,
                       int n) {
    if (n == 1) {  // buildBVH.cuh:31-38 (written to the batch's own node 0)
        AABB zero = {f3(0.0f), f3(0.0f)};
        node_set_boxes(nodes[0], leafBoxes[0], zero);
        nodes[0].idxLeft = 0; nodes[0].idxRight = 0;
        nodes[0].isLeftLeaf = 1; nodes[0].isRightLeaf = 1;
        return;
    }
    for (int i = 0; i < n - 1; ++i) {
        uint32_t m0 = morton[i];
        int dl = lcp(morton, n, m0, i - 1);
        int dr = lcp(morton, n, m0, i + 1);
        int d = (dr - dl) >= 0 ? 1 : -1;
        int deltaMin = lcp(morton, n, m0, i - d);
        int lmax = 2;
        while (lcp(morton, n, m0, i + lmax * d) > deltaMin) lmax *= 2;
        int l = 0;
        for (int t = lmax / 2; t >= 1; t /= 2)
            if (lcp(morton, n, m0, i + (l + t) * d) > deltaMin) l += t;
        int j = i + l * d;
        int deltaNode = lcp(morton, n, m0, j);
        // split search; the reference loops while ceil(l/div) >= 1 (only int overflow ends
        // it) — the extra t == 1 probes are no-ops, so stop after the first t == 1.
        int s = 0;
        int div = 2;
        while (true) {
            int t = (l + div - 1) / div;
            if (lcp(morton, n, m0, i + (s + t) * d) > deltaNode) s += t;
            if (t <= 1) break;
            div *= 2;
        }
        int gamma = i + s * d + std::min(d, 0);
        Node& nd = nodes[i];
        if (std::min(i, j) == gamma) { nd.isLeftLeaf = 1; nd.idxLeft = reorder[gamma]; }
        else { nd.isLeftLeaf = 0; nd.idxLeft = (uint32_t)gamma; }
        if (std::max(i, j) == gamma + 1) { nd.isRightLeaf = 1; nd.idxRight = reorder[gamma + 1]; }
        else { nd.isRightLeaf = 0; nd.idxRight = (uint32_t)(gamma + 1); }
    }
    // post-order refit from the root (node 0)
    std::vector<int> stack;
    std::vector<uint8_t> state(n - 1, 0);
    stack.push_back(0);
    while (!stack.empty()) {
        int v = stack.back();
        Node& nd = nodes[v];
        if (state[v] == 0) {
            state[v] = 1;
            if (!nd.isRightLeaf) stack.push_back((int)nd.idxRight);
            if (!nd.isLeftLeaf) stack.push_back((int)nd.idxLeft);
            continue;
        }
        stack.pop_back();
        AABB l = nd.isLeftLeaf ? leafBoxes[nd.idxLeft] : node_merged(nodes[nd.idxLeft]);
        AABB r = nd.isRightLeaf ? leafBoxes[nd.idxRight] : node_merged(nodes[nd.idxRight]);
        node_set_boxes(nd, l, r);
    }
}

static void stable_sort_1024(uint32_t* keys, uint32_t* reorder) {
    std::vector<uint32_t> idx(1024);
    for (uint32_t i = 0; i < 1024; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
    std::vector<uint32_t> sorted(1024);
    for (int i = 0; i < 1024; ++i) { sorted[i] = keys[idx[i]]; reorder[i] = idx[i]; }
    memcpy(keys, sorted.data(), 1024 * 4);
}

}  // namespace orc

using namespace orc;

extern "C" int orc_build_bvh_mt(const OrcBvhIO* io, int threads);

extern "C" int orc_build_bvh(const OrcBvhIO* io) { return orc_build_bvh_mt(io, 1); }

// threads > 1: the BLAS batches (independent blocks in the reference) spread over host threads;
// the result does not depend on the split
extern "C" int orc_build_bvh_mt(const OrcBvhIO* io, int threads) {
    const uint32_t N = io->triCount, NP = io->triCountPadded;
    if (N < 2 || NP < N || NP % 4 != 0) return -1;
    const uint32_t B = (N + 1023) / 1024;
    if (B >= 1024) return -2;
    const F3* V = (const F3*)io->vertices;
    const F3* NRM = (const F3*)io->normals;
    AABB* aabbs = (AABB*)io->aabbs;  // [NP]
    Node* nodes = (Node*)io->nodes;  // [NP]
    // per-frame memsets
    for (uint32_t k = 0; k < B * 1024; ++k) io->mortonUnsorted[k] = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < 1024; ++k) io->tlasMortonUnsorted[k] = 0xFFFFFFFFu;

    // ---------------- BLAS (one block per batch)
    auto blas = [&](uint32_t b) {
        const uint32_t start = b * 1024;
        const uint32_t cnt = (b + 1 < B) ? 1024u : N - (B - 1) * 1024u;  // init.cu:129-130
        const uint32_t active = (cnt - 1) / 4 + 1;                       // threads with tid*4 <= cnt-1
        AABB scene = aabb_empty();
        std::vector<F3> centers(active * 4);
        for (uint32_t t = 0; t < active * 4; ++t) {
            const uint32_t g = start + t;
            const uint32_t i0 = io->indices[3 * g], i1 = io->indices[3 * g + 1], i2 = io->indices[3 * g + 2];
            F3 v1 = V[i0], v2 = V[i1], v3 = V[i2];
            float* tri = io->triangles + (size_t)g * 18;
            tri[0] = v1.x; tri[1] = v1.y; tri[2] = v1.z;
            tri[3] = v2.x; tri[4] = v2.y; tri[5] = v2.z;
            tri[6] = v3.x; tri[7] = v3.y; tri[8] = v3.z;
            F3 n1 = NRM ? NRM[i0] : f3(0.0f), n2 = NRM ? NRM[i1] : f3(0.0f), n3 = NRM ? NRM[i2] : f3(0.0f);
            tri[9] = n1.x; tri[10] = n1.y; tri[11] = n1.z;
            tri[12] = n2.x; tri[13] = n2.y; tri[14] = n2.z;
            tri[15] = n3.x; tri[16] = n3.y; tri[17] = n3.z;
            F3 mn = min3(v1, min3(v2, v3));
            F3 mx = max3(v1, max3(v2, v3));
            F3 diff = max3(mx - mn, kMachineEps * mx);  // updateGeometry.cuh:176
            mx = mn + diff;
            AABB bx = {mn, mx};
            aabbs[g] = bx;
            centers[t] = (v1 + v2 + v3) / 3.0f;
            scene.min = min3(scene.min, bx.min);
            scene.max = max3(scene.max, bx.max);
        }
        for (uint32_t t = 0; t < active * 4; ++t) io->mortonUnsorted[start + t] = morton_of(centers[t], scene);
        memcpy(io->mortonSorted + start, io->mortonUnsorted + start, 1024 * 4);
        stable_sort_1024(io->mortonSorted + start, io->reorderIdx + start);
        build_lbvh(nodes + start, aabbs + start, io->mortonSorted + start, io->reorderIdx + start, (int)cnt);
        io->batchSceneAabbs[6 * b + 0] = scene.min.x; io->batchSceneAabbs[6 * b + 1] = scene.min.y;
        io->batchSceneAabbs[6 * b + 2] = scene.min.z; io->batchSceneAabbs[6 * b + 3] = scene.max.x;
        io->batchSceneAabbs[6 * b + 4] = scene.max.y; io->batchSceneAabbs[6 * b + 5] = scene.max.z;
    };
    if (threads <= 1 || B < 2) {
        for (uint32_t b = 0; b < B; ++b) blas(b);
    } else {
        std::vector<std::thread> pool;
        const uint32_t T = (uint32_t)threads < B ? (uint32_t)threads : B;
        for (uint32_t t = 0; t < T; ++t)
            pool.emplace_back([&, t] {
                for (uint32_t b = t; b < B; b += T) blas(b);
            });
        for (auto& th : pool) th.join();
    }

    // ---------------- TLAS (one block)
    AABB* taabbs = (AABB*)io->tlasAabbs;
    std::vector<F3> centers(B);
    AABB slot[256];
    for (int s = 0; s < 256; ++s) slot[s] = aabb_empty();
    for (uint32_t b = 0; b < B; ++b) {
        AABB bx = node_merged(nodes[b * 1024]);
        taabbs[b] = bx;
        centers[b] = (bx.max + bx.min) / 2.0f;
        AABB& sl = slot[b / 4];
        if (b % 4 == 0) sl = bx;
        else { sl.min = min3(sl.min, bx.min); sl.max = max3(sl.max, bx.max); }
    }
    // strides 128, 64 then a 32-lane shuffle reduce: no +32 merge (updateGeometry.cuh:317-336)
    AABB quirk = aabb_empty();
    for (int s = 0; s < 256; ++s) {
        if ((s & 63) >= 32) continue;
        quirk.min = min3(quirk.min, slot[s].min);
        quirk.max = max3(quirk.max, slot[s].max);
    }
    io->tlasSceneAabb[0] = quirk.min.x; io->tlasSceneAabb[1] = quirk.min.y; io->tlasSceneAabb[2] = quirk.min.z;
    io->tlasSceneAabb[3] = quirk.max.x; io->tlasSceneAabb[4] = quirk.max.y; io->tlasSceneAabb[5] = quirk.max.z;
    for (uint32_t b = 0; b < B; ++b) io->tlasMortonUnsorted[b] = morton_of(centers[b], quirk);
    memcpy(io->tlasMortonSorted, io->tlasMortonUnsorted, 1024 * 4);
    stable_sort_1024(io->tlasMortonSorted, io->tlasReorderIdx);
    build_lbvh((Node*)io->tlasNodes, taabbs, io->tlasMortonSorted, io->tlasReorderIdx, (int)B);
    return (int)B;
}

extern "C" uint32_t orc_morton3(uint32_t x, uint32_t y, uint32_t z) { return morton3(x, y, z); }
