// scene_gen.cpp — procedural default scene, host C++ (see scene_gen.h for the reference map).
//
// Every floating-point expression keeps the reference's operand order; the file is built
// with -ffp-contract=off so each operation rounds once, as MSVC /fp:precise does.
#include "scene_gen.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>

#include "rtmath.h"

namespace rtscene {
namespace {

// ------------------------------------------------------------------ Perlin (perlin.h:16-78)
// Ken Perlin's reference permutation.
const int kPermutation[256] = {
    151, 160, 137, 91,  90,  15,  131, 13,  201, 95,  96,  53,  194, 233, 7,   225, 140, 36,  103, 30,  69,  142,
    8,   99,  37,  240, 21,  10,  23,  190, 6,   148, 247, 120, 234, 75,  0,   26,  197, 62,  94,  252, 219, 203,
    117, 35,  11,  32,  57,  177, 33,  88,  237, 149, 56,  87,  174, 20,  125, 136, 171, 168, 68,  175, 74,  165,
    71,  134, 139, 48,  27,  166, 77,  146, 158, 231, 83,  111, 229, 122, 60,  211, 133, 230, 220, 105, 92,  41,
    55,  46,  245, 40,  244, 102, 143, 54,  65,  25,  63,  161, 1,   216, 80,  73,  209, 76,  132, 187, 208, 89,
    18,  169, 200, 196, 135, 130, 116, 188, 159, 86,  164, 100, 109, 198, 173, 186, 3,   64,  52,  217, 226, 250,
    124, 123, 5,   202, 38,  147, 118, 126, 255, 82,  85,  212, 207, 206, 59,  227, 47,  16,  58,  17,  182, 189,
    28,  42,  223, 183, 170, 213, 119, 248, 152, 2,   44,  154, 163, 70,  221, 153, 101, 155, 167, 43,  172, 9,
    129, 22,  39,  253, 19,  98,  108, 110, 79,  113, 224, 232, 178, 185, 112, 104, 218, 246, 97,  228, 251, 34,
    242, 193, 238, 210, 144, 12,  191, 179, 162, 241, 81,  51,  145, 235, 249, 14,  239, 107, 49,  192, 214, 31,
    181, 199, 106, 157, 184, 84,  204, 176, 115, 121, 50,  45,  127, 4,   150, 254, 138, 236, 205, 93,  222, 114,
    67,  29,  24,  72,  243, 141, 128, 195, 78,  66,  215, 61,  156, 180};

struct Perlin {
    int p[512];
    Perlin() {
        for (int i = 0; i < 512; ++i) p[i] = kPermutation[i & 255];
    }
    static float fade(float t) { return t * t * t * (t * (t * 6 - 15) + 10); }
    static float lerp(float t, float a, float b) { return a + t * (b - a); }
    static float grad(int hash, float x, float y, float z) {
        int h = hash & 15;
        float u = h < 8 ? x : y;
        float v = h < 4 ? y : (h == 12 || h == 14) ? x : z;
        return ((h & 1) == 0 ? u : -u) + ((h & 2) == 0 ? v : -v);
    }
    float noise3D(float x, float y, float z) const {
        int X = (int)floorf(x) & 255;
        int Y = (int)floorf(y) & 255;
        int Z = (int)floorf(z) & 255;
        x -= floorf(x);
        y -= floorf(y);
        z -= floorf(z);
        float u = fade(x), v = fade(y), w = fade(z);
        int A = p[X] + Y, AA = p[A] + Z, AB = p[A + 1] + Z;
        int B = p[X + 1] + Y, BA = p[B] + Z, BB = p[B + 1] + Z;
        float res = lerp(w,
                         lerp(v, lerp(u, grad(p[AA], x, y, z), grad(p[BA], x - 1, y, z)),
                              lerp(u, grad(p[AB], x, y - 1, z), grad(p[BB], x - 1, y - 1, z))),
                         lerp(v, lerp(u, grad(p[AA + 1], x, y, z - 1), grad(p[BA + 1], x - 1, y, z - 1)),
                              lerp(u, grad(p[AB + 1], x, y - 1, z - 1), grad(p[BB + 1], x - 1, y - 1, z - 1))));
        return (res + 1.0f) / 2.0f;
    }
};

// ------------------------------------------------------------------ voxels (terrain.cpp/.h)
const int kBlockDim = 16, kBlockDimY = 16;
const uint32_t kBorder = 0xFFFF;

struct Voxels {
    int chunkDim, mapDim, mapDimY;
    std::vector<uint8_t> solid;  // [y][x][z] over the whole map
    uint32_t at(int x, int y, int z) const {
        if (x < 0 || z < 0 || y < 0 || x >= mapDim || z >= mapDim || y >= mapDimY) return kBorder;
        return solid[((size_t)y * mapDim + x) * mapDim + z];
    }
};

void generate_voxels(int chunkDim, Voxels& vx) {
    Perlin perlin;
    const float noiseScale = 2.0f, baseY = kBlockDimY / 2.0f, scaleY = kBlockDimY / 2.0f;
    vx.chunkDim = chunkDim;
    vx.mapDim = chunkDim * kBlockDim;
    vx.mapDimY = kBlockDimY;
    vx.solid.assign((size_t)vx.mapDim * vx.mapDim * vx.mapDimY, 0);
    for (int cx = 0; cx < chunkDim; ++cx)
        for (int cz = 0; cz < chunkDim; ++cz)
            for (int i = 0; i < kBlockDim; ++i)
                for (int j = 0; j < kBlockDim; ++j) {
                    float nx = (float)(cx * kBlockDim + i);
                    float nz = (float)(cz * kBlockDim + j);
                    nx *= noiseScale / (float)kBlockDim;
                    nz *= noiseScale / (float)kBlockDim;
                    float noiseVal = perlin.noise3D(nx, nz, 0.5f);
                    noiseVal -= 0.5f;
                    noiseVal *= 1.5f;
                    noiseVal = baseY + noiseVal * scaleY;
                    int gx = cx * kBlockDim + i, gz = cz * kBlockDim + j;
                    for (int k = 0; k < kBlockDimY; ++k) {
                        if ((float)(unsigned)k < noiseVal)
                            vx.solid[((size_t)k * vx.mapDim + gx) * vx.mapDim + gz] = 1;
                        else
                            break;
                    }
                }
}

// 8 corner samples of the cell at (x, y, z): bit0 = -x, bit1 = -y, bit2 = -z
// (GetNeighborBlockAt2, terrain.cpp:165-295; out-of-map cells read as the border value).
void cell_corners(const Voxels& vx, int x, int y, int z, uint32_t out[8]) {
    for (int c = 0; c < 8; ++c) out[c] = vx.at(x - (c & 1), y - ((c >> 1) & 1), z - ((c >> 2) & 1));
}

// IsSolid, marchingCubes.cpp:42-92: border corners inherit the solidity of the nearest
// in-map corner along the walls they sit on.
bool corner_solid(int i, const uint32_t b[8]) {
    if (b[i] == 0) return false;
    if (b[i] != kBorder) return true;
    int nX = i ^ 1, nY = i ^ 2, nZ = i ^ 4;
    int nXY = nX ^ 2, nXZ = nX ^ 4, nYZ = nY ^ 4;
    int opp = (~i) & 7;
    bool bX = b[nX] == kBorder, bY = b[nY] == kBorder, bZ = b[nZ] == kBorder;
    bool bXY = b[nXY] == kBorder, bXZ = b[nXZ] == kBorder, bYZ = b[nYZ] == kBorder;
    bool wallX = bY && bZ && bYZ;
    bool wallY = bX && bZ && bXZ;
    bool wallZ = bX && bY && bXY;
    if (wallX && wallY && wallZ) return b[opp] != 0;
    if (wallY && wallZ) return b[nYZ] != 0;
    if (wallX && wallZ) return b[nXZ] != 0;
    if (wallX && wallY) return b[nXY] != 0;
    if (wallZ) return b[nZ] != 0;
    if (wallY) return b[nY] != 0;
    if (wallX) return b[nX] != 0;
    return false;  // unreachable: a border corner always lies on at least one wall
}

// ------------------------------------------------------------------ marching-cube tiles
struct P3 { float x, y, z; };
using Soup = std::vector<P3>;  // 3 points per triangle

enum Axis { kX, kY, kZ };

P3 rotate_point(const P3& v, Axis axis, int angle) {
    int c, s;
    if (angle == 90) { c = 0; s = 1; }
    else if (angle == -90) { c = 0; s = -1; }
    else if (angle == 180) { c = -1; s = 0; }
    else { c = 1; s = 0; }
    // PointRotate, marchingCubes.cpp:115-127 (int * float products, float sums)
    if (axis == kY) return {c * v.x + s * v.z, v.y, -s * v.x + c * v.z};
    if (axis == kX) return {v.x, c * v.y - s * v.z, s * v.y + c * v.z};
    return {c * v.x - s * v.y, s * v.x + c * v.y, v.z};
}

uint32_t points_to_idx(const std::vector<P3>& pts) {
    uint32_t r = 0;
    for (const P3& p : pts) {
        uint32_t q = (signbit(p.x) ? 1u : 0u) + (signbit(p.y) ? 2u : 0u) + (signbit(p.z) ? 4u : 0u);
        r += 1u << q;
    }
    return r;
}

uint32_t flip_bits8(uint32_t n) { return ~n & 0xFFu; }

void flip_winding(Soup& out, const Soup& in) {
    Soup t(in.size());
    for (size_t k = 0; k + 2 < in.size() + 0 && k < in.size(); k += 3) {
        t[k] = in[k];
        t[k + 1] = in[k + 2];
        t[k + 2] = in[k + 1];
    }
    out.swap(t);
}

struct CubeDef {
    int tile;            // 1..15 -> "<tile>.obj"
    int npts;
    float pts[6][3];
    bool reversible;
};

// The 15 canonical configurations, marchingCubes.cpp:297-533.
const CubeDef kCubes[15] = {
    {1, 1, {{1, 1, 1}}, true},
    {2, 2, {{1, 1, 1}, {1, 1, -1}}, true},
    {3, 2, {{1, 1, 1}, {1, -1, -1}}, false},
    {4, 3, {{1, 1, 1}, {1, -1, 1}, {1, 1, -1}}, true},
    {5, 4, {{1, 1, 1}, {1, 1, -1}, {-1, 1, 1}, {-1, 1, -1}}, false},
    {6, 4, {{1, 1, 1}, {1, -1, 1}, {1, 1, -1}, {-1, -1, -1}}, false},
    {7, 4, {{1, 1, 1}, {1, -1, -1}, {-1, 1, -1}, {-1, -1, 1}}, false},
    {8, 4, {{1, 1, 1}, {1, -1, 1}, {1, 1, -1}, {-1, 1, 1}}, false},
    {9, 4, {{1, 1, 1}, {-1, 1, 1}, {-1, 1, -1}, {-1, -1, -1}}, false},
    {10, 2, {{1, 1, 1}, {-1, -1, -1}}, true},
    {11, 3, {{1, 1, 1}, {-1, -1, 1}, {-1, -1, -1}}, false},
    {12, 3, {{1, 1, 1}, {-1, 1, -1}, {-1, -1, 1}}, false},
    {13, 4, {{1, 1, 1}, {1, -1, 1}, {-1, 1, -1}, {-1, -1, -1}}, false},
    {14, 4, {{1, 1, 1}, {1, -1, 1}, {1, -1, -1}, {-1, -1, -1}}, false},
    {15, 6, {{1, 1, -1}, {1, -1, 1}, {-1, 1, 1}, {-1, 1, -1}, {-1, -1, 1}, {-1, -1, -1}}, false},
};

struct Trans { Axis axis; int angle; int basedOn; };
// transList, marchingCubes.cpp:270-295 (entry 0 is the identity)
const Trans kTrans[24] = {
    {kX, 0, 0},   {kX, 90, 0},  {kX, 180, 0}, {kX, -90, 0}, {kY, 90, 0},  {kY, 90, 1},
    {kY, 90, 2},  {kY, 90, 3},  {kY, 180, 0}, {kY, 180, 1}, {kY, 180, 2}, {kY, 180, 3},
    {kY, -90, 0}, {kY, -90, 1}, {kY, -90, 2}, {kY, -90, 3}, {kZ, 90, 0},  {kZ, 90, 1},
    {kZ, 90, 2},  {kZ, 90, 3},  {kZ, -90, 0}, {kZ, -90, 1}, {kZ, -90, 2}, {kZ, -90, 3},
};

void build_case_meshes(const std::vector<std::vector<float>>& tiles, std::vector<Soup>& meshes,
                       uint32_t& appendedToNonEmpty) {
    meshes.assign(256, Soup());
    appendedToNonEmpty = 0;
    for (const CubeDef& cube : kCubes) {
        std::vector<std::vector<P3>> points(24);
        std::vector<uint32_t> meshIdx(24, 0);
        for (int k = 0; k < cube.npts; ++k) points[0].push_back({cube.pts[k][0], cube.pts[k][1], cube.pts[k][2]});
        meshIdx[0] = points_to_idx(points[0]);
        // LoadScene appends (fileUtils.cu:16-57), then the whole mesh is scaled by 0.5
        Soup& base = meshes[meshIdx[0]];
        if (!base.empty()) ++appendedToNonEmpty;
        const std::vector<float>& t = tiles[cube.tile - 1];
        for (size_t k = 0; k + 2 < t.size(); k += 3) base.push_back({t[k], t[k + 1], t[k + 2]});
        for (P3& p : base) { p.x = p.x * 0.5f; p.y = p.y * 0.5f; p.z = p.z * 0.5f; }
        if (cube.reversible) flip_winding(meshes[flip_bits8(meshIdx[0])], meshes[meshIdx[0]]);
        for (int i = 1; i < 24; ++i) {
            const Trans& tr = kTrans[i];
            for (const P3& p : points[tr.basedOn]) points[i].push_back(rotate_point(p, tr.axis, tr.angle));
            meshIdx[i] = points_to_idx(points[i]);
            uint32_t src = meshIdx[tr.basedOn], dst = meshIdx[i];
            if (meshes[dst].empty()) {
                Soup r(meshes[src].size());
                for (size_t k = 0; k < r.size(); ++k) r[k] = rotate_point(meshes[src][k], tr.axis, tr.angle);
                meshes[dst].swap(r);
            }
            src = meshIdx[i];
            dst = flip_bits8(meshIdx[i]);
            if (cube.reversible && meshes[dst].empty()) flip_winding(meshes[dst], meshes[src]);
        }
    }
}

// ------------------------------------------------------------------ vertex merge
// VertexMerger, marchingCubes.cpp:572-674: first match within 1e-3 over the 27 neighbour
// bins, searched x-major, then y, then z, each bin in insertion order.
struct Merger {
    P3 bmin, bmax;
    float maxDist;
    int dimX, dimY, dimZ;
    float binSize;
    std::vector<std::vector<uint32_t>> bins;
    std::vector<P3>* verts;
    std::vector<uint32_t>* idx;

    void init(uint32_t vertexCount) {
        float ex = bmax.x - bmin.x, ey = bmax.y - bmin.y, ez = bmax.z - bmin.z;
        float arg = (float)vertexCount * ex * ex / ey / ez;
        float dx = rt_powf(arg, 1.0f / 3.0f);
        float dy = dx / ex * ey;
        float dz = dx / ex * ez;
        dimX = (int)dx + 1;
        dimY = (int)dy + 1;
        dimZ = (int)dz + 1;
        binSize = ex / (float)dimX;
        bins.assign((size_t)dimX * dimY * dimZ, {});
    }
    static uint32_t to_bin(float v) {
        // (uint) of a non-negative float; saturate like a well-defined conversion
        if (!(v > 0.0f)) return 0;
        if (v >= 4294967296.0f) return 0xFFFFFFFFu;
        return (uint32_t)v;
    }
    void bin_of(const P3& v, uint32_t& bx, uint32_t& by, uint32_t& bz) const {
        bx = to_bin((v.x - bmin.x) / binSize);
        by = to_bin((v.y - bmin.y) / binSize);
        bz = to_bin((v.z - bmin.z) / binSize);
        bx = std::min(bx, (uint32_t)(dimX - 1));
        by = std::min(by, (uint32_t)(dimY - 1));
        bz = std::min(bz, (uint32_t)(dimZ - 1));
    }
    void process(const P3& v) {
        uint32_t bx, by, bz;
        bin_of(v, bx, by, bz);
        float lim = maxDist * maxDist;
        for (uint32_t i = bx == 0 ? bx : bx - 1; i <= (bx == (uint32_t)dimX - 1 ? bx : bx + 1); ++i)
            for (uint32_t j = by == 0 ? by : by - 1; j <= (by == (uint32_t)dimY - 1 ? by : by + 1); ++j)
                for (uint32_t k = bz == 0 ? bz : bz - 1; k <= (bz == (uint32_t)dimZ - 1 ? bz : bz + 1); ++k)
                    for (uint32_t id : bins[((size_t)i * dimY + j) * dimZ + k]) {
                        const P3& w = (*verts)[id];
                        float d = (v.x - w.x) * (v.x - w.x) + (v.y - w.y) * (v.y - w.y) + (v.z - w.z) * (v.z - w.z);
                        if (d <= lim) { idx->push_back(id); return; }
                    }
        uint32_t id = (uint32_t)verts->size();
        idx->push_back(id);
        verts->push_back(v);
        bins[((size_t)bx * dimY + by) * dimZ + bz].push_back(id);
    }
};

}  // namespace

bool load_tiles(const std::string& path, std::vector<std::vector<float>>& tiles, std::string& err) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open tile file " + path; return false; }
    uint32_t n = 0;
    bool ok = fread(&n, 4, 1, f) == 1 && n == 15;
    tiles.clear();
    for (uint32_t t = 0; ok && t < n; ++t) {
        uint32_t nt = 0;
        ok = fread(&nt, 4, 1, f) == 1 && nt < 100000;
        if (!ok) break;
        std::vector<float> v((size_t)nt * 9);
        ok = fread(v.data(), 4, v.size(), f) == v.size();
        tiles.push_back(std::move(v));
    }
    fclose(f);
    if (!ok) err = "malformed tile file " + path;
    return ok;
}

bool generate(int chunkDim, const std::vector<std::vector<float>>& tiles, SceneMesh& out, std::string& err) {
    if (chunkDim < 1 || chunkDim > 8) { err = "chunkDim out of range [1,8]"; return false; }
    if (tiles.size() != 15) { err = "need 15 tiles"; return false; }
    Voxels vx;
    generate_voxels(chunkDim, vx);
    std::vector<Soup> meshes;
    build_case_meshes(tiles, meshes, out.tilesAppendedToNonEmpty);

    // corners in VoxelToMesh order: x (i), then z (j), then y (k), translated by (i, k, j)
    std::vector<P3> corners;
    P3 bmax = {-3.402823466e+38f, -3.402823466e+38f, -3.402823466e+38f};
    P3 bmin = {3.402823466e+38f, 3.402823466e+38f, 3.402823466e+38f};
    for (int i = 0; i < vx.mapDim + 1; ++i)
        for (int j = 0; j < vx.mapDim + 1; ++j)
            for (int k = 0; k < vx.mapDimY + 1; ++k) {
                uint32_t b[8];
                cell_corners(vx, i, k, j, b);
                uint32_t id = 0;
                for (int c = 0; c < 8; ++c) id += (corner_solid(c, b) ? 1u : 0u) << c;
                const float tx = (float)(unsigned)i, ty = (float)(unsigned)k, tz = (float)(unsigned)j;
                for (const P3& p : meshes[id]) {
                    P3 q = {p.x + tx, p.y + ty, p.z + tz};
                    corners.push_back(q);
                    bmax = {bmax.x > q.x ? bmax.x : q.x, bmax.y > q.y ? bmax.y : q.y, bmax.z > q.z ? bmax.z : q.z};
                    bmin = {bmin.x < q.x ? bmin.x : q.x, bmin.y < q.y ? bmin.y : q.y, bmin.z < q.z ? bmin.z : q.z};
                }
            }
    if (corners.empty()) { err = "empty scene"; return false; }

    std::vector<P3> verts;
    std::vector<uint32_t> idx;
    idx.reserve(corners.size());
    Merger m;
    m.bmin = bmin;
    m.bmax = bmax;
    m.maxDist = 0.001f;
    m.verts = &verts;
    m.idx = &idx;
    m.init((uint32_t)corners.size());
    for (const P3& c : corners) m.process(c);

    out.cornerCount = (uint32_t)corners.size();
    out.triCount = (uint32_t)(idx.size() / 3);
    out.triCountPadded = (out.triCount + 3u) & ~3u;
    idx.resize((size_t)out.triCountPadded * 3, 0u);  // padding triangles repeat index 0
    out.indices.swap(idx);
    out.vertices.resize(verts.size() * 3);
    for (size_t v = 0; v < verts.size(); ++v) {
        out.vertices[3 * v] = verts[v].x;
        out.vertices[3 * v + 1] = verts[v].y;
        out.vertices[3 * v + 2] = verts[v].z;
    }
    return true;
}

// Perlin::noise3D (perlin.h:50-78) of the terrain generator, for the reference-pinned tests
float noise3d(float x, float y, float z) {
    static const Perlin perlin;
    return perlin.noise3D(x, y, z);
}

}  // namespace rtscene
