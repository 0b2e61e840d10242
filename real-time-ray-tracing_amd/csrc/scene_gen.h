// scene_gen.h — host-side procedural default scene (the hot path's input).
//
// Restates RayTracer::init's scene construction (init.cu:78-130): Perlin voxel terrain
// (terrain.cpp:5-58, perlin.h:50-78), marching-cube tiling with the 15 round-cube tiles
// (marchingCubes.cpp:216-537), per-cell translation (marchingCubes.cpp:704-750) and the
// 1e-3 vertex merge (marchingCubes.cpp:572-674, 751-757), then padding to a multiple of 4
// triangles with index 0 (init.cu:103-115).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace rtscene {

struct SceneMesh {
    std::vector<float> vertices;    // xyz per vertex
    std::vector<uint32_t> indices;  // 3 per triangle, padded to a multiple of 4 triangles
    uint32_t triCount = 0;          // real triangles (before padding)
    uint32_t triCountPadded = 0;    // multiple of 4 (KernalBatchSize)
    // diagnostics
    uint32_t cornerCount = 0;       // triangle corners fed to the vertex merger
    uint32_t tilesAppendedToNonEmpty = 0;
};

// Loads the tile soups written by tools/extract_reference_data.py (roundcubes_l2.bin).
bool load_tiles(const std::string& path, std::vector<std::vector<float>>& tiles, std::string& err);

// chunkDim = VoxelsGenerator::kChunkDim (1 for the default scene, 4 for the ~1M variant).
bool generate(int chunkDim, const std::vector<std::vector<float>>& tiles, SceneMesh& out, std::string& err);

// Perlin::noise3D (perlin.h:50-78) with the reference permutation: the terrain heights' source
float noise3d(float x, float y, float z);

}  // namespace rtscene
