// ORACLE REFERENCE BUILD (test infrastructure only): runs the reference's own Perlin class,
// /root/reference/src/perlin.h, compiled here with plain g++ from where it lies (no stand-in
// headers: the file needs only <vector>, <cmath>, <random>, <algorithm>, <numeric>).
//
// Writes binary float32 records to stdout:
//   [16384][3] inputs + [16384] noise3D values: the lattice Chunk::Generate samples for
//   VoxelsGenerator::kChunkDim = 8 (terrain.cpp:5-17: nx = (float)(x*kBlockDim + i) *
//   (noiseScale / (float)kBlockDim), noise3D(nx, nz, 0.5f)); kChunkDim 1 and 4 are its
//   [16][16] and [64][64] corners;
//   [4096][3] inputs + [4096] values at scattered points in [-300, 300)^3 (negative and
//   wrapped lattice cells), from a fixed integer LCG.
// Used by tests/golden/make_ref_fixtures.py; outputs go to oracle/_ref/ only.
#include <stdint.h>
#include <stdio.h>

#include <vector>

#include "perlin.h"

int main() {
    Perlin perlin;  // the reference permutation (perlin.h:13-30)
    const unsigned kBlockDim = 16, kChunkDim = 8;
    const float noiseScale = 2.0f;  // VoxelsGenerator::noiseScale (terrain.h:38)
    std::vector<float> rec;
    for (unsigned x = 0; x < kChunkDim; ++x)
        for (unsigned i = 0; i < kBlockDim; ++i)
            for (unsigned z = 0; z < kChunkDim; ++z)
                for (unsigned j = 0; j < kBlockDim; ++j) {
                    float nx = (float)(x * kBlockDim + i);
                    float nz = (float)(z * kBlockDim + j);
                    nx *= noiseScale / (float)kBlockDim;
                    nz *= noiseScale / (float)kBlockDim;
                    rec.push_back(nx);
                    rec.push_back(nz);
                    rec.push_back(0.5f);
                }
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (int k = 0; k < 4096 * 3; ++k) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t r = (uint32_t)(s >> 40);  // 24 bits
        rec.push_back((float)((double)r / 16777216.0 * 600.0 - 300.0));
    }
    const size_t n = rec.size() / 3;
    std::vector<float> out(n);
    for (size_t k = 0; k < n; ++k) out[k] = perlin.noise3D(rec[3 * k], rec[3 * k + 1], rec[3 * k + 2]);
    fwrite(rec.data(), 4, rec.size(), stdout);
    fwrite(out.data(), 4, out.size(), stdout);
    return 0;
}
