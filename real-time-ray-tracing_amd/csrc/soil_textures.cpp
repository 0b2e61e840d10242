// soil_textures.cpp — the synthetic soil texture pair (an INPUT, see soil_textures.h).  Linked by
// the product (level 0 uploaded, mips built on the device) and by the oracle (its own mips).
#include "soil_textures.h"

namespace rtscene {

namespace {
uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) { return mix32(a * 0x9E3779B1U ^ mix32(b * 0x85EBCA77U ^ mix32(c + 0x632BE5ABU))); }
// [0, 1) with 16-bit resolution
double unit(uint32_t h) { return (double)(h >> 16) / 65536.0; }
uint16_t to16(double v) {
    if (v < 0.0) v = 0.0;
    if (v > 1.0) v = 1.0;
    return (uint16_t)(v * 65535.0 + 0.5);
}
}  // namespace

void make_textures(TexturePair& t) {
    size_t total = 0;
    for (int l = 0; l < TexturePair::kLevels; ++l) {
        t.size[l] = 1024 >> l;
        t.offset[l] = total;
        total += (size_t)t.size[l] * t.size[l];
    }
    t.albedoAo.assign(total * 4, 0);
    t.normalRough.assign(total * 4, 0);
    const double base[3] = {0.42, 0.33, 0.24};  // dry soil, pre-gamma (the shader applies ^2.2)
    for (uint32_t y = 0; y < 1024; ++y)
        for (uint32_t x = 0; x < 1024; ++x) {
            const size_t p = ((size_t)y * 1024 + x) * 4;
            const double cell = unit(hash3(x >> 5, y >> 5, 7u));     // 32-texel pebbles
            const double grain = unit(hash3(x, y, 11u));             // per-texel grain
            for (int c = 0; c < 3; ++c) {
                const double tint = unit(hash3(x >> 5, y >> 5, 20u + (uint32_t)c));
                t.albedoAo[p + c] = to16(base[c] * (0.75 + 0.5 * cell) * (0.9 + 0.2 * grain) * (0.95 + 0.1 * tint));
            }
            t.albedoAo[p + 3] = to16(0.8 + 0.2 * unit(hash3(x >> 3, y >> 3, 31u)));
            const double nx = unit(hash3(x >> 2, y >> 2, 41u)) - 0.5, ny = unit(hash3(x >> 2, y >> 2, 43u)) - 0.5;
            t.normalRough[p + 0] = to16(0.5 + 0.2 * nx);
            t.normalRough[p + 1] = to16(0.5 + 0.2 * ny);
            t.normalRough[p + 2] = 65535;
            t.normalRough[p + 3] = to16(0.4 + 0.4 * unit(hash3(x >> 4, y >> 4, 53u)));
        }
    // levels 1..10 are left to MipmapGen: the renderer's device kernel (texture.hip) and the
    // oracle's own restatement (oracle/texture.cpp) each build them from this level 0

}

}  // namespace rtscene
