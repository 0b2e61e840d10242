// soil_textures.h — synthetic stand-in for the soil textures the reference loads but does not
// ship (an input of the hot path, not part of it; shared on purpose by the product and the oracle).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace rtscene {

// Synthetic stand-in for the soil texture pair the reference loads but does not ship
// (init.cu:524-549, .MISSING_LARGE_BLOBS): SoilAlbedoAo and SoilNormalRoughness, 1024^2
// ushort4, laid out as the reference's 11-level mip chain; make_textures fills level 0 only
// (deterministic integer hash): the mips are MipmapGen's (mipgen.cu:121-182), built on the device
// by the renderer (texture.hip) and restated by the oracle (oracle/texture.cpp).
struct TexturePair {
    static constexpr int kLevels = 11;
    int size[kLevels];                 // 1024 >> level
    size_t offset[kLevels];            // texel offset of each level (ushort4 units)
    std::vector<uint16_t> albedoAo;     // ushort4 texels, all levels concatenated
    std::vector<uint16_t> normalRough;  // ushort4 texels, all levels concatenated
};
void make_textures(TexturePair& t);

}  // namespace rtscene
