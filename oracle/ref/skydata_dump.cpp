// ORACLE REFERENCE BUILD (test infrastructure only): the reference's Hosek-Wilkie / solar /
// limb-darkening / CIE tables, /root/reference/src/skyData.h, compiled here with plain g++ from
// where it lies (static float arrays, no includes).  Writes them to stdout in the layout of
// real-time-ray-tracing_amd/data/sky_tables.bin (u32 count 7, u32 lengths[7], float32 tables in
// the order skyDataSets, skyDataSetsRad, h_solarDatasets, h_limbDarkeningDatasets, spectrumCieX,
// spectrumCieY, spectrumCieZ), so the shipped table file can be compared byte for byte.
#include <stdint.h>
#include <stdio.h>

#include "skyData.h"

template <size_t N>
static void put(const float (&a)[N]) { fwrite(a, 4, N, stdout); }

int main() {
    const uint32_t count = 7;
    const uint32_t len[7] = {sizeof(skyDataSets) / 4, sizeof(skyDataSetsRad) / 4, sizeof(h_solarDatasets) / 4,
                             sizeof(h_limbDarkeningDatasets) / 4, sizeof(spectrumCieX) / 4, sizeof(spectrumCieY) / 4,
                             sizeof(spectrumCieZ) / 4};
    fwrite(&count, 4, 1, stdout);
    fwrite(len, 4, 7, stdout);
    put(skyDataSets);
    put(skyDataSetsRad);
    put(h_solarDatasets);
    put(h_limbDarkeningDatasets);
    put(spectrumCieX);
    put(spectrumCieY);
    put(spectrumCieZ);
    return 0;
}
