// ORACLE REFERENCE BUILD (test infrastructure only): the reference's default parameter structs,
// /root/reference/src/settingParams.h, compiled here with plain g++ from where it lies (it needs
// only <vector>, <utility>, <string>, <tuple>).  Prints their default member values as JSON, in
// the field order of include/rtx_amd.h's rt_params (bools as 0/1, the tone-map enum as its value).
#include <stdio.h>

#include "settingParams.h"

static void f(const char* name, double v, bool last = false) { printf("  \"%s\": %.9g%s\n", name, v, last ? "" : ","); }

int main() {
    SkyParams sky;
    SampleParams smp;
    RenderPassSettings ps;
    PostProcessParams pp;
    DenoisingParams dn;
    printf("{\n");
    f("sky.needRegenerate", sky.needRegenerate);
    f("sky.timeOfDay", sky.timeOfDay);
    f("sky.sunAxisAngle", sky.sunAxisAngle);
    f("sky.skyScalar", sky.skyScalar);
    f("sky.sunScalar", sky.sunScalar);
    f("sky.sunAngle", sky.sunAngle);
    f("sample.sampleSurfaceVsLightUseMisWeight", smp.sampleSurfaceVsLightUseMisWeight);
    f("sample.sampleSkyVsSunUseFluxWeight", smp.sampleSkyVsSunUseFluxWeight);
    f("sample.sampleSurfaceVsLight", smp.sampleSurfaceVsLight);
    f("sample.sampleSkyVsSun", smp.sampleSkyVsSun);
    f("pass.enableTemporalDenoising", ps.enableTemporalDenoising);
    f("pass.enableLocalSpatialFilter", ps.enableLocalSpatialFilter);
    f("pass.enableNoiseLevelVisualize", ps.enableNoiseLevelVisualize);
    f("pass.enableWideSpatialFilter", ps.enableWideSpatialFilter);
    f("pass.enableTemporalDenoising2", ps.enableTemporalDenoising2);
    f("pass.enablePostProcess", ps.enablePostProcess);
    f("pass.enableDownScalePasses", ps.enableDownScalePasses);
    f("pass.enableHistogram", ps.enableHistogram);
    f("pass.enableAutoExposure", ps.enableAutoExposure);
    f("pass.enableBloomEffect", ps.enableBloomEffect);
    f("pass.enableLensFlare", ps.enableLensFlare);
    f("pass.enableToneMapping", ps.enableToneMapping);
    f("pass.enableSharpening", ps.enableSharpening);
    f("post.toneMappingType", (int)pp.toneMappingType);
    f("post.exposure", pp.exposure);
    f("post.gain", pp.gain);
    f("post.maxWhite", pp.maxWhite);
    f("post.gamma", pp.gamma);
    f("denoise.local_denoise_sigma_normal", dn.local_denoise_sigma_normal);
    f("denoise.local_denoise_sigma_depth", dn.local_denoise_sigma_depth);
    f("denoise.local_denoise_sigma_material", dn.local_denoise_sigma_material);
    f("denoise.large_denoise_sigma_normal", dn.large_denoise_sigma_normal);
    f("denoise.large_denoise_sigma_depth", dn.large_denoise_sigma_depth);
    f("denoise.large_denoise_sigma_material", dn.large_denoise_sigma_material);
    f("denoise.temporal_denoise_sigma_normal", dn.temporal_denoise_sigma_normal);
    f("denoise.temporal_denoise_sigma_depth", dn.temporal_denoise_sigma_depth);
    f("denoise.temporal_denoise_sigma_material", dn.temporal_denoise_sigma_material);
    f("denoise.noise_threshold_local", dn.noise_threshold_local);
    f("denoise.noise_threshold_large", dn.noise_threshold_large, true);
    printf("}\n");
    return 0;
}
