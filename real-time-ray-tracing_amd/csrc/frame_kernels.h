// frame_kernels.h — launch interface of the per-frame path-trace, denoise and post kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct FrameResources {
    int dummy;
};
