// frame.cpp — RayTracer::draw (kernel.cu:259-398) and GetBuffer2D behind the C-ABI.
#include "context.h"

extern "C" int rt_draw(rt_context* ctx, uint8_t* rgba8_out, float* hdr_out) {
    (void)rgba8_out;
    (void)hdr_out;
    if (!ctx) return RT_ERR_ARG;
    ctx->err = "rt_draw: path tracer not built in this revision";
    return RT_ERR_STATE;
}

extern "C" int rt_get_buffer(const rt_context* ctx, int name, void* dst, size_t bytes) {
    (void)name;
    (void)dst;
    (void)bytes;
    if (!ctx) return RT_ERR_ARG;
    return RT_ERR_STATE;
}
