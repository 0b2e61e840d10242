/* rtx_amd.h — C-ABI of the MI355X-native real-time path tracer (librtx.so).
 *
 * Drop-in boundary for the reference's renderer API, class RayTracer
 * (/root/reference/src/kernel.cuh:431-470) and its config surface LoadConfig
 * (configLoader.cpp:5-27).  Plain C: opaque handle, plain pointers and sizes, status codes
 * instead of the reference's exit() on errors (cudaError.cuh:6-13).  Not thread-safe per
 * handle (same as the reference).  All output buffers are caller-owned host memory.
 *
 * Every entry point below names the reference interface it replaces.
 */
#ifndef RTX_AMD_H
#define RTX_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_ERR_ARG (-1)         /* invalid argument / size */
#define RT_ERR_HIP (-2)         /* HIP runtime error (rt_last_error has the text) */
#define RT_ERR_IO (-3)          /* config / data file problem */
#define RT_ERR_STATE (-4)       /* call out of order (e.g. draw before init) */
#define RT_ERR_NO_DEVICE (-5)   /* no gfx950 device visible */
#define RT_ERR_DEVICE (-6)      /* a kernel reported a failure (rt_last_error has the text): the LBVH's
                                   TLAS workgroup timed out waiting for a batch; the frames since the
                                   last check may be wrong, the renderer re-armed itself.  Reported
                                   once, by the call that finds it: rt_sync, rt_build_bvh, the draws
                                   and the reads (rt_get_buffer, rt_download, rt_get_ray_count,
                                   rt_save_image ...).  Setters (rt_set_*stream, rt_bind_buffer,
                                   rt_set_collective_hook, rt_upload_texture) never return it: they
                                   do their work and leave the report to the next such call */

typedef struct rt_context rt_context;

/* ---------------------------------------------------------------- lifecycle */

/* RayTracer::RayTracer(screenWidth, screenHeight), kernel.cuh:435-441, plus LoadConfig
 * (configLoader.cpp:5-27).  config_toml may be NULL (defaults) or a path to a TOML file with
 * the reference's [resolution] / [file] / [optimziation] tables; extensions: [scene]
 * chunkDim (VoxelsGenerator::kChunkDim, terrain.h:42), [render] spp, [render] device.
 * [tuning] (scheduling A/B aids; the defaults are the measured best): arena (bool),
 * streams ("cumask" | "prio"), tracePerCu / trace4PerCu (0: automatic), trace3ShortPerCu (a short queue
 * 3's workgroups per CU on one GPU; 0: all of them), chain ("serial" | "off" |
 * "always"), shadeOnSide (bool), shadeBlocksPerCu (synchronous frames; 0: the kernel's residency),
 * overlapAfter / cameraAfter (-1: automatic); the synchronous draws' launches ahead (rt_draw):
 * syncSpec (bool), specAfter (the kernel of this frame they follow: 1 shade), specShade (0 / 1 / 2:
 * the shade kernel never / beside the lean bounce kernels / always), specShadePerCu, specTracePerCu,
 * specChain (-1: by queue 3's length); the denoise list passes: dnSplit (0 / 1 / 2: two threads per
 * pixel never / in synchronous frames / always; default 0), dnFold (bool, default false: the last
 * a-trous pass over list 1 only).  [debug] (fault
 * injection, tests): bvhSkipPublish, bvhSkipPublishBuilds, bvhWaitMs.  The library reads no
 * environment variables. */
int rt_create(int screen_width, int screen_height, const char* config_toml, rt_context** out);

/* RayTracer::init, init.cu:53-410: builds the procedural default scene, allocates every device
 * resource, uploads blue-noise/sky tables, runs the frame-1 smooth normals.  Like the reference it
 * ignores [file] inputMeshFileName (its LoadTrianglesFromFile call is commented out, init.cu:78-82);
 * the extension [scene] meshFile loads a meshProcessor .bin instead (u32 count + count 128-B
 * Triangle records, init.cu:28-50; a shorter file is refused with RT_ERR_IO).  The scene is built
 * and checked before any device call (RT_ERR_IO / RT_ERR_ARG on any machine), then the device
 * (RT_ERR_NO_DEVICE without a gfx950). */
int rt_init(rt_context* ctx);

/* RayTracer::draw, kernel.cu:259-398 (with UpdateFrame, kernel.cu:61-137): one synchronous
 * frame.  rgba8_out (screen W*H*4) and hdr_out (render W*H*4 floats, pre-tone-map HDR) may
 * each be NULL.  With [optimziation] useDynamicResolution the render size follows the frame
 * time from the second frame on (rt_get_info's renderWidth/Height); size hdr_out for
 * maxWidth x maxHeight.
 * Synchronous draws (this one, and rt_draw_device without RT_DRAW_ASYNC) on one GPU launch the
 * next frame's camera-ray and shade kernels ahead, beside this frame's bounces and denoise, into
 * the other G-buffer set ([tuning] syncSpec): the draw still returns with its frame complete, and
 * those kernels may still run on the context's side stream.  The next draw uses their results only
 * when its launch parameters (camera, sky, size, frame number, materials, buffers) equal theirs;
 * any call that waits for the streams (rt_sync, the reads, the setters) discards them first. */
int rt_draw(rt_context* ctx, uint8_t* rgba8_out, float* hdr_out);

/* RayTracer::draw(SurfObj* renderTarget), kernel.cu:259-398 (CopyToOutput kernel.cu:26-59 writes
 * the caller's surface): one frame whose screen-size RGBA8 image is written straight into
 * caller-owned DEVICE memory (row pitch in bytes, 0 = width * 4; 4-byte aligned).  flags 0: returns
 * when the frame is complete, as the reference's draw does (it ends with a device sync).
 * RT_DRAW_ASYNC: returns once the frame is enqueued; frames are pipelined (the denoise/post of
 * frame f overlaps the trace of f+1 on an internal stream (low priority under [tuning] streams = "prio") unless rt_set_post_stream
 * named one) and each frame's target must stay valid until rt_sync (or a later synchronous
 * call) has returned.  rt_download(RT_ARR_RGBA8) reads the last frame's target. */
#define RT_DRAW_ASYNC 1
int rt_draw_device(rt_context* ctx, void* rgba8_device, size_t pitch_bytes, int flags);

/* RayTracer::cleanup + ~RayTracer, init.cu:601-663, kernel.cuh:443-446 */
void rt_destroy(rt_context* ctx);

/* last error text for this handle (NULL handle: last rt_create failure) */
const char* rt_last_error(const rt_context* ctx);

/* ---------------------------------------------------------------- parameter surface */

/* SkyParams, settingParams.h:26-47 */
typedef struct rt_sky_params {
    int32_t needRegenerate;
    float timeOfDay, sunAxisAngle, skyScalar, sunScalar, sunAngle;
} rt_sky_params;

/* SampleParams, settingParams.h:49-66 */
typedef struct rt_sample_params {
    int32_t sampleSurfaceVsLightUseMisWeight, sampleSkyVsSunUseFluxWeight;
    float sampleSurfaceVsLight, sampleSkyVsSun;
} rt_sample_params;

/* RenderPassSettings, settingParams.h:68-104 */
typedef struct rt_render_pass_settings {
    int32_t enableTemporalDenoising, enableLocalSpatialFilter, enableNoiseLevelVisualize, enableWideSpatialFilter,
        enableTemporalDenoising2, enablePostProcess, enableDownScalePasses, enableHistogram, enableAutoExposure,
        enableBloomEffect, enableLensFlare, enableToneMapping, enableSharpening;
} rt_render_pass_settings;

/* PostProcessParams, settingParams.h:106-124 (toneMappingType: 0 Uncharted, 1 ACES1,
 * 2 ACES2, 3 Reinhard) */
typedef struct rt_post_process_params {
    int32_t toneMappingType;
    float exposure, gain, maxWhite, gamma;
} rt_post_process_params;

/* DenoisingParams, settingParams.h:126-157 */
typedef struct rt_denoising_params {
    float local_denoise_sigma_normal, local_denoise_sigma_depth, local_denoise_sigma_material;
    float large_denoise_sigma_normal, large_denoise_sigma_depth, large_denoise_sigma_material;
    float temporal_denoise_sigma_normal, temporal_denoise_sigma_depth, temporal_denoise_sigma_material;
    float noise_threshold_local, noise_threshold_large;
} rt_denoising_params;

/* public members skyParams .. sampleParams, kernel.cuh:465-470 */
typedef struct rt_params {
    rt_sky_params sky;
    rt_sample_params sample;
    rt_render_pass_settings pass;
    rt_post_process_params post;
    rt_denoising_params denoise;
} rt_params;

int rt_get_params(const rt_context* ctx, rt_params* out);
int rt_set_params(rt_context* ctx, const rt_params* in);

/* Camera fields the app sets (init.cu:412-439, kernel.cuh:78-121); fovX in radians */
typedef struct rt_camera {
    float pos[3];
    float yaw, pitch;
    float focal, aperture;
    float fovX;
} rt_camera;

int rt_get_camera(const rt_context* ctx, rt_camera* out); /* RayTracer::GetCamera */
int rt_set_camera(rt_context* ctx, const rt_camera* in);

/* Input (inputControl.cu:29-113): a windowing host forwards GLFW events (key, action and
 * modifier values are GLFW's).  keyboardUpdate sets the W/S/A/D/C/X movement flags and the
 * shift slow-down, or with ctrl saves (C) / loads (V) the camera at [file] cameraSaveFileName;
 * cursorPosUpdate turns the cursor delta into yaw / pitch (the first event after a cursor reset
 * only records the position); scrollUpdate and mouseButtenUpdate are no-ops as in the
 * reference.  rt_draw moves the camera by the held keys once per frame (InputControlUpdate,
 * pos += dir * deltaTime * moveSpeed).  cursorReset (kernel.cuh:465) starts set. */
int rt_keyboard_update(rt_context* ctx, int key, int scancode, int action, int mods);
int rt_cursor_pos_update(rt_context* ctx, double xpos, double ypos);
int rt_scroll_update(rt_context* ctx, double xoffset, double yoffset);
int rt_mouse_button_update(rt_context* ctx, int button, int action, int mods);
int rt_set_cursor_reset(rt_context* ctx, int reset);

/* RayTracer::SaveCameraToFile / LoadCameraFromFile (inputControl.cu:115-149): the reference's
 * 176-byte binary Camera record (kernel.cuh:78-100, derived fields included).  Loading takes
 * pos, pitch, yaw, focal, aperture and fov.x from the record; the derived fields are recomputed
 * by Camera::update every frame, as in the reference.  rt_init loads [file] inputCameraFileName
 * when loadCameraAtInit is true (init.cu:433-435). */
int rt_save_camera(const rt_context* ctx, const char* path);
int rt_load_camera(rt_context* ctx, const char* path);

/* Offscreen presentation (replaces the Vulkan swapchain blit, main.cu:1295-1310): the last
 * frame's RGBA8 output as a binary PPM (P6, screen size), or the denoised pre-tone-map HDR
 * colour as a PFM (PF, render size, bottom row first as the format prescribes). */
#define RT_IMAGE_PPM_RGBA8 0
#define RT_IMAGE_PFM_HDR 1
int rt_save_image(rt_context* ctx, const char* path, int kind);

/* Texture path, init.cu:524-580 + MipmapGen (mipgen.cu:121-182): a 16-bit texture of the atlas
 * (MipmapTextureName, texture.h:5-12) — its level 0 as stbi_load_16 returns it, rows of
 * width * channels ushorts — is copied to the device and its 11-level mip chain is generated there
 * (2x2 mean in float, min 65535, truncated to ushort).  The atlas is 1024 x 1024: 4 channels for
 * the albedo/AO and normal/roughness maps the diffuse shading samples, 1 for the height map.
 * rt_init uploads a deterministic synthetic pair (the PNGs are missing from the reference tree).
 * Synchronous. */
#define RT_TEX_SOIL_ALBEDO_AO 0
#define RT_TEX_SOIL_NORMAL_ROUGHNESS 1
#define RT_TEX_SOIL_HEIGHT 2
int rt_upload_texture(rt_context* ctx, int which, const uint16_t* texels, int width, int height, int channels);

/* Scene input (host only, no device needed): Perlin::noise3D (perlin.h:50-78) with the reference
 * permutation, the source of the procedural terrain's voxel heights (Chunk::Generate,
 * terrain.cpp:5-45), at n points (xyz triples). */
int rt_scene_noise3d(const float* xyz, size_t n, float* out);

/* The denoiser's Gaussian weights (GetGaussian3x3 / 5x5 / 7x7, gaussian.cuh:12-43; the precomputed
 * tables, USE_PRECALCULATED_GAUSSIAN): size 3, 5 or 7, row-major size*size floats into out (count
 * >= size*size).  The same values the device kernels use.  Host only, no device needed. */
int rt_filter_kernel(int size, float* out, int count);

/* Scan(in, out, tmp, size, blockSize, postfix), scan.cuh:258-298: prefix sum of `size` floats in
 * DEVICE memory — blocks of block_size scanned in LDS (Blelloch tree order), the block totals
 * scanned in one workgroup into tmp (>= size / block_size floats; unused for one block), then added.
 * postfix 1: inclusive, 0: exclusive.  size and block_size powers of two, block_size and the block
 * count each <= 8192 (the reference's asserts).  Enqueued on `stream` (a hipStream_t; NULL = null
 * stream), asynchronous.  Errors: RT_ERR_ARG / RT_ERR_HIP with rt_last_error(NULL). */
int rt_scan_device(const float* in, float* out, float* tmp, int size, int block_size, int postfix, void* stream);

/* Determinism hooks the reference lacks: the frame counter is a function static
 * (kernel.cu:64) and AutoExposure reads wall-clock deltaTime (postprocessing.cu:46-51). */
int rt_set_frame_index(rt_context* ctx, int frame_num); /* next rt_draw renders this frameNum */
int rt_set_delta_time(rt_context* ctx, float ms);       /* <= 0: wall clock */

/* ---------------------------------------------------------------- queries */

typedef struct rt_info {
    uint32_t triCount;          /* real triangles */
    uint32_t triCountPadded;    /* RayTracer::GetTriangleCount (kernel.cuh:462) */
    uint32_t batchCount;        /* BLAS batches of 1024 */
    uint32_t vertexCount;
    int32_t renderWidth, renderHeight, screenWidth, screenHeight;
    int32_t frameNum;           /* frame index of the last rt_draw (0 before the first) */
    int32_t deviceId;
    uint32_t spp;               /* samples (reference PathTrace evaluations) per frame */
    int32_t gbufferSet;         /* G-buffer set the last rt_path_trace wrote (0..2, see rt_set_post_stream) */
    int32_t denoiseRowBegin, denoiseRowEnd; /* rows of a strip-local denoise (rt_set_collective_hook) */
    int32_t gbufferRowBegin, gbufferRowEnd; /* G-buffer rows the next denoise reads: its strip plus
                                               halo when it is strip-local, else the whole frame */
    int32_t stripLocalDenoise;  /* 1: the next denoise is strip-local (the same on every rank) */
    int32_t shadeOnSide;        /* 1: pipelined frames run the shade kernel behind the camera kernel on
                                   the side stream (rt_set_post_stream), not on the context stream */
    int32_t lastChain;          /* 1: the last rt_path_trace ran its bounce stages as the fused k_pt_chain
                                   (serial frames while the previous serial frame's queue 3 was short),
                                   0: as the four kernels trace<3> .. resume<4>; profiles differ */
} rt_info;

int rt_get_info(const rt_context* ctx, rt_info* out);

/* GetBuffer2D, kernel.cuh:459: copies a render buffer to host memory.  Names follow the
 * Buffer2DName enum (kernel.cuh:286-315); half buffers come back as uint16 bit patterns. */
enum rt_buffer_name {
    RT_BUF_RENDER_COLOR = 0,   /* half4 (rgb + ushort material mask), render res */
    RT_BUF_ACCUMULATION = 1,   /* half4 */
    RT_BUF_HISTORY_COLOR = 2,  /* half4 */
    RT_BUF_SCALED_COLOR = 3,   /* half4, screen res */
    RT_BUF_NORMAL = 10,        /* half4 */
    RT_BUF_DEPTH = 11,         /* half */
    RT_BUF_HISTORY_DEPTH = 12, /* half */
    RT_BUF_MOTION = 13,        /* half2 */
    RT_BUF_NOISE_LEVEL = 14,   /* half, 8x8-tile grid */
    RT_BUF_NOISE_LEVEL16 = 15, /* half, 16x16-tile grid */
    RT_BUF_SKY = 16,           /* float4 512x256 */
    RT_BUF_SUN = 17,           /* float4 32x32 */
    RT_BUF_ALBEDO = 18,        /* half4 */
    RT_BUF_RGBA8 = 19,         /* uint8 x4, screen res: the last frame's output (CopyToOutput) */
    RT_BUF_HISTOGRAM = 20      /* uint32[64] luminance histogram (Histogram2) */
};
int rt_get_buffer(const rt_context* ctx, int name, void* dst, size_t bytes);
size_t rt_buffer_bytes(const rt_context* ctx, int name); /* 0 for names not available */

/* ---------------------------------------------------------------- hot-path stages */

/* BuildBvhLevel1 + BuildBvhLevel2 (bvh.cu:7-97): one per-frame two-level LBVH rebuild,
 * enqueued on the context stream (asynchronous). */
int rt_build_bvh(rt_context* ctx);

/* BASELINE config 2: GenerateRay + RaySceneIntersect for every render pixel with the
 * blue-noise sample of frame_num (pathtrace.cuh:116-130), enqueued asynchronously.
 * with_detail != 0 also stores normals / shading normals / traversal counters. */
int rt_trace_primary(rt_context* ctx, int frame_num, int with_detail);

/* PathTrace (pathtrace.cuh:11-128) for frame_num into the G-buffers (RT_BUF_RENDER_COLOR,
 * NORMAL, ALBEDO, DEPTH, MOTION), after UpdateFrame's sky/sun regeneration when the sky
 * parameters changed (kernel.cu:286-307).  spp > 1 ([render] spp) averages spp reference
 * samples (frame indices spp*(frame_num-1)+1 ...).  with_detail != 0 also stores the per-pixel
 * traced-ray count (RT_ARR_RAYS).  Asynchronous; the history camera advances (kernel.cu:357). */
int rt_path_trace(rt_context* ctx, int frame_num, int with_detail);

/* TemporalSpatialDenoising + PostProcessing + CopyToOutput (denoising.cu:5-189,
 * postprocessing.cu:5-161, kernel.cu:376-381) on the G-buffers of the last rt_path_trace, for
 * frame_num (frame 1 skips the temporal passes).  Afterwards RT_BUF_RENDER_COLOR holds the
 * denoised HDR colour and RT_BUF_SCALED_COLOR the tone-mapped screen image; the RGBA8 image and
 * (with_hdr) a float4 HDR copy are kept on the device for rt_draw.  Asynchronous. */
int rt_denoise_post(rt_context* ctx, int frame_num, int with_hdr);

/* Traced rays (RaySceneIntersect calls that ran a traversal) accumulated since the last reset. */
int rt_get_ray_count(rt_context* ctx, uint64_t* rays, int reset);

/* Enqueue every later stage on `stream` (a hipStream_t, e.g. the caller's framework stream so
 * its collectives order with the renderer).  NULL is the device's null stream (a framework's
 * default stream, e.g. torch's, is that stream); RT_OWN_STREAM restores the context's own. */
#define RT_OWN_STREAM ((void*)(intptr_t)-1)
#define RT_STREAM_OFF ((void*)(intptr_t)-2) /* rt_set_gather_stream: no gather stream */
int rt_set_stream(rt_context* ctx, void* stream);

/* Frame pipelining (no reference counterpart; the reference draws frames strictly one after
 * another): with a post stream set, rt_denoise_post runs the denoiser and post chain on that
 * stream, after everything enqueued on the context stream so far (path trace, G-buffer
 * gathers), and the path tracer alternates between two G-buffer sets, so the trace of frame
 * f+1 overlaps the denoise of frame f; the LBVH build and camera rays of the next frame run on
 * an internal third stream beside the current frame's trace kernels (two LBVH sets,
 * RT_GBUFFER_SETS G-buffer sets).  Results are identical to the serial order.  Host reads
 * (rt_get_buffer, rt_download, rt_sync, rt_draw's copies) wait for all streams.  NULL turns it off.
 * rt_info.gbufferSet names the set the last path trace wrote; bind the other sets' buffers
 * with name | RT_BUF_SET1 / RT_BUF_SET2 / RT_BUF_SET3. */
#define RT_GBUFFER_SETS 4
#define RT_BUF_SET1 0x100
#define RT_BUF_SET2 0x200
#define RT_BUF_SET3 0x300
int rt_set_post_stream(rt_context* ctx, void* stream);

/* Multi-GPU gathers off the trace chain (no reference counterpart): each later rt_denoise_post
 * also waits for the work enqueued on `stream` up to that call, so a host that gathers a
 * frame's G-buffer rows on its own stream (after the path trace; rtx/dist.py) keeps the next
 * frame's path trace free of the collective.  The gathers must not write a G-buffer set the
 * renderer is still using: gather the set rt_info.gbufferSet names, right after its path trace.
 * NULL is the null stream (as in rt_set_stream); RT_STREAM_OFF (the default) turns it off. */
int rt_set_gather_stream(rt_context* ctx, void* stream);

/* Multi-GPU strip-local denoise (no reference counterpart, the reference runs on one
 * GPU).  With stripCount > 1 and a hook set, each rank runs the denoise/post chain only for its own
 * contiguous rows [rowBegin, rowEnd) — the frame's 64-row blocks split evenly over the ranks — plus
 * the halo rows its passes read (the summed stencil radius, ~64 rows each side), instead of the
 * whole frame.  Two exchanges per frame make the result identical to one GPU; the renderer asks the
 * host to enqueue them on `stream` (the stream the denoise runs on) through the hook:
 *   RT_HOOK_HISTOGRAM  sum the ranks' 64-bin histograms (RT_BUF_HISTOGRAM) in place (all-reduce)
 *                      before AutoExposure reads them;
 *   RT_HOOK_ROWS       give every rank every rank's rows [rowBegin, rowEnd) of the accumulation
 *                      buffer, of history buffer `historySet` (the final HDR of the frame) and of the
 *                      RGBA8 output (all-gather), before the next frame's temporal passes read them.
 * The host binds those buffers to its own device memory (rt_bind_buffer: RT_BUF_ACCUMULATION,
 * RT_BUF_HISTORY_COLOR sets 0 and 1, RT_BUF_HISTOGRAM, RT_BUF_RGBA8) so its collectives move them
 * in place (rtx/dist.py StripDenoise).  The hook returns 0 on success.  Without a hook (or with the
 * noise visualisation, bloom or lens flare on) every rank denoises the whole frame. */
typedef struct rt_strip_exchange {
    int32_t frameNum;
    int32_t rowBegin, rowEnd;   /* this rank's rows */
    int32_t historySet;         /* history buffer (0 / 1) TemporalFilter2 wrote this frame */
    int32_t gbufferSet;         /* G-buffer set the frame was traced into (RT_HOOK_GBUFFERS) */
    int32_t stripLocal;         /* 1: the denoise is strip-local (rt_info.stripLocalDenoise) */
} rt_strip_exchange;
#define RT_HOOK_HISTOGRAM 0
#define RT_HOOK_ROWS 1
/* Optional third stage (rt_set_hook_stages): before the denoise, give every rank the G-buffer rows its
 * denoise reads (rt_info.gbufferRowBegin/End of each rank; the whole frame when stripLocal is 0) from
 * the ranks that traced them, in G-buffer set gbufferSet — what rtx/dist.py's StripGather does outside
 * the renderer.  With it, rt_draw and rt_draw_device run a multi-GPU frame by themselves
 * (include/rtx_dist.h implements all three stages). */
#define RT_HOOK_GBUFFERS 2
typedef int (*rt_collective_fn)(void* arg, int stage, void* stream, const rt_strip_exchange* x);
int rt_set_collective_hook(rt_context* ctx, rt_collective_fn fn, void* arg);
/* which stages the hook is called for: bit (1 << RT_HOOK_*); default HISTOGRAM | ROWS.  HISTOGRAM and
 * ROWS are mandatory whenever a strip-local denoise runs (a mask without either is refused with
 * RT_ERR_ARG); the mask only opts into RT_HOOK_GBUFFERS. */
int rt_set_hook_stages(rt_context* ctx, uint32_t stage_mask);

/* Use caller-owned device memory (>= the buffer's size at the largest render size, i.e.
 * maxWidth x maxHeight with dynamic resolution, else rt_buffer_bytes; 16-B aligned) as one of the path-trace
 * G-buffers (RT_BUF_RENDER_COLOR / NORMAL / ALBEDO / DEPTH / MOTION), e.g. so a multi-GPU host
 * can all-gather screen strips in place; and the strip-local denoise's exchanged buffers
 * (RT_BUF_ACCUMULATION, RT_BUF_HISTORY_COLOR | RT_BUF_SET1 for the second of the pair,
 * RT_BUF_HISTOGRAM, RT_BUF_RGBA8), whose current contents are copied over.  The memory must
 * outlive the context's use of it. */
int rt_bind_buffer(rt_context* ctx, int name, void* device_ptr, size_t bytes);

/* wait for all work on the context stream */
int rt_sync(rt_context* ctx);

/* HIP-event timing on the context stream: runs `iters` back-to-back launches of a stage
 * (0 = BVH build, 1 = primary rays, 2 = path trace, 3 = full frame: BVH + path trace + denoise
 * + post, 4 = denoise + post) and returns the total
 * milliseconds between the first launch and the end of the last. */
int rt_time_stage(rt_context* ctx, int stage, int iters, float* total_ms);

/* Test entry (no reference counterpart): the denoiser's packed-pair transcendentals (rtmath_pk.h)
 * beside their scalar rtmath.h forms, over a caller-owned device array x of n floats (element i
 * is paired with i ^ 1).  fn 0: pow(x, y) (x finite >= 0, y finite > 0), 1: expf(x), 2: x / y
 * through c = RN(1 / y) (rt_div_rcp).  out_pk / out_scalar (device, n floats each) receive the two
 * results, which must agree bit for bit.  Null stream, synchronising; RT_ERR_ARG on bad arguments. */
int rt_debug_pk_math(int fn, const float* x, float y, float c, float* out_pk, float* out_scalar, size_t n);

/* HIP-event split of the path-trace stage (stage 2 above): runs `iters` path traces with an
 * event recorded between consecutive kernels and writes the average milliseconds of each kernel
 * (n >= 7: camera, shade, trace bounce queue, resume, trace shadow queue, resume, resolve).
 * Measurement aid for the roofline in bench.py; no reference counterpart. */
int rt_time_path_trace_kernels(rt_context* ctx, int iters, float* kernel_ms, int n);

/* The same split over `iters` whole frames (LBVH build + path trace + denoise/post of frames
 * first_frame, first_frame + 1, ...) run exactly as a caller runs them: on a pipelined context
 * (rt_set_post_stream) each kernel is timed on the stream it runs on, beside the other streams'
 * work.  With n >= 15 entries 7..14 are the denoise / post chain's kernels (TemporalFilter,
 * SpatialFilter7x7, the three a-trous passes, TemporalFilter2, the DownScale4 / histogram /
 * AutoExposure chain, the scale / sharpen / tone map / dither pass), each averaged over the frames
 * that launched it.  Waits for the frames.  Measurement aid for bench.py's per-kernel roofline. */
int rt_time_frame_kernels(rt_context* ctx, int first_frame, int iters, float* kernel_ms, int n);

/* The same split recorded inside the caller's own frames: the next `frames` frames (each a path
 * trace and the rt_denoise_post that follows it) bracket the kernels whose bit is set in
 * kernel_mask (bit k = kernel k, the 15 kernels above) with HIP events on the stream each runs on
 * (two events per kernel, no synchronisation); rt_frame_marks_read waits, writes the per-kernel
 * average milliseconds over the frames recorded (n >= 7 entries, up to 15; -1 for kernels not
 * marked) and stops recording.  bench.py's warm-up and timed frames use it. */
int rt_frame_marks_begin(rt_context* ctx, int frames, uint32_t kernel_mask);
int rt_frame_marks_read(rt_context* ctx, float* kernel_ms, int n, int* frames_recorded);

/* Copies device arrays to host (debug dumps of bvh.cu:15-96, traversal outputs). */
enum rt_array_name {
    RT_ARR_VERTICES = 0,         /* float[nv][3] */
    RT_ARR_INDICES = 1,          /* uint32[triCountPadded][3] */
    RT_ARR_NORMALS = 2,          /* float[nv][3] (smooth normals) */
    RT_ARR_TRI_POS = 3,          /* float4[triCountPadded][3] */
    RT_ARR_AABBS = 4,            /* float[triCountPadded][6] min xyz max xyz */
    RT_ARR_MORTON = 5,           /* uint32[B*1024] sorted codes (morton2.csv) */
    RT_ARR_REORDER = 6,          /* uint32[B*1024] (reorderIdx.csv) */
    RT_ARR_NODES = 7,            /* 64-B nodes [triCountPadded]: lmin lmax rmin rmax (12 f32), idxL idxR leafL leafR */
    RT_ARR_TLAS_AABBS = 8,       /* float[B][6] */
    RT_ARR_TLAS_MORTON = 9,      /* uint32[1024] sorted */
    RT_ARR_TLAS_REORDER = 10,    /* uint32[1024] */
    RT_ARR_TLAS_NODES = 11,      /* 64-B nodes [B] */
    RT_ARR_TLAS_SCENE_AABB = 12, /* float[6] */
    RT_ARR_BATCH_SCENE_AABBS = 13, /* float[B][6] */
    RT_ARR_HITS = 14,            /* float4[W*H]: t, objectIdx (int bits), u, v */
    RT_ARR_HIT_NORMALS = 15,     /* float4[W*H]: geometric normal, hit flag */
    RT_ARR_HIT_FAKE_NORMALS = 16,/* float4[W*H]: shading normal, ray offset */
    RT_ARR_HIT_STATS = 17,       /* uint32[W*H][4]: node visits, tri tests, dropped pushes, iterations */
    RT_ARR_TRI_NRM = 18,         /* float4[triCountPadded][3] */
    RT_ARR_RAYS = 19,            /* uint32[W*H] traced rays per pixel (rt_path_trace with_detail) */
    RT_ARR_SKY_PDF = 20,         /* float[131072] sky luminance (Sky kernel, sky.cuh:296-297) */
    RT_ARR_SKY_CDF = 21,         /* float[131072] inclusive scan of the sky pdf */
    RT_ARR_SUN_PDF = 22,         /* float[1024] */
    RT_ARR_SUN_CDF = 23,         /* float[1024] */
    RT_ARR_SUN_DIR = 24,         /* float[4]: sunDir xyz, cos(sun half-angle) (host values) */
    RT_ARR_HISTOGRAM = 25,       /* uint32[64] luminance histogram (Histogram2) */
    RT_ARR_EXPOSURE = 26,        /* float[4] exposure, adapted lum, bright lum, bright bin lum */
    RT_ARR_COLOR4 = 27,          /* half4 [ceil(W/4) * ceil(H/4)] DownScale4 chain */
    RT_ARR_COLOR16 = 28,         /* half4 [ceil(W/16) * ceil(H/16)] */
    RT_ARR_COLOR64 = 29,         /* half4 [ceil(W/64) * ceil(H/64)] */
    RT_ARR_RGBA8 = 30,           /* uint8[Ws*Hs][4] final output of the last rt_draw / rt_denoise_post */
    RT_ARR_PT_QUEUE = 32,        /* uint32[64] path-trace wavefront counters of the last launch: [0] rays
                                    deferred at step 3, [1] at step 4, [4] pixels resolved late,
                                    [8]/[9] longest traversal (iterations) of the step-3/4 queues
                                    (detail launches only), [10] internal errors (must be 0),
                                    [11] pixels with a sample that hit geometry; detail launches
                                    also: node visits / triangle tests of [12,13] the camera
                                    kernel, [14,15] the shade kernel (inline glossy traces),
                                    [16,17] the step-3 and [18,19] the step-4 queue tracers,
                                    diffuse events of [20] the shade and [21] the resume<3> kernel,
                                    [22] camera rays settled by the scene cull (no traversal) */
    RT_ARR_PT_Q3_ORIGINS = 33,   /* float4[cap] step-3 queue rays of the last launch: origin xyz, pixel bits */
    RT_ARR_PT_Q3_DIRS = 34,      /* float4[cap] direction xyz, flags bits ([0] of RT_ARR_PT_QUEUE are valid) */
    RT_ARR_PT_Q4_ORIGINS = 35,   /* float4[cap] step-4 queue, same layout ([1] valid) */
    RT_ARR_PT_Q4_DIRS = 36,
    RT_ARR_PT_STATS = 31,        /* uint32[W*H][4] rays, node visits, triangle tests, diffuse events
                                    (rt_path_trace with_detail) */
    RT_ARR_TEX_ALBEDO_AO = 37,   /* ushort4, 11-level mip chain of 1024^2 (levels concatenated, 1024 -> 1) */
    RT_ARR_TEX_NORMAL_ROUGHNESS = 38, /* ushort4, same layout */
    RT_ARR_TEX_HEIGHT = 39,      /* ushort, same layout (zero unless uploaded) */
    RT_ARR_HDR = 40,             /* float4[W*H] pre-tone-map HDR of the last rt_draw / rt_denoise_post with_hdr */
    RT_ARR_BVH_ARENA = 41        /* the traversal's record arena as the device holds it (64-B records: B*1024 BLAS
                                    nodes, B TLAS nodes, triCountPadded triangle records); the
                                    NODES / TLAS_NODES / TRI_POS arrays are views of it in the reference layout */
};
int rt_download(const rt_context* ctx, int what, void* dst, size_t bytes);

/* Batch ray query: the reference's RaySceneIntersect traversal (traverse.cuh:107-253, the
 * closest hit of TraverseBvh with its 16-entry stack and 1024-iteration cap) for n caller rays,
 * run by the persistent queue tracer on the BVH of the last rt_build_bvh.
 *   rays  n x 8 floats: origin xyz, (unused), direction xyz, (unused)
 *   hits  n x 4 floats: t (RayMax on a miss), triangle index as int32 bits (-1 on a miss), u, v
 *   iters optional n x uint32: TraverseBvh loop iterations per ray
 *   kernel_ms optional: HIP-event time of the tracer kernel alone
 * n must not exceed width x strip rows x spp (the queue capacity).  Host buffers; synchronous. */
int rt_trace_rays(rt_context* ctx, const float* rays, uint32_t n, float* hits, uint32_t* iters, float* kernel_ms);
size_t rt_array_bytes(const rt_context* ctx, int what);

#ifdef __cplusplus
}
#endif

#endif /* RTX_AMD_H */
