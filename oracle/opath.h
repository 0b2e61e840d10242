// ORACLE (test infrastructure only; see ocommon.h) — shared declarations of the
// per-pixel restatement (camera, sampler, path tracer, sky).
#pragma once
#include "ocommon.h"
#include "oracle.h"

namespace orc {

static const float kPiOver4 = 0.7853981633974483096156608458198757210492f;  // linearMath.h:11-20
static const float kPiOver2 = 1.5707963267948966192313216916397514420985f;
static const float kPi = 3.1415926535897932384626422832795028841971f;
static const float kTwoPi = 6.2831853071795864769252867665590057683943f;
static const float kPiOver180 = 0.01745329251f;

struct Camera {
    F3 pos, dir, left, up;
    float yaw, pitch, focal, aperture;
    F2 res, invRes, fov, tanHalfFov;
    F3 adjustedLeft, adjustedUp, adjustedFront, apertureLeft, apertureUp;
};

void camera_update(const OrcCamera& in, Camera& c);
float bluenoise(const uint8_t* tables, int px, int py, int sampleIdx, int dim);
F2 concentric_disk(F2 u);
void generate_ray(const Camera& c, int ix, int iy, F2 pix, F2 ap, F3& orig, F3& dir, F3& centerDir, F2& sampleUv);
float ray_cone_width(const Camera& c, int ix, int iy);
void intersect_one(const OrcScene* sc, F3 org, F3 dir, OrcHit& out);

}  // namespace orc
