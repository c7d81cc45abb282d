// sng_math.h -- host/device math for the MI355X SyNeRFgine render path.
//
// Float semantics follow the reference's device code (tcnn vec/mat, cited per
// function) evaluated IEEE-exactly: the library is compiled with
// -ffp-contract=off so that marching decisions match the CPU oracle bitwise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SNG_HD __host__ __device__ __forceinline__

namespace sng {

// ---- constants: nerf_device.cuh:25-43, common_device.cuh:32-33, testbed_nerf.cu:47-50
constexpr uint32_t GRID_SIZE = 128;
constexpr uint32_t GRID_CELLS = GRID_SIZE * GRID_SIZE * GRID_SIZE;
constexpr uint32_t N_CASCADES = 8;
constexpr uint32_t NERF_STEPS = 1024;
constexpr float SQRT3 = 1.73205080757f;
constexpr float MIN_STEP = SQRT3 / NERF_STEPS;
constexpr float MAX_STEP = MIN_STEP * (1 << (N_CASCADES - 1)) * NERF_STEPS / GRID_SIZE;
constexpr float MAX_DEPTH = 16384.0f;
constexpr float MIN_DEPTH = 0.00001f;
constexpr uint32_t MARCH_ITER = 10000;
constexpr uint32_t MAX_STEPS_BETWEEN_COMPACTION = 8;
constexpr float MIN_OPTICAL_THICKNESS = 0.01f;
constexpr float PI_F = 3.14159265358979323846f;
constexpr uint32_t PT_SEED = 1999;  // synerfgine/common.cuh:20

struct f3 { float x, y, z; };
SNG_HD f3 mk(float x, float y, float z) { return {x, y, z}; }
SNG_HD f3 splat(float s) { return {s, s, s}; }
SNG_HD f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
SNG_HD f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
SNG_HD f3 operator-(f3 a) { return {-a.x, -a.y, -a.z}; }
SNG_HD f3 operator*(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
SNG_HD f3 operator/(f3 a, f3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
SNG_HD f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
SNG_HD f3 operator*(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
SNG_HD f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
SNG_HD f3 operator+(f3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }
SNG_HD f3 operator-(f3 a, float s) { return {a.x - s, a.y - s, a.z - s}; }
SNG_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
SNG_HD f3 cross(f3 a, f3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
SNG_HD float length(f3 a) { return sqrtf(dot(a, a)); }
// tcnn normalize(): zero-length guard returns the first unit vector [tcnn vec.h]
SNG_HD f3 normalize(f3 a) {
    float l = length(a);
    if (!(l > 0.0f)) return {1.0f, 0.0f, 0.0f};
    return a / l;
}
SNG_HD f3 inv(f3 a) { return {1.0f / a.x, 1.0f / a.y, 1.0f / a.z}; }
SNG_HD float fractf_(float x) { return x - floorf(x); }
SNG_HD float sgnf(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
// Deterministic exp / log.  The reference builds with --use_fast_math (CMakeLists.txt:82), so its
// expf/logf are approximations; no bit pattern is "the" reference.  These two are written with
// IEEE basic operations and fmaf only (<= ~1 ulp), so the CPU oracle (its own copy in
// oracle/sng_oracle.cpp) and the GPU produce identical bits wherever a marching or termination
// DECISION depends on them (cone stepping, compositing alpha).
// x / d, correctly rounded, from y = RN(1/d): q0 = RN(x*y) plus one FMA remainder correction
// (Markstein).  Verified bit-identical to IEEE division for every float t in [1e-9, 4e4] with
// d = MIN_STEP and for 4e8 random (x, d) pairs (tools/divtest: 0 mismatches).
SNG_HD float div_by(float x, float d, float y) {
    const float q0 = x * y;
    const float r = fmaf(-q0, d, x);
    return fmaf(r, y, q0);
}
// RN(1/d) for 2^-126 <= |d| < 2^126: on the device v_rcp_f32 plus one FMA correction, which equals IEEE
// 1.0f / d for every such d (tools/rcp_check.hip: all 2^32 inputs on gfx950, profiles/rcp_check_r02.txt);
// the host divides.
SNG_HD float recip_rn(float d) {
#ifdef __HIP_DEVICE_COMPILE__
    const float y = __builtin_amdgcn_rcpf(d);
    return fmaf(fmaf(-d, y, 1.0f), y, y);
#else
    return 1.0f / d;
#endif
}
SNG_HD float sng_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935f) return __builtin_huge_valf();
    if (x < -103.972084f) return 0.0f;
    const float n = rintf(x * 1.44269502f);
    float r = fmaf(n, -0.693145752f, x);          // ln2 split: hi has 12 trailing zero bits
    r = fmaf(n, -1.42860677e-06f, r);
    float p = 1.98412698e-04f;                    // Taylor to r^7 on |r| <= 0.35
    p = fmaf(p, r, 1.38888889e-03f);
    p = fmaf(p, r, 8.33333377e-03f);
    p = fmaf(p, r, 4.16666679e-02f);
    p = fmaf(p, r, 1.66666672e-01f);
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return scalbnf(p, (int)n);
}
SNG_HD float sng_logf(float x) {
    if (x != x || x < 0.0f) return x != x ? x : __builtin_nanf("");
    if (x == 0.0f) return -__builtin_huge_valf();
    if (x == __builtin_huge_valf()) return x;
    int e;
    float m = frexpf(x, &e);                      // [0.5, 1)
    if (m < 0.707106769f) { m = m * 2.0f; e -= 1; }
    const float f = m - 1.0f;                     // exact (Sterbenz)
    // f / (2 + f) as div_by with the exact reciprocal: equal to the IEEE division for every f this
    // function forms (all 2^24 mantissas, tests/native/march_check.cpp)
    const float s = div_by(f, 2.0f + f, recip_rn(2.0f + f));
    const float z = s * s;
    const float R = z * fmaf(z, fmaf(z, fmaf(z, 0.222222224f, 0.285714298f), 0.400000006f), 0.666666687f);
    const float hf = 0.5f * f * f;
    const float dk = (float)e;
    return fmaf(dk, 0.693145752f, (f - (hf - fmaf(s, hf + R, dk * 1.42860677e-06f))));
}
SNG_HD float logistic(float x) { return 1.0f / (1.0f + sng_expf(-x)); }
SNG_HD float smoothstep(float x) { return x * x * (3.0f - 2.0f * x); }
SNG_HD f3 reflect(f3 i, f3 n) { return 2.0f * dot(i, n) * n - i; }

// column-major 3x3; mat*vec accumulates columns as tcnn's tmat operator*
struct m3 { f3 c0, c1, c2; };
SNG_HD f3 mul(const m3& m, f3 v) {
    f3 r = splat(0.0f);
    r = r + m.c0 * v.x;
    r = r + m.c1 * v.y;
    r = r + m.c2 * v.z;
    return r;
}
SNG_HD m3 mulm(const m3& a, const m3& b) { return {mul(a, b.c0), mul(a, b.c1), mul(a, b.c2)}; }

// get_xform_given_rolling_shutter's rotation (common_device.cuh:361-368): glm-style quat_cast of
// both cameras, slerp(q0, q1, t), normalize, to_mat3 [tcnn quat, unvendored: parity unpinned]
struct q4 { float x, y, z, w; };
SNG_HD q4 quat_from_m3(const m3& M) {
    auto e = [&](int i, int j) { const f3& c = i == 0 ? M.c0 : (i == 1 ? M.c1 : M.c2); return j == 0 ? c.x : (j == 1 ? c.y : c.z); };
    const float fx = e(0, 0) - e(1, 1) - e(2, 2), fy = e(1, 1) - e(0, 0) - e(2, 2), fz = e(2, 2) - e(0, 0) - e(1, 1), fw = e(0, 0) + e(1, 1) + e(2, 2);
    int bi = 0;
    float fb = fw;
    if (fx > fb) { fb = fx; bi = 1; }
    if (fy > fb) { fb = fy; bi = 2; }
    if (fz > fb) { fb = fz; bi = 3; }
    const float bv = sqrtf(fb + 1.0f) * 0.5f, mult = 0.25f / bv;
    switch (bi) {
        case 0: return {(e(1, 2) - e(2, 1)) * mult, (e(2, 0) - e(0, 2)) * mult, (e(0, 1) - e(1, 0)) * mult, bv};
        case 1: return {bv, (e(0, 1) + e(1, 0)) * mult, (e(2, 0) + e(0, 2)) * mult, (e(1, 2) - e(2, 1)) * mult};
        case 2: return {(e(0, 1) + e(1, 0)) * mult, bv, (e(1, 2) + e(2, 1)) * mult, (e(2, 0) - e(0, 2)) * mult};
        default: return {(e(2, 0) + e(0, 2)) * mult, (e(1, 2) + e(2, 1)) * mult, bv, (e(0, 1) - e(1, 0)) * mult};
    }
}
SNG_HD m3 shutter_rotation(q4 a, q4 b, float t) {
    float cos_theta = a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
    if (cos_theta < 0.0f) { b = {-b.x, -b.y, -b.z, -b.w}; cos_theta = -cos_theta; }   // the short way round
    q4 s;
    if (cos_theta > 1.0f - 1.1920929e-7f) {   // mix(a, b, t)
        s = {a.x * (1.0f - t) + b.x * t, a.y * (1.0f - t) + b.y * t, a.z * (1.0f - t) + b.z * t, a.w * (1.0f - t) + b.w * t};
    } else {
        const float angle = acosf(cos_theta), s0 = sinf((1.0f - t) * angle), s1 = sinf(t * angle), sa = sinf(angle);
        s = {(s0 * a.x + s1 * b.x) / sa, (s0 * a.y + s1 * b.y) / sa, (s0 * a.z + s1 * b.z) / sa, (s0 * a.w + s1 * b.w) / sa};
    }
    const float len = sqrtf(s.x * s.x + s.y * s.y + s.z * s.z + s.w * s.w);
    s = {s.x / len, s.y / len, s.z / len, s.w / len};
    const float qxx = s.x * s.x, qyy = s.y * s.y, qzz = s.z * s.z, qxz = s.x * s.z, qxy = s.x * s.y, qyz = s.y * s.z;
    const float qwx = s.w * s.x, qwy = s.w * s.y, qwz = s.w * s.z;
    return {mk(1.0f - 2.0f * (qyy + qzz), 2.0f * (qxy + qwz), 2.0f * (qxz - qwy)),
            mk(2.0f * (qxy - qwz), 1.0f - 2.0f * (qxx + qzz), 2.0f * (qyz + qwx)),
            mk(2.0f * (qxz + qwy), 2.0f * (qyz - qwx), 1.0f - 2.0f * (qxx + qyy))};
}

// sRGB: common_device.cuh:35-70
SNG_HD float srgb_to_linear(float s) { return s <= 0.04045f ? s / 12.92f : powf((s + 0.055f) / 1.055f, 2.4f); }
SNG_HD float linear_to_srgb(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * powf(l, 0.41666f) - 0.055f; }

// ---- Morton (tcnn common_device.h) --------------------------------------------
SNG_HD uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
SNG_HD uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) { return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2); }
SNG_HD uint32_t morton3D_invert(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

// ---- AABB slab test: bounding_box.cuh:163-211 ---------------------------------
struct aabb { f3 lo, hi; };
constexpr float INV_MIN_STEP = 1.0f / MIN_STEP;   // RN(1/MIN_STEP), folded at compile time

struct f2 { float x, y; };

// ---- lens models: ELensMode / Lens (common.h:188-205), distortion deltas and the Newton undistortion
// (common_device.cuh:250-338), uv_to_ray's direction per mode (403-447), pos_to_uv's forward distortion (507-541).
// tcnn's mat2 inverse (vec.h, unvendored) is restated as 1/det times the adjugate.
enum : int32_t { LENS_PERSPECTIVE = 0, LENS_OPENCV = 1, LENS_FTHETA = 2, LENS_LATLONG = 3, LENS_OPENCV_FISHEYE = 4, LENS_EQUIRECTANGULAR = 5 };
struct Lens { int32_t mode; float params[7]; };

// opencv_lens_distortion_delta (common_device.cuh:250-266): params k1 k2 p1 p2
SNG_HD void opencv_delta(const float* p, float u, float v, float& du, float& dv) {
    const float k1 = p[0], k2 = p[1], p1 = p[2], p2 = p[3];
    const float u2 = u * u, uv = u * v, v2 = v * v;
    const float r2 = u2 + v2;
    const float radial = k1 * r2 + k2 * r2 * r2;
    du = u * radial + 2.0f * p1 * uv + p2 * (r2 + 2.0f * u2);
    dv = v * radial + 2.0f * p2 * uv + p1 * (r2 + 2.0f * v2);
}
// opencv_fisheye_lens_distortion_delta (268-292): params k1 k2 k3 k4; the threshold is double's epsilon as a float
SNG_HD void fisheye_delta(const float* p, float u, float v, float& du, float& dv) {
    const float r = sqrtf(u * u + v * v);
    if (r > 2.220446049250313e-16f) {
        const float theta = atanf(r);
        const float t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t4 * t4;
        const float thetad = theta * (1.0f + p[0] * t2 + p[1] * t4 + p[2] * t6 + p[3] * t8);
        du = u * thetad / r - u;
        dv = v * thetad / r - v;
    } else {
        du = 0.0f;
        dv = 0.0f;
    }
}
SNG_HD void lens_delta(int32_t mode, const float* p, float u, float v, float& du, float& dv) {
    if (mode == LENS_OPENCV_FISHEYE) fisheye_delta(p, u, v, du, dv);
    else opencv_delta(p, u, v, du, dv);
}
// iterative_lens_undistortion (294-330): Newton on x + delta(x) = x0 with central-difference Jacobians, at most 100
// iterations, stop once |step|^2 < 1e-10
SNG_HD void lens_undistort(int32_t mode, const float* p, float& u, float& v) {
    const float x0u = u, x0v = v;
    float xu = u, xv = v;
#pragma unroll 1
    for (uint32_t i = 0; i < 100; ++i) {
        const float s0 = fmaxf(1.1920929e-07f, fabsf(1e-6f * xu));   // max(FLT_EPSILON, |kRelStepSize x|)
        const float s1 = fmaxf(1.1920929e-07f, fabsf(1e-6f * xv));
        float du, dv, u0b, v0b, u0f, v0f, u1b, v1b, u1f, v1f;
        lens_delta(mode, p, xu, xv, du, dv);
        lens_delta(mode, p, xu - s0, xv, u0b, v0b);
        lens_delta(mode, p, xu + s0, xv, u0f, v0f);
        lens_delta(mode, p, xu, xv - s1, u1b, v1b);
        lens_delta(mode, p, xu, xv + s1, u1f, v1f);
        // J column-major: J[0][0] J[0][1] first column, J[1][0] J[1][1] second
        const float j00 = 1.0f + (u0f - u0b) / (2.0f * s0);
        const float j10 = (u1f - u1b) / (2.0f * s1);
        const float j01 = (v0f - v0b) / (2.0f * s0);
        const float j11 = 1.0f + (v1f - v1b) / (2.0f * s1);
        const float d = 1.0f / (j00 * j11 - j10 * j01);
        const float i00 = d * j11, i01 = -d * j01, i10 = -d * j10, i11 = d * j00;   // inverse(J), column-major
        const float ru = xu + du - x0u, rv = xv + dv - x0v;
        const float su = i00 * ru + i10 * rv, sv = i01 * ru + i11 * rv;
        xu -= su;
        xv -= sv;
        if (su * su + sv * sv < 1e-10f) break;
    }
    u = xu;
    v = xv;
}
// uv_to_ray's camera-space direction (common_device.cuh:425-447) for a non-foveated, unmasked view: false when the
// ray is invalid (F-Theta outside its domain)
SNG_HD bool lens_dir(const Lens& L, f2 uv, f2 sc, int W, int H, f2 focal, f3& dir) {
    if (L.mode == LENS_FTHETA) {   // f_theta_undistortion (370-384), error direction 0
        const float xpix = (uv.x - sc.x) * L.params[5], ypix = (uv.y - sc.y) * L.params[6];
        const float norm = sqrtf(xpix * xpix + ypix * ypix);
        const float alpha = L.params[0] + norm * (L.params[1] + norm * (L.params[2] + norm * (L.params[3] + norm * L.params[4])));
        float sa, ca;
        sincosf(alpha, &sa, &ca);
        if (ca <= 1.17549435e-38f || norm == 0.0f) { dir = splat(0.0f); return false; }
        sa *= 1.0f / norm;
        dir = mk(sa * xpix, sa * ypix, ca);
        return true;
    }
    if (L.mode == LENS_LATLONG) {   // latlong_to_dir (386-393)
        const float theta = (uv.y - 0.5f) * PI_F, phi = (uv.x - 0.5f) * PI_F * 2.0f;
        float sp, cp, st, ct;
        sincosf(theta, &st, &ct);
        sincosf(phi, &sp, &cp);
        dir = mk(sp * ct, st, cp * ct);
        return true;
    }
    if (L.mode == LENS_EQUIRECTANGULAR) {   // equirectangular_to_dir (395-401)
        const float ct = (uv.y - 0.5f) * 2.0f;
        const float st = sqrtf(fmaxf(1.0f - ct * ct, 0.0f));
        const float phi = (uv.x - 0.5f) * PI_F * 2.0f;
        float sp, cp;
        sincosf(phi, &sp, &cp);
        dir = mk(sp * st, ct, cp * st);
        return true;
    }
    dir = mk((uv.x - sc.x) * (float)W / focal.x, (uv.y - sc.y) * (float)H / focal.y, 1.0f);
    if (L.mode == LENS_OPENCV || L.mode == LENS_OPENCV_FISHEYE) lens_undistort(L.mode, L.params, dir.x, dir.y);
    return true;
}

SNG_HD void fswap(float& a, float& b) { float t = a; a = b; b = t; }
SNG_HD float aabb_entry(const aabb& b, f3 pos, f3 dir) {
    const float FMAX = 3.402823466e+38f;
    float tmin = (b.lo.x - pos.x) / dir.x;
    float tmax = (b.hi.x - pos.x) / dir.x;
    if (tmin > tmax) fswap(tmin, tmax);
    float tymin = (b.lo.y - pos.y) / dir.y;
    float tymax = (b.hi.y - pos.y) / dir.y;
    if (tymin > tymax) fswap(tymin, tymax);
    if (tmin > tymax || tymin > tmax) return FMAX;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (b.lo.z - pos.z) / dir.z;
    float tzmax = (b.hi.z - pos.z) / dir.z;
    if (tzmin > tzmax) fswap(tzmin, tzmax);
    if (tmin > tzmax || tzmin > tmax) return FMAX;
    if (tzmin > tmin) tmin = tzmin;
    return tmin;
}
// BVH box entry (bounding_box.cuh:163-211 as the reference compiles it: CMakeLists.txt:82 builds
// with --use_fast_math, which turns each slab quotient (b - pos) / dir into (b - pos) * rcp(dir)).
// Restated as (b - pos) * y with y = RN(1 / dir) formed once per ray (inv()): subtract, then multiply
// by the reciprocal -- the reference's operation order, with a correctly rounded reciprocal instead
// of the hardware approximation.  The CPU oracle (sng_oracle.cpp bvh_box_entry) evaluates the same
// expressions, so GPU and oracle traversals agree bit for bit.  The NeRF volume's box tests keep
// aabb_entry (IEEE division) above.
SNG_HD float bvh_box_entry(const aabb& b, f3 pos, f3 y) {
    const float FMAX = 3.402823466e+38f;
    float tmin = (b.lo.x - pos.x) * y.x;
    float tmax = (b.hi.x - pos.x) * y.x;
    if (tmin > tmax) fswap(tmin, tmax);
    float tymin = (b.lo.y - pos.y) * y.y;
    float tymax = (b.hi.y - pos.y) * y.y;
    if (tymin > tymax) fswap(tymin, tymax);
    if (tmin > tymax || tymin > tmax) return FMAX;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (b.lo.z - pos.z) * y.z;
    float tzmax = (b.hi.z - pos.z) * y.z;
    if (tzmin > tzmax) fswap(tzmin, tzmax);
    if (tmin > tzmax || tzmin > tmax) return FMAX;
    if (tzmin > tmin) tmin = tzmin;
    return tmin;
}
// bvh_box_entry, branch-free: with no NaN or infinity in play (slab_fast_ok() for the ray, |coord| <
// 2^40 for the boxes, checked on the host), its swaps are min/max and its two early-outs together
// test every pair (a_min > b_max), i.e. max(mins) > min(maxes); the value returned otherwise is
// max(mins).  Only the sign of a zero result can differ, which no caller observes (the result is
// only compared).  The (lo, hi) pair of each axis is one packed-f32 operand (v_pk_add / v_pk_mul).
typedef float pf2 __attribute__((ext_vector_type(2)));
// sx, sy, sz: the box's (lo, hi) slab of each axis
SNG_HD float slab_entry_fast(pf2 sx, pf2 sy, pf2 sz, f3 pos, f3 y) {
    const float FMAX = 3.402823466e+38f;
    const pf2 tx = (sx - pos.x) * y.x;
    const pf2 ty = (sy - pos.y) * y.y;
    const pf2 tz = (sz - pos.z) * y.z;
    const float tmin = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
    const float tmax = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
    return tmin > tmax ? FMAX : tmin;
}
SNG_HD float aabb_entry_fast(const aabb& b, f3 pos, f3 y) {
    return slab_entry_fast(pf2{b.lo.x, b.hi.x}, pf2{b.lo.y, b.hi.y}, pf2{b.lo.z, b.hi.z}, pos, y);
}
constexpr float SLAB_FAST_MAX_COORD = 1099511627776.0f;   // 2^40
SNG_HD bool slab_fast_ok(f3 pos, f3 dir) {
    const float lo = 8.673617379884035e-19f /* 2^-60 */, hi = 1.152921504606846976e18f /* 2^60 */;
    const float ax = fabsf(dir.x), ay = fabsf(dir.y), az = fabsf(dir.z);
    return ax >= lo && ax <= hi && ay >= lo && ay <= hi && az >= lo && az <= hi && fabsf(pos.x) < SLAB_FAST_MAX_COORD &&
           fabsf(pos.y) < SLAB_FAST_MAX_COORD && fabsf(pos.z) < SLAB_FAST_MAX_COORD;
}
SNG_HD bool aabb_contains(const aabb& b, f3 p) {
    return p.x >= b.lo.x && p.x <= b.hi.x && p.y >= b.lo.y && p.y <= b.hi.y && p.z >= b.lo.z && p.z <= b.hi.z;
}

// ---- stepping: nerf_device.cuh:266-441 ----------------------------------------
SNG_HD float warp_dt(float dt) {
    float max_stepsize = MIN_STEP * (1 << (N_CASCADES - 1));
    return (dt - MIN_STEP) / (max_stepsize - MIN_STEP);
}
SNG_HD float unwarp_dt(float dt) {
    float max_stepsize = MIN_STEP * (1 << (N_CASCADES - 1));
    return dt * (max_stepsize - MIN_STEP) + MIN_STEP;
}
SNG_HD float to_stepping_space(float t, float cone) {
    if (cone <= 1e-5f) return div_by(t, MIN_STEP, INV_MIN_STEP);   // == t / MIN_STEP
    float log1p_c = sng_logf(1.0f + cone);
    float a = (sng_logf(MIN_STEP) - sng_logf(log1p_c)) / log1p_c;
    float b = (sng_logf(MAX_STEP) - sng_logf(log1p_c)) / log1p_c;
    float at = sng_expf(a * log1p_c);
    float bt = sng_expf(b * log1p_c);
    if (t <= at) return (t - at) / MIN_STEP + a;
    else if (t <= bt) return sng_logf(t) / log1p_c;
    else return (t - bt) / MAX_STEP + b;
}
SNG_HD float from_stepping_space(float n, float cone) {
    if (cone <= 1e-5f) return n * MIN_STEP;
    float log1p_c = sng_logf(1.0f + cone);
    float a = (sng_logf(MIN_STEP) - sng_logf(log1p_c)) / log1p_c;
    float b = (sng_logf(MAX_STEP) - sng_logf(log1p_c)) / log1p_c;
    float at = sng_expf(a * log1p_c);
    float bt = sng_expf(b * log1p_c);
    if (n <= a) return (n - a) * MIN_STEP + at;
    else if (n <= b) return sng_expf(n * log1p_c);
    else return (n - b) * MAX_STEP + bt;
}
SNG_HD float advance_n_steps(float t, float cone, float n) { return from_stepping_space(to_stepping_space(t, cone) + n, cone); }
// The same three functions with their cone-only constants (log1p(c), a, b, e^a, e^b) computed once per
// frame by step_space() -- identical float expressions, so identical bits; the marchers' inner loops
// then spend one log or exp per conversion instead of seven.
struct StepSpace {
    float cone, log1p_c, a, b, at, bt, rlog1p_c;   // rlog1p_c = RN(1 / log1p_c)
};
SNG_HD StepSpace step_space(float cone) {
    StepSpace k{};
    k.cone = cone;
    if (cone <= 1e-5f) return k;
    k.log1p_c = sng_logf(1.0f + cone);
    k.a = (sng_logf(MIN_STEP) - sng_logf(k.log1p_c)) / k.log1p_c;
    k.b = (sng_logf(MAX_STEP) - sng_logf(k.log1p_c)) / k.log1p_c;
    k.at = sng_expf(k.a * k.log1p_c);
    k.bt = sng_expf(k.b * k.log1p_c);
    k.rlog1p_c = recip_rn(k.log1p_c);
    return k;
}
// The per-trip log / exp of the cone-stepping conversions below: the deterministic sng_logf / sng_expf (the NeRF
// marcher and its schedule, equal on host and device), or -- in a translation unit that defines
// SNG_FAST_TRANSCENDENTALS before including this header (mesh.hip: the shadow marches of the raytracer and the NeRF
// shadow pass, in the reference's --use_fast_math model, where logf / expf are __logf / __expf) -- the hardware forms.
#if defined(SNG_FAST_TRANSCENDENTALS) && defined(__HIP_DEVICE_COMPILE__)
#define SNG_STEP_EXPF __expf
#define SNG_STEP_LOGF __logf
#else
#define SNG_STEP_EXPF sng_expf
#define SNG_STEP_LOGF sng_logf
#endif
// The two constant divisions as exact reciprocal forms: x / MIN_STEP is div_by (see above), and since
// MAX_STEP == MIN_STEP * 2^10 exactly, x / MAX_STEP == (x / MIN_STEP) * 2^-10 (power-of-two scaling
// commutes with rounding in the normal range).
SNG_HD float to_stepping_space(float t, const StepSpace& k) {
    if (k.cone <= 1e-5f) return div_by(t, MIN_STEP, INV_MIN_STEP);
    if (t <= k.at) return div_by(t - k.at, MIN_STEP, INV_MIN_STEP) + k.a;
    else if (t <= k.bt) return div_by(SNG_STEP_LOGF(t), k.log1p_c, k.rlog1p_c);   // the IEEE quotient (Markstein, as div_by above)
    else return div_by(t - k.bt, MIN_STEP, INV_MIN_STEP) * (1.0f / 1024.0f) + k.b;
}
static_assert(MAX_STEP == MIN_STEP * 1024.0f, "MAX_STEP / MIN_STEP must be 2^10");
SNG_HD float from_stepping_space(float n, const StepSpace& k) {
    if (k.cone <= 1e-5f) return n * MIN_STEP;
    if (n <= k.a) return (n - k.a) * MIN_STEP + k.at;
    else if (n <= k.b) return SNG_STEP_EXPF(n * k.log1p_c);
    else return (n - k.b) * MAX_STEP + k.bt;
}
SNG_HD float advance_n_steps(float t, const StepSpace& k, float n) { return from_stepping_space(to_stepping_space(t, k) + n, k); }
SNG_HD float calc_dt(float t, const StepSpace& k) { return advance_n_steps(t, k, 1.0f) - t; }
SNG_HD float calc_dt(float t, float cone) { return advance_n_steps(t, cone, 1.0f) - t; }

SNG_HD float distance_to_next_voxel(f3 pos, f3 dir, f3 idir, float res) {
    f3 p = res * (pos - 0.5f);
    float tx = (floorf(p.x + 0.5f + 0.5f * sgnf(dir.x)) - p.x) * idir.x;
    float ty = (floorf(p.y + 0.5f + 0.5f * sgnf(dir.y)) - p.y) * idir.y;
    float tz = (floorf(p.z + 0.5f + 0.5f * sgnf(dir.z)) - p.z) * idir.z;
    float t = fminf(fminf(tx, ty), tz);
    return fmaxf(t / res, 0.0f);
}
SNG_HD float advance_to_next_voxel(float t, float cone, f3 pos, f3 dir, f3 idir, uint32_t mip) {
    float res = scalbnf((float)GRID_SIZE, -(int)mip);
    float t_target = t + distance_to_next_voxel(pos, dir, idir, res);
    t = to_stepping_space(t, cone);
    t_target = to_stepping_space(t_target, cone);
    return from_stepping_space(t + ceilf(fmaxf(t_target - t, 0.5f)), cone);
}
// distance_to_next_voxel with res = 128 * 2^-mip; its final t / res is the exact power-of-two scaling
// t * 2^(mip - 7)
SNG_HD float distance_to_next_voxel_mip(f3 pos, f3 dir, f3 idir, uint32_t mip) {
    const float res = scalbnf((float)GRID_SIZE, -(int)mip);
    f3 p = res * (pos - 0.5f);
    float tx = (floorf(p.x + 0.5f + 0.5f * sgnf(dir.x)) - p.x) * idir.x;
    float ty = (floorf(p.y + 0.5f + 0.5f * sgnf(dir.y)) - p.y) * idir.y;
    float tz = (floorf(p.z + 0.5f + 0.5f * sgnf(dir.z)) - p.z) * idir.z;
    float t = fminf(fminf(tx, ty), tz);
    return fmaxf(t * scalbnf(1.0f / (float)GRID_SIZE, (int)mip), 0.0f);
}
SNG_HD float advance_to_next_voxel(float t, const StepSpace& k, f3 pos, f3 dir, f3 idir, uint32_t mip) {
    float t_target = t + distance_to_next_voxel_mip(pos, dir, idir, mip);
    t = to_stepping_space(t, k);
    t_target = to_stepping_space(t_target, k);
    return from_stepping_space(t + ceilf(fmaxf(t_target - t, 0.5f)), k);
}
SNG_HD uint32_t mip_from_pos(f3 pos, uint32_t max_cascade) {
    int exponent;
    f3 d = pos - 0.5f;
    float maxval = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    frexpf(maxval, &exponent);
    int e = exponent + 1;
    e = e < 0 ? 0 : e;
    return (uint32_t)(e > (int)max_cascade ? (int)max_cascade : e);
}
SNG_HD uint32_t cascaded_grid_idx_at(f3 pos, uint32_t mip) {
    float mip_scale = scalbnf(1.0f, -(int)mip);
    pos = pos - splat(0.5f);
    pos = pos * mip_scale;
    pos = pos + splat(0.5f);
    f3 f = pos * (float)GRID_SIZE;
    int ix = (int)f.x, iy = (int)f.y, iz = (int)f.z;
    if (ix < 0 || ix >= (int)GRID_SIZE || iy < 0 || iy >= (int)GRID_SIZE || iz < 0 || iz >= (int)GRID_SIZE) return 0xFFFFFFFFu;
    return morton3D(ix, iy, iz);
}
SNG_HD bool occupied_at(f3 pos, const uint8_t* bf, uint32_t mip) {
    uint32_t idx = cascaded_grid_idx_at(pos, mip);
    if (idx == 0xFFFFFFFFu) return false;
    return bf[idx / 8 + (GRID_CELLS * mip) / 8] & (1 << (idx % 8));
}
// occupied_at through the x-fastest rows of every cascade (Volume::occ_lin_all): the same cell (cascaded_grid_idx_at's
// float expressions), the same bit, without the Morton encoding's twelve quarter-rate multiplies
SNG_HD bool occupied_at_lin(f3 pos, const uint32_t* occ, uint32_t mip) {
    float mip_scale = scalbnf(1.0f, -(int)mip);
    pos = pos - splat(0.5f);
    pos = pos * mip_scale;
    pos = pos + splat(0.5f);
    f3 f = pos * (float)GRID_SIZE;
    int ix = (int)f.x, iy = (int)f.y, iz = (int)f.z;
    if (ix < 0 || ix >= (int)GRID_SIZE || iy < 0 || iy >= (int)GRID_SIZE || iz < 0 || iz >= (int)GRID_SIZE) return false;
    const uint32_t w = ((mip * GRID_SIZE + (uint32_t)iz) * GRID_SIZE + (uint32_t)iy) * (GRID_SIZE / 32) + ((uint32_t)ix >> 5);
    return (occ[w] >> (ix & 31)) & 1u;
}

// Volume description shared by the marcher, shadow rays and the path tracer.
struct Volume {
    aabb render_aabb;    // m_render_aabb
    aabb train_aabb;     // m_aabb (warp_position)
    m3 to_local;         // m_render_aabb_to_local
    int to_local_identity;
    float cone;          // cone_angle_constant
    uint32_t max_mip;    // max_cascade
    float min_transmittance;
    const uint8_t* bitfield;
    const uint32_t* occ_linear;  // mip-0 occupancy as x-fastest bit rows (same bits as the Morton bitfield)
    const uint32_t* occ_lin_all; // every cascade's occupancy in that layout, [mip][z][y][x / 32] (nullptr: Morton lookups)
    int linear;                  // cone == 0 && max_mip == 0: the exact fast marcher applies
    StepSpace ss;                // step_space(cone)
    // mip-0 occupancy as 8^3-cell bricks (same bits, OccBrick layout below), small enough to stage in LDS:
    // the linear marchers' loops then make no global load.  occ_brick_words == 0: not available.
    const uint32_t* occ_brick;
    uint32_t occ_brick_words;
    const uint32_t* occ_brick_g;  // the same blob in global memory whenever it is built (its size need not be known on the host):
                                  // the training generator reads it through L1 / L2 when it cannot stage it (nullptr: not built)
};
SNG_HD bool occupied_vol(f3 pos, const Volume& vol, uint32_t mip) {
    return vol.occ_lin_all ? occupied_at_lin(pos, vol.occ_lin_all, mip) : occupied_at(pos, vol.bitfield, mip);
}
// OccBrick layout (u32 words): [0, 128) = 4096-bit "dilated" brick mask (bit b: an occupied cell lies within one
// cell of brick b -- the conservative test of path_last_occupied_t), [128, 2176) = u16 slot per brick
// b = (iz/8)*256 + (iy/8)*16 + ix/8 (0xffff: no occupied cell), then 16 words per occupied brick: word
// (iz%8)*2 + (iy%8)/4, bit (iy%4)*8 + ix%8.
constexpr uint32_t OCC_BRICK_TAB = 128;
constexpr uint32_t OCC_BRICK_HDR_WORDS = OCC_BRICK_TAB + 2048;
constexpr uint32_t OCC_BRICK_CAP_WORDS = OCC_BRICK_HDR_WORDS + 4096 * 16;
SNG_HD f3 to_local(const Volume& v, f3 p) { return v.to_local_identity ? p : mul(v.to_local, p); }

// Exact specialisation of if_unoccupied_advance_to_next_occupied_voxel<false> for unit-cube
// scenes (cone_angle_constant == 0, max_cascade == 0): every float operation of the general
// path is kept (mip clamps to 0, scalbnf(.,0) is the identity, /128 is an exact *2^-7), only the
// divisions by MIN_STEP use div_by and the Morton bitfield lookup uses an equivalent linear copy.
SNG_HD bool occupied_linear(f3 pos, const uint32_t* occ) {
    f3 q = ((pos - splat(0.5f)) + splat(0.5f)) * (float)GRID_SIZE;   // cascaded_grid_idx_at, mip 0
    int ix = (int)q.x, iy = (int)q.y, iz = (int)q.z;
    if (ix < 0 || ix >= (int)GRID_SIZE || iy < 0 || iy >= (int)GRID_SIZE || iz < 0 || iz >= (int)GRID_SIZE) return false;
    return (occ[((uint32_t)iz * GRID_SIZE + (uint32_t)iy) * (GRID_SIZE / 32) + ((uint32_t)ix >> 5)] >> (ix & 31)) & 1u;
}
// occupied_linear with the last loaded occupancy word kept in registers: the trips of a march mostly stay
// in one 32-cell x-row word (4-5 samples per occupied cell, x steps of the DDA), and those need no load on
// the march's dependent chain.  Same bits as occupied_linear.
struct OccCache {
    uint32_t w = 0xffffffffu, bits = 0u;
};
SNG_HD bool occupied_linear_c(f3 pos, const uint32_t* occ, OccCache& c) {
    f3 q = ((pos - splat(0.5f)) + splat(0.5f)) * (float)GRID_SIZE;   // cascaded_grid_idx_at, mip 0
    int ix = (int)q.x, iy = (int)q.y, iz = (int)q.z;
    if (ix < 0 || ix >= (int)GRID_SIZE || iy < 0 || iy >= (int)GRID_SIZE || iz < 0 || iz >= (int)GRID_SIZE) return false;
    const uint32_t w = ((uint32_t)iz * GRID_SIZE + (uint32_t)iy) * (GRID_SIZE / 32) + ((uint32_t)ix >> 5);
    if (w != c.w) {
        c.w = w;
        c.bits = occ[w];
    }
    return (c.bits >> (ix & 31)) & 1u;
}
#if defined(__HIP__)
// occupied_linear through the LDS copy of the OccBrick blob, with the last 32-cell group in registers
__device__ __forceinline__ bool occupied_brick_c(f3 pos, const uint32_t* lds, OccCache& c) {
    f3 q = ((pos - splat(0.5f)) + splat(0.5f)) * (float)GRID_SIZE;   // cascaded_grid_idx_at, mip 0
    int ix = (int)q.x, iy = (int)q.y, iz = (int)q.z;
    if (ix < 0 || ix >= (int)GRID_SIZE || iy < 0 || iy >= (int)GRID_SIZE || iz < 0 || iz >= (int)GRID_SIZE) return false;
    const uint32_t b = ((uint32_t)iz >> 3) * 256u + ((uint32_t)iy >> 3) * 16u + ((uint32_t)ix >> 3);
    const uint32_t sub = ((uint32_t)iz & 7u) * 2u + (((uint32_t)iy & 7u) >> 2);
    const uint32_t key = (b << 4) | sub;
    if (key != c.w) {
        c.w = key;
        const uint32_t slot = reinterpret_cast<const uint16_t*>(lds + OCC_BRICK_TAB)[b];
        c.bits = slot == 0xffffu ? 0u : lds[OCC_BRICK_HDR_WORDS + slot * 16u + sub];
    }
    return (c.bits >> ((((uint32_t)iy & 3u) << 3) | ((uint32_t)ix & 7u))) & 1u;
}
// the same bit without branches: both LDS reads every call (the second from a clamped slot), the cell's
// in-grid test and the brick's occupancy folded into the result -- for marcher loops whose lanes diverge
__device__ __forceinline__ bool occupied_brick_nb(f3 pos, const uint32_t* lds) {
    f3 q = ((pos - splat(0.5f)) + splat(0.5f)) * (float)GRID_SIZE;   // cascaded_grid_idx_at, mip 0
    const int ix = (int)q.x, iy = (int)q.y, iz = (int)q.z;
    const bool in = (uint32_t)ix < GRID_SIZE && (uint32_t)iy < GRID_SIZE && (uint32_t)iz < GRID_SIZE;
    const uint32_t ux = (uint32_t)ix & (GRID_SIZE - 1), uy = (uint32_t)iy & (GRID_SIZE - 1), uz = (uint32_t)iz & (GRID_SIZE - 1);
    const uint32_t b = (uz >> 3) * 256u + (uy >> 3) * 16u + (ux >> 3);
    const uint32_t sub = (uz & 7u) * 2u + ((uy & 7u) >> 2);
    const uint32_t slot = reinterpret_cast<const uint16_t*>(lds + OCC_BRICK_TAB)[b];
    const uint32_t empty = (uint32_t)(slot == 0xffffu);
    const uint32_t w = lds[OCC_BRICK_HDR_WORDS + (slot & (empty - 1u)) * 16u + sub];   // empty brick: slot 0's word, masked
    const uint32_t bit = (w >> (((uy & 3u) << 3) | (ux & 7u))) & 1u;
    return (bit & (uint32_t)in & (empty ^ 1u)) != 0u;   // bit operations: no short-circuit branches
}
// aabb_contains without short-circuit branches: p >= lo <=> fl(p - lo) >= 0 and p <= hi <=> fl(hi - p) >= 0 (IEEE
// subtraction keeps the sign and is 0 only for equal operands); p is finite in the marchers
__device__ __forceinline__ bool aabb_contains_nb(const aabb& b, f3 p) {
    const float m0 = fminf(fminf(p.x - b.lo.x, p.y - b.lo.y), p.z - b.lo.z);
    const float m1 = fminf(fminf(b.hi.x - p.x, b.hi.y - p.y), b.hi.z - p.z);
    return fminf(m0, m1) >= 0.0f;
}
// The largest t at which the ray o + t d (t >= t0) can still be in an occupied mip-0 cell, or -1 when it
// cannot at all: a walk over the 16^3 bricks of the unit cube that keeps the exit t of the last brick whose
// dilated mask bit is set.  Conservative for the exact marchers: their float positions stay within ~1e-6 of
// the line and a brick's mask bit covers every occupied cell within one cell (1/128) of it, so a marcher
// past the returned t only ever meets unoccupied cells until it leaves the volume -- stopping there drops
// no sample.  (Unit-cube occupancy, identity render_aabb_to_local: the linear marchers.)
__device__ __forceinline__ float path_last_occupied_t(f3 o, f3 d, f3 idir, float t0, const uint32_t* lds) {
    // the line's span inside [0,1]^3, from t0
    float ta = t0, tb = 3.0e38f;
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z}, ii[3] = {idir.x, idir.y, idir.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (dd[k] == 0.0f) {
            if (oo[k] < 0.0f || oo[k] > 1.0f) return -1.0f;
        } else {
            const float u = (0.0f - oo[k]) * ii[k], v = (1.0f - oo[k]) * ii[k];
            ta = fmaxf(ta, fminf(u, v));
            tb = fminf(tb, fmaxf(u, v));
        }
    }
    if (!(ta <= tb)) return -1.0f;
    const float tm = 0.5f * (ta + tb);   // a point safely inside for the start brick, then walk from ta
    int b[3], st[3];
    float tmax[3], tdel[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float pk = oo[k] + dd[k] * ta;
        int c = (int)floorf(pk * 16.0f);
        c = c < 0 ? 0 : (c > 15 ? 15 : c);
        b[k] = c;
        if (dd[k] > 0.0f) { st[k] = 1; tmax[k] = ((float)(c + 1) * 0.0625f - oo[k]) * ii[k]; tdel[k] = 0.0625f * ii[k]; }
        else if (dd[k] < 0.0f) { st[k] = -1; tmax[k] = ((float)c * 0.0625f - oo[k]) * ii[k]; tdel[k] = -0.0625f * ii[k]; }
        else { st[k] = 0; tmax[k] = 3.0e38f; tdel[k] = 3.0e38f; }
    }
    (void)tm;
    float last = -1.0f;
#pragma unroll 1
    for (int n = 0; n < 48; ++n) {
        const uint32_t bi = (uint32_t)b[2] * 256u + (uint32_t)b[1] * 16u + (uint32_t)b[0];
        const float tx = fminf(fminf(tmax[0], tmax[1]), tmax[2]);
        if ((lds[bi >> 5] >> (bi & 31u)) & 1u) last = fminf(tx, tb);
        if (tx >= tb) break;
        const int k = tmax[0] == tx ? 0 : (tmax[1] == tx ? 1 : 2);
        b[k] += st[k];
        if (b[k] < 0 || b[k] > 15) break;
        tmax[k] += tdel[k];
    }
    return last < 0.0f ? -1.0f : last * 1.00001f + 1e-5f;
}
// copy the OccBrick blob into LDS (every thread of the block; words padded to a multiple of 4)
__device__ __forceinline__ void stage_occ_brick(uint32_t* lds, const uint32_t* g, uint32_t words) {
    for (uint32_t k = threadIdx.x * 4u; k < words; k += blockDim.x * 4u) *reinterpret_cast<uint4*>(lds + k) = *reinterpret_cast<const uint4*>(g + k);
    __syncthreads();
}
#endif
// advance_to_next_voxel(mip 0) with distance_to_next_voxel(res = 128), cone == 0
SNG_HD float dda_step_linear(float t, f3 pos, f3 idir, f3 hs /* 0.5*sign(d) */) {
    const f3 p = (float)GRID_SIZE * (pos - 0.5f);
    const float tx = (floorf(p.x + 0.5f + hs.x) - p.x) * idir.x;
    const float ty = (floorf(p.y + 0.5f + hs.y) - p.y) * idir.y;
    const float tz = (floorf(p.z + 0.5f + hs.z) - p.z) * idir.z;
    const float dist = fmaxf(fminf(fminf(tx, ty), tz) * (1.0f / (float)GRID_SIZE), 0.0f);
    const float t_target = t + dist;
    const float ts = to_stepping_space(t, 0.0f);
    const float tts = to_stepping_space(t_target, 0.0f);
    return (ts + ceilf(fmaxf(tts - ts, 0.5f))) * MIN_STEP;
}
SNG_HD float advance_to_occupied_linear(float t, f3 o, f3 d, f3 idir, f3 hs /* 0.5*sign(d) */, const Volume& vol) {
    OccCache oc;
    while (true) {
        const f3 pos = o + d * t;
        if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) return MAX_DEPTH;
        if (occupied_linear_c(pos, vol.occ_linear, oc)) return t;
        t = dda_step_linear(t, pos, idir, hs);
    }
}
SNG_HD f3 half_sign(f3 d) { return {0.5f * sgnf(d.x), 0.5f * sgnf(d.y), 0.5f * sgnf(d.z)}; }

// if_unoccupied_advance_to_next_occupied_voxel<false>: nerf_device.cuh:462-495
SNG_HD float advance_to_occupied(float t, float cone, f3 o, f3 d, f3 idir, uint32_t min_mip, uint32_t max_mip, const Volume& vol) {
    if (vol.linear && vol.bitfield && min_mip == 0 && max_mip == 0 && cone <= 1e-5f) return advance_to_occupied_linear(t, o, d, idir, half_sign(d), vol);
    while (true) {
        f3 pos = o + d * t;
        if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) return MAX_DEPTH;
        uint32_t mip = mip_from_pos(pos, N_CASCADES - 1);
        mip = mip < min_mip ? min_mip : mip;
        mip = mip > max_mip ? max_mip : mip;
        if (!vol.bitfield || occupied_vol(pos, vol, mip)) return t;
        while (mip < max_mip && !occupied_vol(pos, vol, mip + 1)) ++mip;
        t = advance_to_next_voxel(t, cone, pos, d, idir, mip);
    }
}

// ONE trip of the general advance_to_occupied loop above: returns true when t is final (an occupied
// voxel, or MAX_DEPTH when the ray left the render aabb), else t moved to the next voxel boundary.
// Marchers that take several samples loop over it "flattened" (each trip one DDA step or one
// sample), so a lane costs its own trips instead of the wave's slowest walk per sample.
SNG_HD bool occ_step(float& t, const StepSpace& cone, f3 o, f3 d, f3 idir, uint32_t min_mip, uint32_t max_mip, const Volume& vol) {
    const f3 pos = o + d * t;
    if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) { t = MAX_DEPTH; return true; }
    uint32_t mip = mip_from_pos(pos, N_CASCADES - 1);
    mip = mip < min_mip ? min_mip : mip;
    mip = mip > max_mip ? max_mip : mip;
    if (!vol.bitfield || occupied_vol(pos, vol, mip)) return true;
    // (loading every cascade's byte up front, to save the escalation's dependent loads, measured slower:
    // C4 14.7 -> 13.7 frames/s -- empty-space trips rarely escalate more than once)
    while (mip < max_mip && !occupied_vol(pos, vol, mip + 1)) ++mip;
    t = advance_to_next_voxel(t, cone, pos, d, idir, mip);
    return false;
}

// ---- scrambled Sobol: random_val.cuh:162-325 ---------------------------------
SNG_HD uint32_t reverse_bits(uint32_t x) {
    x = (((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1));
    x = (((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2));
    x = (((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4));
    x = (((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8));
    return ((x >> 16) | (x << 16));
}
SNG_HD uint32_t lk_permutation(uint32_t x, uint32_t seed) {
    x += seed;
    x ^= x * 0x6c50b47cu;
    x ^= x * 0xb82f1e52u;
    x ^= x * 0xc7afe638u;
    x ^= x * 0x8d22f6e6u;
    return x;
}
SNG_HD uint32_t nested_scramble(uint32_t x, uint32_t seed) { return reverse_bits(lk_permutation(reverse_bits(x), seed)); }
SNG_HD uint32_t hash_combine(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
// Sobol dimension 0 is the bit reversal (van der Corput); dimension 1 uses the
// Pascal-matrix directions 0x80000000 ^ ... generated as (d_{k} = d_{k-1} ^ d_{k-1}>>1).
SNG_HD uint32_t sobol_dim0(uint32_t index) { return reverse_bits(index); }
SNG_HD uint32_t sobol_dim1(uint32_t index) {
    uint32_t X = 0, d = 0x80000000u;
    for (uint32_t bit = 0; bit < 32; ++bit) {
        if ((index >> bit) & 1u) X ^= d;
        d ^= d >> 1;
    }
    return X;
}
SNG_HD float ld_random_val0(uint32_t index, uint32_t seed) {
    constexpr float S = float(1.0 / (1ull << 32));
    index = nested_scramble(index, seed);
    return (float)nested_scramble(sobol_dim0(index), hash_combine(seed, 0)) * S;
}
SNG_HD f2 ld_random_val_2d(uint32_t index, uint32_t seed) {
    constexpr float S = float(1.0 / (1ull << 32));
    index = nested_scramble(index, seed);
    return {(float)nested_scramble(sobol_dim0(index), hash_combine(seed, 0)) * S,
            (float)nested_scramble(sobol_dim1(index), hash_combine(seed, 1)) * S};
}
SNG_HD f2 ld_random_pixel_offset(uint32_t spp) {
    f2 a = ld_random_val_2d(0, 0xdeadbeefu), b = ld_random_val_2d(spp, 0xdeadbeefu);
    return {fractf_(0.5f - a.x + b.x), fractf_(0.5f - a.y + b.y)};
}

// ---- cuRAND XORWOW state (curand_kernel.h), SoA-friendly ----------------------
struct Xorwow { uint32_t v0, v1, v2, v3, v4, d; };
SNG_HD uint32_t xorwow_next(Xorwow& s) {
    uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1; s.v1 = s.v2; s.v2 = s.v3; s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v4 + s.d;
}
SNG_HD float curand_uniform(Xorwow& s) {
    const float INV = 2.3283064e-10f;  // CURAND_2POW32_INV
    return (float)xorwow_next(s) * INV + (INV / 2.0f);
}

// ---- scene records ------------------------------------------------------------
struct BvhNode { float lo[3], hi[3]; int left, right; };   // TriangleBvhNode (32 B)
struct Tri { f3 a, b, c; };                                 // Triangle (36 B)
// Traversal layout of the same BVH (host_scene.cpp wide_bvh): one 64-B record per INNER node holding
// both children's boxes and references, so visiting a node is four 16-B loads and a leaf needs none
// (its triangle range travels in the stack entry).  Each box is stored slab by slab
// (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z) so that an axis is one packed-f32 register pair.
// ref >= 0: inner record index; ref < 0: leaf, ~ref = first_triangle | triangle_count << 24.
// Records are 80 B apart (one 16-B pad slot): ds_read_b128 serves 16 lanes per LDS cycle from the 16 slots of a
// 256-B bank row, and the q-th load of record i sits in slot (5 i + q) mod 16 -- distinct for 16 consecutive
// records -- where a 64-B stride put every record's q-th load in one of only 4 slots (up to 4-way conflicts
// between lanes walking different records).
struct alignas(16) BvhWide {
    float s0[6], s1[6];
    int ref0, ref1, pad0, pad1;
    int pad2[4];
};
constexpr uint32_t WIDE_MAX_BEGIN = 1u << 24, WIDE_MAX_COUNT = 127u;
constexpr int WIDE_DONE = (int)0x80000000;   // traversal sentinel; wide_bvh never encodes a leaf as ~0x7FFFFFFF
// Traversal copy of a triangle (host_scene.cpp upload_scene): a, e1 = b - a, e2 = c - a and n = cross(e1, e2),
// the values Triangle::ray_intersect (triangle.cuh:45-59) forms first, evaluated once on the host with
// the same float operations, so the test reads them instead of recomputing them per ray.  48 B, three
// 16-B loads: v = {a.x a.y a.z e1.x | e1.y e1.z e2.x e2.y | e2.z n.x n.y n.z}.
struct alignas(16) TriT { float v[12]; };
SNG_HD TriT make_trit(const Tri& t) {
    const f3 e1 = t.b - t.a, e2 = t.c - t.a, n = cross(e1, e2);
    return TriT{{t.a.x, t.a.y, t.a.z, e1.x, e1.y, e1.z, e2.x, e2.y, e2.z, n.x, n.y, n.z}};
}
struct ObjectGpu {                                           // ObjectTransform + hoisted inverse
    const BvhNode* nodes;
    const Tri* tris;                // the mesh's triangles (hit normals and perturb frames)
    const TriT* trit;               // their traversal copies
    m3 rot;
    f3 pos;
    float scale;
    int mat_id;
    m3 world_to_obj;   // (I/scale) * inverse(rot), triangle_bvh.cu:313-319
    int fast_slab;     // every BVH box coordinate < 2^40 in magnitude: aabb_entry_fast is exact
    uint32_t lds_nodes, lds_trit;   // byte offsets of this object's arrays in the scene blob
    const BvhWide* wide;            // traversal layout (nullptr: walk the TriangleBvhNode array)
    uint32_t lds_wide;              // its byte offset in the scene blob
    int root_ref;                   // stack entry of the root
};
struct LightGpu { f3 pos; float intensity; float size; int type; };
struct MaterialGpu { f3 ka, kd, ks; float n, rg, spec_angle; int type; };

}  // namespace sng
