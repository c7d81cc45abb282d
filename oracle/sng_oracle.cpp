/*
 * sng_oracle.cpp -- CPU ORACLE for the SyNeRFgine render hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product
 * (synerfgine_amd / libsng_hip.so) never links or calls it.
 *
 * A deliberately plain, scalar restatement of the reference algorithm,
 * structured like the reference (wavefront trace_alt loop, per-pixel kernels
 * as loops) so that it can be read side by side with the cited lines.  All
 * citations are relative to the reference root (/root/reference).
 *
 * Float semantics: IEEE fp32 (built with -ffp-contract=off, no fast-math),
 * except where the reference evaluates in double through implicit promotion
 * (cited inline).  The reference itself builds with --use_fast_math
 * (CMakeLists.txt:82), so results agree with it within the per-pixel
 * tolerance stated in DESIGN.md, not bitwise.
 *
 * Parity: PARTIALLY PINNED -- see sng_oracle.h header and DESIGN.md.
 */
#include "sng_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <stack>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

/* ------------------------------------------------------------------------- */
/* small vector math, mirroring tcnn's vec/mat semantics [tcnn, unvendored]    */
/* ------------------------------------------------------------------------- */
struct V2 { float x, y; };
struct V3 { float x, y, z; float& operator[](int i) { return (&x)[i]; } float operator[](int i) const { return (&x)[i]; } };
struct V4 { float x, y, z, w; };
struct M3 { V3 c[3]; };   /* column-major */
struct M43 { V3 c[4]; };  /* column-major, c[3] = translation */

inline V3 v3(float x, float y, float z) { return {x, y, z}; }
inline V3 v3s(float s) { return {s, s, s}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 operator/(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 operator+(V3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }
inline V3 operator-(V3 a, float s) { return {a.x - s, a.y - s, a.z - s}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float length2(V3 a) { return dot(a, a); }
inline float length(V3 a) { return std::sqrt(dot(a, a)); }
/* tcnn normalize(): guards zero length by returning the first unit vector [tcnn, unvendored] */
inline V3 normalize(V3 a) {
    float l = length(a);
    if (!(l > 0.0f)) return {1.0f, 0.0f, 0.0f};
    return a / l;
}
inline float vmax(V3 a) { return std::max(std::max(a.x, a.y), a.z); }
inline V3 vmin3(V3 a, V3 b) { return {std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)}; }
inline V3 vmax3(V3 a, V3 b) { return {std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)}; }
/* tmat * tvec: result = 0; result += m[i] * v[i] (column accumulation) [tcnn] */
inline V3 mul(const M3& m, V3 v) {
    V3 r = v3s(0.0f);
    r = r + m.c[0] * v.x;
    r = r + m.c[1] * v.y;
    r = r + m.c[2] * v.z;
    return r;
}
inline M3 mulm(const M3& a, const M3& b) { return {{mul(a, b.c[0]), mul(a, b.c[1]), mul(a, b.c[2])}}; }
inline M3 m3_load(const float* p) { return {{v3(p[0], p[1], p[2]), v3(p[3], p[4], p[5]), v3(p[6], p[7], p[8])}}; }
inline M43 m43_load(const float* p) { return {{v3(p[0], p[1], p[2]), v3(p[3], p[4], p[5]), v3(p[6], p[7], p[8]), v3(p[9], p[10], p[11])}}; }
inline M3 m3_of(const M43& m) { return {{m.c[0], m.c[1], m.c[2]}}; }
inline bool m3_is_identity(const M3& m) {
    return m.c[0].x == 1 && m.c[0].y == 0 && m.c[0].z == 0 && m.c[1].x == 0 && m.c[1].y == 1 && m.c[1].z == 0 &&
           m.c[2].x == 0 && m.c[2].y == 0 && m.c[2].z == 1;
}
/* glm-style adjugate inverse used by tcnn::inverse(tmat3) [tcnn, unvendored] */
inline M3 inverse(const M3& m0) {
    auto m = [&](int i, int j) { return m0.c[i][j]; };
    float det = m(0, 0) * (m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) - m(1, 0) * (m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2)) +
                m(2, 0) * (m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2));
    M3 r;
    r.c[0][0] = +(m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2));
    r.c[1][0] = -(m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2));
    r.c[2][0] = +(m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1));
    r.c[0][1] = -(m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2));
    r.c[1][1] = +(m(0, 0) * m(2, 2) - m(2, 0) * m(0, 2));
    r.c[2][1] = -(m(0, 0) * m(2, 1) - m(2, 0) * m(0, 1));
    r.c[0][2] = +(m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2));
    r.c[1][2] = -(m(0, 0) * m(1, 2) - m(1, 0) * m(0, 2));
    r.c[2][2] = +(m(0, 0) * m(1, 1) - m(1, 0) * m(0, 1));
    for (int i = 0; i < 3; ++i) r.c[i] = r.c[i] / det;
    return r;
}

inline float fractf(float x) { return x - std::floor(x); } /* random_val.cuh:82-84 */
/* exp / log as the device computes them (synerfgine_amd/csrc/sng_math.h sng_expf/sng_logf):
 * the reference's --use_fast_math __expf/__logf are approximations, so CPU and GPU share one
 * deterministic <= ~1 ulp formulation wherever a marching/termination decision depends on it. */
inline float det_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935f) return HUGE_VALF;
    if (x < -103.972084f) return 0.0f;
    const float n = std::rint(x * 1.44269502f);
    float r = std::fma(n, -0.693145752f, x);
    r = std::fma(n, -1.42860677e-06f, r);
    float p = 1.98412698e-04f;
    p = std::fma(p, r, 1.38888889e-03f);
    p = std::fma(p, r, 8.33333377e-03f);
    p = std::fma(p, r, 4.16666679e-02f);
    p = std::fma(p, r, 1.66666672e-01f);
    p = std::fma(p, r, 0.5f);
    p = std::fma(p, r, 1.0f);
    p = std::fma(p, r, 1.0f);
    return std::scalbn(p, (int)n);
}
inline float det_logf(float x) {
    if (x != x || x < 0.0f) return x != x ? x : NAN;
    if (x == 0.0f) return -HUGE_VALF;
    if (x == HUGE_VALF) return x;
    int e;
    float m = std::frexp(x, &e);
    if (m < 0.707106769f) { m = m * 2.0f; e -= 1; }
    const float f = m - 1.0f;
    const float s = f / (2.0f + f);
    const float z = s * s;
    const float R = z * std::fma(z, std::fma(z, std::fma(z, 0.222222224f, 0.285714298f), 0.400000006f), 0.666666687f);
    const float hf = 0.5f * f * f;
    const float dk = (float)e;
    return std::fma(dk, 0.693145752f, (f - (hf - std::fma(s, hf + R, dk * 1.42860677e-06f))));
}
inline float logistic(float x) { return 1.0f / (1.0f + det_expf(-x)); } /* [tcnn] */
inline float smoothstep(float x) { return x * x * (3.0f - 2.0f * x); } /* [tcnn] */
inline float sgn(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

/* ---- constants: nerf_device.cuh:25-43, common_device.cuh:32-33 ----------- */
constexpr uint32_t NERF_GRIDSIZE = 128;
constexpr uint32_t NERF_GRID_N_CELLS = NERF_GRIDSIZE * NERF_GRIDSIZE * NERF_GRIDSIZE;
constexpr uint32_t NERF_STEPS = 1024;
constexpr uint32_t NERF_CASCADES = 8;
constexpr float SQRT3 = 1.73205080757f;
constexpr float STEPSIZE = SQRT3 / NERF_STEPS;
constexpr float MIN_CONE_STEPSIZE = STEPSIZE;
constexpr float MAX_CONE_STEPSIZE = STEPSIZE * (1 << (NERF_CASCADES - 1)) * NERF_STEPS / NERF_GRIDSIZE;
constexpr float NERF_MIN_OPTICAL_THICKNESS = 0.01f;
constexpr float MAX_DEPTH = 16384.0f;
constexpr float MIN_DEPTH = 0.00001f;
constexpr uint32_t MARCH_ITER = 10000;                 /* testbed_nerf.cu:47 */
constexpr uint32_t MIN_STEPS_INBETWEEN_COMPACTION = 1; /* testbed_nerf.cu:49 */
constexpr uint32_t MAX_STEPS_INBETWEEN_COMPACTION = 8; /* testbed_nerf.cu:50 */
constexpr uint32_t BATCH_SIZE_GRANULARITY = 256;        /* tcnn (common.h) */

/* trace_alt's per-iteration sizes: n_steps_between_compaction = clamp(target_n_queries / n_alive, 1, 8)
 * (testbed_nerf.cu:2188-2190) and the batch the network evaluates, n_elements =
 * next_multiple(n_alive * n_steps, BATCH_SIZE_GRANULARITY) (:2210).  Pinned against the reference's own
 * executions (its nvprof traces, tests/test_ref_schedule.py). */
static uint32_t wavefront_steps(uint32_t n_alive, uint32_t target) {
    return std::min(std::max(target / n_alive, MIN_STEPS_INBETWEEN_COMPACTION), MAX_STEPS_INBETWEEN_COMPACTION);
}
static uint64_t wavefront_elements(uint32_t n_alive, uint32_t n_steps) {
    return ((uint64_t)n_alive * n_steps + BATCH_SIZE_GRANULARITY - 1) / BATCH_SIZE_GRANULARITY * BATCH_SIZE_GRANULARITY;
}
constexpr float PI_F = 3.14159265358979323846f;        /* tcnn::PI / random_val.cuh:27 */

/* ------------------------------------------------------------------------- */
/* fp16 conversion (round-to-nearest-even, subnormals preserved)              */
/* ------------------------------------------------------------------------- */
uint16_t half_round_ld(long double v) {
    uint16_t sign = std::signbit((double)v) ? 0x8000u : 0u;
    if (std::isnan((double)v)) return (uint16_t)(sign | 0x7e00u);
    long double av = std::fabs(v);
    if (av == 0.0L) return sign;
    if (av >= 65520.0L) return (uint16_t)(sign | 0x7c00u);
    int e;
    std::frexp(av, &e); /* av = m*2^e, m in [0.5,1) */
    int qexp = std::max(e - 1 - 10, -24);
    long double scaled = std::ldexp(av, -qexp);
    long double fl = std::floor(scaled);
    long double rem = scaled - fl;
    uint64_t h = (uint64_t)fl;
    if (rem > 0.5L || (rem == 0.5L && (h & 1))) ++h;
    if (qexp == -24 && h < 1024) return (uint16_t)(sign | h);
    int E = qexp + 25;
    if (h == 2048) { h = 1024; ++E; }
    if (E >= 31) return (uint16_t)(sign | 0x7c00u);
    return (uint16_t)(sign | (E << 10) | (h - 1024));
}
float h2f(uint16_t h) {
    uint32_t sign = (h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1f;
    uint32_t m = h & 0x3ff;
    float r;
    if (e == 0) r = std::ldexp((float)m, -24);
    else if (e == 31) r = m ? std::numeric_limits<float>::quiet_NaN() : std::numeric_limits<float>::infinity();
    else r = std::ldexp((float)(m | 0x400), (int)e - 25);
    uint32_t bits;
    std::memcpy(&bits, &r, 4);
    bits |= sign;
    std::memcpy(&r, &bits, 4);
    return r;
}
inline uint16_t f2h(float f) { return half_round_ld((long double)f); }
/* fused half fma: one rounding of the exact a*b+c, as __hfma / v_fma_f16 */
inline uint16_t hfma(uint16_t a, uint16_t b, uint16_t c) {
    long double r = (long double)h2f(a) * (long double)h2f(b) + (long double)h2f(c);
    return half_round_ld(r);
}

/* ------------------------------------------------------------------------- */
/* Morton codes [tcnn common_device.h, unvendored; SURVEY Appendix C]         */
/* ------------------------------------------------------------------------- */
inline uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
inline uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) { return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2); }
inline uint32_t morton3D_invert(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

/* ------------------------------------------------------------------------- */
/* Scrambled Sobol: random_val.cuh:162-325                                    */
/* ------------------------------------------------------------------------- */
const uint32_t SOBOL_DIRECTIONS[5][32] = {
    {0x80000000, 0x40000000, 0x20000000, 0x10000000, 0x08000000, 0x04000000, 0x02000000, 0x01000000,
     0x00800000, 0x00400000, 0x00200000, 0x00100000, 0x00080000, 0x00040000, 0x00020000, 0x00010000,
     0x00008000, 0x00004000, 0x00002000, 0x00001000, 0x00000800, 0x00000400, 0x00000200, 0x00000100,
     0x00000080, 0x00000040, 0x00000020, 0x00000010, 0x00000008, 0x00000004, 0x00000002, 0x00000001},
    {0x80000000, 0xc0000000, 0xa0000000, 0xf0000000, 0x88000000, 0xcc000000, 0xaa000000, 0xff000000,
     0x80800000, 0xc0c00000, 0xa0a00000, 0xf0f00000, 0x88880000, 0xcccc0000, 0xaaaa0000, 0xffff0000,
     0x80008000, 0xc000c000, 0xa000a000, 0xf000f000, 0x88008800, 0xcc00cc00, 0xaa00aa00, 0xff00ff00,
     0x80808080, 0xc0c0c0c0, 0xa0a0a0a0, 0xf0f0f0f0, 0x88888888, 0xcccccccc, 0xaaaaaaaa, 0xffffffff},
    {0x80000000, 0xc0000000, 0x60000000, 0x90000000, 0xe8000000, 0x5c000000, 0x8e000000, 0xc5000000,
     0x68800000, 0x9cc00000, 0xee600000, 0x55900000, 0x80680000, 0xc09c0000, 0x60ee0000, 0x90550000,
     0xe8808000, 0x5cc0c000, 0x8e606000, 0xc5909000, 0x6868e800, 0x9c9c5c00, 0xeeee8e00, 0x5555c500,
     0x8000e880, 0xc0005cc0, 0x60008e60, 0x9000c590, 0xe8006868, 0x5c009c9c, 0x8e00eeee, 0xc5005555},
    {0x80000000, 0xc0000000, 0x20000000, 0x50000000, 0xf8000000, 0x74000000, 0xa2000000, 0x93000000,
     0xd8800000, 0x25400000, 0x59e00000, 0xe6d00000, 0x78080000, 0xb40c0000, 0x82020000, 0xc3050000,
     0x208f8000, 0x51474000, 0xfbea2000, 0x75d93000, 0xa0858800, 0x914e5400, 0xdbe79e00, 0x25db6d00,
     0x58800080, 0xe54000c0, 0x79e00020, 0xb6d00050, 0x800800f8, 0xc00c0074, 0x200200a2, 0x50050093},
    {0x80000000, 0x40000000, 0x20000000, 0xb0000000, 0xf8000000, 0xdc000000, 0x7a000000, 0x9d000000,
     0x5a800000, 0x2fc00000, 0xa1600000, 0xf0b00000, 0xda880000, 0x6fc40000, 0x81620000, 0x40bb0000,
     0x22878000, 0xb3c9c000, 0xfb65a000, 0xddb2d000, 0x78022800, 0x9c0b3c00, 0x5a0fb600, 0x2d0ddb00,
     0xa2878080, 0xf3c9c040, 0xdb65a020, 0x6db2d0b0, 0x800228f8, 0x400b3cdc, 0x200fb67a, 0xb00ddb9d},
};
inline uint32_t sobol(uint32_t index, uint32_t dim) {
    uint32_t X = 0;
    for (uint32_t bit = 0; bit < 32; bit++) X ^= ((index >> bit) & 1u) * SOBOL_DIRECTIONS[dim][bit];
    return X;
}
inline uint32_t hash_combine(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
inline uint32_t reverse_bits(uint32_t x) {
    x = (((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1));
    x = (((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2));
    x = (((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4));
    x = (((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8));
    return ((x >> 16) | (x << 16));
}
inline uint32_t laine_karras_permutation(uint32_t x, uint32_t seed) {
    x += seed;
    x ^= x * 0x6c50b47cu;
    x ^= x * 0xb82f1e52u;
    x ^= x * 0xc7afe638u;
    x ^= x * 0x8d22f6e6u;
    return x;
}
inline uint32_t nested_uniform_scramble_base2(uint32_t x, uint32_t seed) {
    x = reverse_bits(x);
    x = laine_karras_permutation(x, seed);
    return reverse_bits(x);
}
inline float ld_random_val(uint32_t index, uint32_t seed, uint32_t dim = 0) {
    constexpr float S = float(1.0 / (1ull << 32));
    index = nested_uniform_scramble_base2(index, seed);
    return (float)nested_uniform_scramble_base2(sobol(index, dim), hash_combine(seed, dim)) * S;
}
inline V2 ld_random_val_2d(uint32_t index, uint32_t seed) {
    constexpr float S = float(1.0 / (1ull << 32));
    index = nested_uniform_scramble_base2(index, seed);
    uint32_t x0 = nested_uniform_scramble_base2(sobol(index, 0), hash_combine(seed, 0));
    uint32_t x1 = nested_uniform_scramble_base2(sobol(index, 1), hash_combine(seed, 1));
    return {(float)x0 * S, (float)x1 * S};
}
inline V2 ld_random_pixel_offset(uint32_t spp) { /* random_val.cuh:320-325 */
    V2 a = ld_random_val_2d(0, 0xdeadbeef), b = ld_random_val_2d(spp, 0xdeadbeef);
    V2 o = {0.5f - a.x + b.x, 0.5f - a.y + b.y};
    return {fractf(o.x), fractf(o.y)};
}

/* ------------------------------------------------------------------------- */
/* cuRAND XORWOW [cuRAND, unvendored]: SURVEY Appendix C                       */
/* ------------------------------------------------------------------------- */
struct Gf2Mat { uint32_t col[160][5]; }; /* column j = image of basis vector e_j */
void gf2_apply(const Gf2Mat& m, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int j = 0; j < 160; ++j)
        if ((in[j >> 5] >> (j & 31)) & 1u)
            for (int w = 0; w < 5; ++w) r[w] ^= m.col[j][w];
    std::memcpy(out, r, sizeof(r));
}
void xorwow_step_v(uint32_t v[5]) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}
Gf2Mat gf2_mul(const Gf2Mat& a, const Gf2Mat& b) {
    Gf2Mat r;
    for (int j = 0; j < 160; ++j) gf2_apply(a, b.col[j], r.col[j]);
    return r;
}
struct XorwowTables {
    Gf2Mat step_pow[64];   /* M^(2^i) */
    Gf2Mat seq_pow[32];    /* M^(2^67 * 2^i) */
    XorwowTables() {
        Gf2Mat m;
        for (int j = 0; j < 160; ++j) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[j >> 5] = 1u << (j & 31);
            xorwow_step_v(v);
            std::memcpy(m.col[j], v, sizeof(v));
        }
        step_pow[0] = m;
        for (int i = 1; i < 64; ++i) step_pow[i] = gf2_mul(step_pow[i - 1], step_pow[i - 1]);
        Gf2Mat a = step_pow[63];
        for (int i = 63; i < 67; ++i) a = gf2_mul(a, a); /* M^(2^67) */
        seq_pow[0] = a;
        for (int i = 1; i < 32; ++i) seq_pow[i] = gf2_mul(seq_pow[i - 1], seq_pow[i - 1]);
    }
};
const XorwowTables& xorwow_tables() {
    static XorwowTables* t = nullptr;
    static std::once_flag once;
    std::call_once(once, [] { t = new XorwowTables(); });
    return *t;
}
/* curand_init(seed, subsequence, offset): curand_kernel.h _curand_init_scratch */
void xorwow_init(uint64_t seed, uint64_t subsequence, uint64_t offset, uint32_t st[6]) {
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    uint32_t v[5] = {123456789u + t0, 362436069u ^ t0, 521288629u + t1, 88675123u ^ t1, 5783321u + t0};
    uint32_t d = 6615241u + t1 + t0;
    const XorwowTables& T = xorwow_tables();
    for (int i = 0; i < 32 && subsequence; ++i, subsequence >>= 1)
        if (subsequence & 1) gf2_apply(T.seq_pow[i], v, v);
    uint64_t off = offset;
    for (int i = 0; i < 64 && off; ++i, off >>= 1)
        if (off & 1) gf2_apply(T.step_pow[i], v, v);
    d += (uint32_t)(offset * 362437ull);
    std::memcpy(st, v, sizeof(v));
    st[5] = d;
}
inline uint32_t xorwow_next(uint32_t* st) {
    uint32_t t = st[0] ^ (st[0] >> 2);
    st[0] = st[1]; st[1] = st[2]; st[2] = st[3]; st[3] = st[4];
    st[4] = (st[4] ^ (st[4] << 4)) ^ (t ^ (t << 1));
    st[5] += 362437u;
    return st[4] + st[5];
}
/* curand_uniform: x * 2^-32 + 2^-33  (CURAND_2POW32_INV = 2.3283064e-10f) */
inline float curand_uniform(uint32_t* st) {
    const float INV = 2.3283064e-10f;
    return (float)xorwow_next(st) * INV + (INV / 2.0f);
}

/* ------------------------------------------------------------------------- */
/* AABB: bounding_box.cuh:163-222                                              */
/* ------------------------------------------------------------------------- */
struct BBox { V3 min, max; };
inline V2 bb_ray_intersect(const BBox& b, V3 pos, V3 dir) {
    float tmin = (b.min.x - pos.x) / dir.x;
    float tmax = (b.max.x - pos.x) / dir.x;
    if (tmin > tmax) std::swap(tmin, tmax);
    float tymin = (b.min.y - pos.y) / dir.y;
    float tymax = (b.max.y - pos.y) / dir.y;
    if (tymin > tymax) std::swap(tymin, tymax);
    const float FMAX = std::numeric_limits<float>::max();
    if (tmin > tymax || tymin > tmax) return {FMAX, FMAX};
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (b.min.z - pos.z) / dir.z;
    float tzmax = (b.max.z - pos.z) / dir.z;
    if (tzmin > tzmax) std::swap(tzmin, tzmax);
    if (tmin > tzmax || tzmin > tmax) return {FMAX, FMAX};
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return {tmin, tmax};
}
/* orc_set_literal (sng_oracle.h): 1 = the reference's text as written, 0 = the product's fast-math restatements */
static int g_literal = 1;
/* The BVH's box test: bounding_box.cuh:163-211 as the reference compiles it (--use_fast_math,
 * CMakeLists.txt:82, makes each (b - pos) / dir a multiply by rcp(dir)); restated as (b - pos) * y
 * with y = RN(1 / dir) per ray, the same expressions as the GPU's bvh_box_entry (sng_math.h). */
inline float bvh_box_entry(const BBox& b, V3 pos, V3 y) {
    float tmin = (b.min.x - pos.x) * y.x;
    float tmax = (b.max.x - pos.x) * y.x;
    if (tmin > tmax) std::swap(tmin, tmax);
    float tymin = (b.min.y - pos.y) * y.y;
    float tymax = (b.max.y - pos.y) * y.y;
    if (tymin > tymax) std::swap(tymin, tymax);
    const float FMAX = std::numeric_limits<float>::max();
    if (tmin > tymax || tymin > tmax) return FMAX;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (b.min.z - pos.z) * y.z;
    float tzmax = (b.max.z - pos.z) * y.z;
    if (tzmin > tzmax) std::swap(tzmin, tzmax);
    if (tmin > tzmax || tzmin > tmax) return FMAX;
    if (tzmin > tmin) tmin = tzmin;
    return tmin;
}
inline bool bb_contains(const BBox& b, V3 p) {
    return p.x >= b.min.x && p.x <= b.max.x && p.y >= b.min.y && p.y <= b.max.y && p.z >= b.min.z && p.z <= b.max.z;
}

/* ------------------------------------------------------------------------- */
/* occupancy stepping: nerf_device.cuh:266-495                                 */
/* ------------------------------------------------------------------------- */
inline V3 warp_position(V3 pos, const BBox& aabb) { return (pos - aabb.min) / (aabb.max - aabb.min); }
inline V3 unwarp_position(V3 pos, const BBox& aabb) { return aabb.min + pos * (aabb.max - aabb.min); }
inline V3 warp_direction(V3 dir) { return (dir + 1.0f) * 0.5f; }
inline float warp_dt(float dt) {
    float max_stepsize = MIN_CONE_STEPSIZE * (1 << (NERF_CASCADES - 1));
    return (dt - MIN_CONE_STEPSIZE) / (max_stepsize - MIN_CONE_STEPSIZE);
}
inline float unwarp_dt(float dt) {
    float max_stepsize = MIN_CONE_STEPSIZE * (1 << (NERF_CASCADES - 1));
    return dt * (max_stepsize - MIN_CONE_STEPSIZE) + MIN_CONE_STEPSIZE;
}
inline uint32_t cascaded_grid_idx_at(V3 pos, uint32_t mip) {
    float mip_scale = std::scalbn(1.0f, -(int)mip);
    pos = pos - v3s(0.5f);
    pos = pos * mip_scale;
    pos = pos + v3s(0.5f);
    V3 f = pos * (float)NERF_GRIDSIZE;
    int ix = (int)f.x, iy = (int)f.y, iz = (int)f.z;
    if (ix < 0 || ix >= (int)NERF_GRIDSIZE || iy < 0 || iy >= (int)NERF_GRIDSIZE || iz < 0 || iz >= (int)NERF_GRIDSIZE) return 0xFFFFFFFFu;
    return morton3D(ix, iy, iz);
}
inline bool density_grid_occupied_at(V3 pos, const uint8_t* bf, uint32_t mip) {
    uint32_t idx = cascaded_grid_idx_at(pos, mip);
    if (idx == 0xFFFFFFFFu) return false;
    return bf[idx / 8 + (NERF_GRID_N_CELLS * mip) / 8] & (1 << (idx % 8));
}
inline float distance_to_next_voxel(V3 pos, V3 dir, V3 idir, float res) {
    V3 p = res * (pos - 0.5f);
    float tx = (std::floor(p.x + 0.5f + 0.5f * sgn(dir.x)) - p.x) * idir.x;
    float ty = (std::floor(p.y + 0.5f + 0.5f * sgn(dir.y)) - p.y) * idir.y;
    float tz = (std::floor(p.z + 0.5f + 0.5f * sgn(dir.z)) - p.z) * idir.z;
    float t = std::min(std::min(tx, ty), tz);
    return std::fmax(t / res, 0.0f);
}
inline float to_stepping_space(float t, float cone_angle) {
    if (cone_angle <= 1e-5f) return t / MIN_CONE_STEPSIZE;
    float log1p_c = det_logf(1.0f + cone_angle);
    float a = (det_logf(MIN_CONE_STEPSIZE) - det_logf(log1p_c)) / log1p_c;
    float b = (det_logf(MAX_CONE_STEPSIZE) - det_logf(log1p_c)) / log1p_c;
    float at = det_expf(a * log1p_c);
    float bt = det_expf(b * log1p_c);
    if (t <= at) return (t - at) / MIN_CONE_STEPSIZE + a;
    else if (t <= bt) return det_logf(t) / log1p_c;
    else return (t - bt) / MAX_CONE_STEPSIZE + b;
}
inline float from_stepping_space(float n, float cone_angle) {
    if (cone_angle <= 1e-5f) return n * MIN_CONE_STEPSIZE;
    float log1p_c = det_logf(1.0f + cone_angle);
    float a = (det_logf(MIN_CONE_STEPSIZE) - det_logf(log1p_c)) / log1p_c;
    float b = (det_logf(MAX_CONE_STEPSIZE) - det_logf(log1p_c)) / log1p_c;
    float at = det_expf(a * log1p_c);
    float bt = det_expf(b * log1p_c);
    if (n <= a) return (n - a) * MIN_CONE_STEPSIZE + at;
    else if (n <= b) return det_expf(n * log1p_c);
    else return (n - b) * MAX_CONE_STEPSIZE + bt;
}
inline float advance_n_steps(float t, float cone_angle, float n) { return from_stepping_space(to_stepping_space(t, cone_angle) + n, cone_angle); }
inline float calc_dt(float t, float cone_angle) { return advance_n_steps(t, cone_angle, 1.0f) - t; }
inline float advance_to_next_voxel(float t, float cone_angle, V3 pos, V3 dir, V3 idir, uint32_t mip) {
    float res = std::scalbn((float)NERF_GRIDSIZE, -(int)mip);
    float t_target = t + distance_to_next_voxel(pos, dir, idir, res);
    t = to_stepping_space(t, cone_angle);
    t_target = to_stepping_space(t_target, cone_angle);
    return from_stepping_space(t + std::ceil(std::fmax(t_target - t, 0.5f)), cone_angle);
}
inline uint32_t mip_from_pos(V3 pos, uint32_t max_cascade) {
    int exponent;
    V3 d = pos - 0.5f;
    float maxval = vmax(v3(std::fabs(d.x), std::fabs(d.y), std::fabs(d.z)));
    std::frexp(maxval, &exponent);
    return (uint32_t)std::min(std::max(exponent + 1, 0), (int)max_cascade);
}
struct Volume {
    BBox render_aabb, train_aabb;
    M3 to_local;
    bool to_local_identity;
    float cone;
    uint32_t max_mip;
    float min_transmittance;
    const uint8_t* bitfield;
};
inline V3 to_local(const Volume& v, V3 p) { return v.to_local_identity ? p : mul(v.to_local, p); }
float if_unoccupied_advance_to_next_occupied_voxel(float t, float cone_angle, V3 o, V3 d, V3 idir, const uint8_t* grid,
                                                   uint32_t min_mip, uint32_t max_mip, const Volume& vol) {
    while (true) {
        V3 pos = o + d * t;
        if (t >= MAX_DEPTH || !bb_contains(vol.render_aabb, to_local(vol, pos))) return MAX_DEPTH;
        uint32_t mip = std::min(std::max(mip_from_pos(pos, NERF_CASCADES - 1), min_mip), max_mip);
        if (!grid || density_grid_occupied_at(pos, grid, mip)) return t;
        while (mip < max_mip && !density_grid_occupied_at(pos, grid, mip + 1)) ++mip;
        t = advance_to_next_voxel(t, cone_angle, pos, d, idir, mip);
    }
}

/* ------------------------------------------------------------------------- */
/* Network: NerfNetwork::inference_mixed_precision (nerf_network.h:105-139)   */
/*   hash grid [tcnn GridEncoding, unvendored], SH deg 4 [tcnn], 2 MLPs       */
/*   [tcnn FullyFusedMLP], extract_density (nerf_network.h:31-43)             */
/* ------------------------------------------------------------------------- */
struct Grid {
    uint32_t L, F, log2T, Nmin;
    float pls, log2_pls;
    std::vector<uint32_t> offsets; /* L+1, in entries */
    std::vector<uint32_t> res;
    std::vector<float> scale;
    const uint16_t* params;        /* grid params (entries x F) */
};
inline float grid_scale(uint32_t level, float log2_pls, uint32_t base_res) {
    /* exp2f(level*log2(b)) * Nmin - 1, contracted to an fma as nvcc does */
    return std::fma(std::exp2((float)level * log2_pls), (float)base_res, -1.0f);
}
inline uint32_t grid_resolution(float scale) { return (uint32_t)std::ceil(scale) + 1; }
Grid make_grid(const orc_model* m) {
    Grid g;
    g.L = m->n_levels; g.F = m->n_features; g.log2T = m->log2_hashmap_size; g.Nmin = m->base_resolution;
    g.pls = m->per_level_scale;
    g.log2_pls = std::log2(m->per_level_scale);
    uint32_t offset = 0;
    for (uint32_t i = 0; i < g.L; ++i) {
        float sc = grid_scale(i, g.log2_pls, g.Nmin);
        uint32_t r = grid_resolution(sc);
        uint32_t max_params = std::numeric_limits<uint32_t>::max() / 2;
        uint32_t pil = std::pow((float)r, 3.0f) > (float)max_params ? max_params : r * r * r;
        pil = (pil + 7u) / 8u * 8u;
        pil = std::min(pil, 1u << g.log2T);
        g.offsets.push_back(offset);
        g.res.push_back(r);
        g.scale.push_back(sc);
        offset += pil;
    }
    g.offsets.push_back(offset);
    g.params = m->params + 3072 + 7168;
    return g;
}
inline uint32_t grid_index(uint32_t hashmap_size, uint32_t res, const uint32_t pg[3]) {
    uint32_t stride = 1, index = 0;
    for (uint32_t dim = 0; dim < 3 && stride <= hashmap_size; ++dim) {
        index += pg[dim] * stride;
        stride *= res;
    }
    if (hashmap_size < stride) index = (pg[0] * 1u) ^ (pg[1] * 2654435761u) ^ (pg[2] * 805459861u);
    return index % hashmap_size;
}
void encode_one(const Grid& g, const float* x, uint16_t* out /* L*F */) {
    for (uint32_t level = 0; level < g.L; ++level) {
        const uint16_t* grid = g.params + (size_t)g.offsets[level] * g.F;
        uint32_t hashmap_size = g.offsets[level + 1] - g.offsets[level];
        float scale = g.scale[level];
        uint32_t res = g.res[level];
        float pos[3];
        uint32_t pg[3];
        for (int d = 0; d < 3; ++d) {
            float p = std::fma(scale, x[d], 0.5f);
            float tmp = std::floor(p);
            pg[d] = (uint32_t)(int)tmp;
            pos[d] = p - tmp;
        }
        uint16_t result[8] = {0};
        for (uint32_t idx = 0; idx < 8; ++idx) {
            float weight = 1.0f;
            uint32_t pl[3];
            for (uint32_t d = 0; d < 3; ++d) {
                if ((idx & (1u << d)) == 0) { weight *= 1.0f - pos[d]; pl[d] = pg[d]; }
                else { weight *= pos[d]; pl[d] = pg[d] + 1; }
            }
            uint32_t index = grid_index(hashmap_size, res, pl) * g.F;
            uint16_t wh = f2h(weight);
            for (uint32_t f = 0; f < g.F; ++f) result[f] = hfma(wh, grid[index + f], result[f]);
        }
        for (uint32_t f = 0; f < g.F; ++f) out[level * g.F + f] = result[f];
    }
}
void sh_one(float dx, float dy, float dz, uint16_t* o) {
    float x = dx * 2.f - 1.f, y = dy * 2.f - 1.f, z = dz * 2.f - 1.f;
    float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    o[0] = f2h(0.28209479177387814f);
    o[1] = f2h(-0.48860251190291987f * y);
    o[2] = f2h(0.48860251190291987f * z);
    o[3] = f2h(-0.48860251190291987f * x);
    o[4] = f2h(1.0925484305920792f * xy);
    o[5] = f2h(-1.0925484305920792f * yz);
    o[6] = f2h(0.94617469575755997f * z2 - 0.31539156525251999f);
    o[7] = f2h(-1.0925484305920792f * xz);
    o[8] = f2h(0.54627421529603959f * x2 - 0.54627421529603959f * y2);
    o[9] = f2h(0.59004358992664352f * y * (-3.0f * x2 + y2));
    o[10] = f2h(2.8906114426405538f * xy * z);
    o[11] = f2h(0.45704579946446572f * y * (1.0f - 5.0f * z2));
    o[12] = f2h(0.3731763325901154f * z * (5.0f * z2 - 3.0f));
    o[13] = f2h(0.45704579946446572f * x * (1.0f - 5.0f * z2));
    o[14] = f2h(1.4453057213202769f * z * (x2 - y2));
    o[15] = f2h(0.59004358992664352f * x * (-x2 + 3.0f * y2));
}
/* dense layer y = W x (W row-major [n_out][n_in], fp16), optional ReLU, result rounded to fp16
 * [tcnn FullyFusedMLP, unvendored].  Two accumulation models (orc_set_mlp_accum):
 *   mode 0 (default): one fp32 accumulator over the whole K, rounded to fp16 once -- what this repository's
 *     MFMA kernel computes (v_mfma_f32_16x16x32_f16 keeps an f32 accumulator);
 *   mode 1: tcnn's FullyFusedMLP on sm >= 70 (nerf_network.h:120,130 -> fully_fused_mlp.cu): WMMA fragments
 *     with __half accumulators (wmma::fragment<accumulator,16,16,16,__half>), so the running sum is
 *     rounded to fp16 after every k-chunk of `chunk` products (16 = one wmma::mma_sync; the products of
 *     a chunk summed in fp32).  The tensor core's internal alignment/truncation inside a chunk is not
 *     modelled (unpublished; parity unpinned). */
static int g_mlp_accum = 0, g_mlp_chunk = 16;
void dense(const uint16_t* W, uint32_t n_out, uint32_t n_in, const uint16_t* x, uint16_t* y, bool relu) {
    for (uint32_t o = 0; o < n_out; ++o) {
        float acc = 0.0f;
        if (g_mlp_accum == 0) {
            for (uint32_t k = 0; k < n_in; ++k) acc += h2f(W[o * n_in + k]) * h2f(x[k]);
        } else {
            for (uint32_t k0 = 0; k0 < n_in; k0 += (uint32_t)g_mlp_chunk) {
                float part = 0.0f;
                for (uint32_t k = k0; k < std::min(n_in, k0 + (uint32_t)g_mlp_chunk); ++k) part += h2f(W[o * n_in + k]) * h2f(x[k]);
                acc = h2f(f2h(acc + part));
            }
        }
        if (relu && acc < 0.0f) acc = 0.0f;
        y[o] = f2h(acc);
    }
}
/* Testbed::render_nerf's extra network passes (testbed_nerf.cu:2363-2366) [tcnn, unvendored]: tcnn gets the
 * network input matrix as its own output, so the NerfCoordinate is rewritten in place.
 *   Normals (2): NerfNetwork::input_gradient(dim 3) -- backward_impl (nerf_network.h:189-268) with dL/doutput
 *     one-hot at the density row: the rgb branch carries zero gradient, so rows 4-6 (direction) become 0;
 *     the density MLP backward (ReLU mask from the forward activation) gives dL/d(encoding); GridEncoding's
 *     input gradient sums, per level and axis, the 4 edges along the axis weighted by the other two axes'
 *     linear weights times the level scale (kernel_grid dy_dx).  Row 3 (dt) is not an input: untouched.
 *     Computed in float (tcnn: fp16 backprop with loss scale 128).
 *   EncodingVis (10): visualize_activation(layer, dim) -> extract_dimension_pos_neg_kernel over the 7-row
 *     output: (max(-v, 0), max(v, 0), 0, 1, 1, 1, 1). */
static int g_vis_layer = 0, g_vis_dim = 0;
void probe_one(const orc_model* m, const Grid& g, float* cc, int mode) {
    const uint16_t* dW0 = m->params;
    const uint16_t* dW1 = dW0 + 64 * 32;
    const uint16_t* rW0 = m->params + 3072;
    const uint16_t* rW1 = rW0 + 64 * 32;
    uint16_t enc[32], h[64];
    encode_one(g, cc, enc);
    dense(dW0, 64, 32, enc, h, true);
    if (mode == 2) {
        float gh[64], gx[3] = {0.0f, 0.0f, 0.0f};
        for (int j = 0; j < 64; ++j) gh[j] = h2f(h[j]) > 0.0f ? h2f(dW1[j]) : 0.0f;
        for (uint32_t level = 0; level < g.L; ++level) {
            float ge[4] = {0, 0, 0, 0};
            for (uint32_t f = 0; f < g.F; ++f)
                for (int j = 0; j < 64; ++j) ge[f] = std::fma(h2f(dW0[j * 32 + level * g.F + f]), gh[j], ge[f]);
            const uint16_t* grid = g.params + (size_t)g.offsets[level] * g.F;
            uint32_t hashmap_size = g.offsets[level + 1] - g.offsets[level];
            float scale = g.scale[level];
            uint32_t res = g.res[level];
            float pos[3];
            uint32_t pg[3];
            for (int d = 0; d < 3; ++d) {
                float p = std::fma(scale, cc[d], 0.5f);
                float tmp = std::floor(p);
                pg[d] = (uint32_t)(int)tmp;
                pos[d] = p - tmp;
            }
            for (uint32_t gd = 0; gd < 3; ++gd) {
                for (uint32_t idx = 0; idx < 4; ++idx) {
                    float w = scale;
                    uint32_t pl[3];
                    for (uint32_t ng = 0; ng < 2; ++ng) {
                        const uint32_t dim = ng >= gd ? ng + 1 : ng;
                        if ((idx & (1u << ng)) == 0) { w *= 1.0f - pos[dim]; pl[dim] = pg[dim]; }
                        else { w *= pos[dim]; pl[dim] = pg[dim] + 1; }
                    }
                    pl[gd] = pg[gd];
                    const uint32_t il = grid_index(hashmap_size, res, pl) * g.F;
                    pl[gd] = pg[gd] + 1;
                    const uint32_t ir = grid_index(hashmap_size, res, pl) * g.F;
                    for (uint32_t f = 0; f < g.F; ++f) gx[gd] += ge[f] * (w * (h2f(grid[ir + f]) - h2f(grid[il + f])));
                }
            }
        }
        cc[0] = gx[0]; cc[1] = gx[1]; cc[2] = gx[2];
        cc[4] = 0.0f; cc[5] = 0.0f; cc[6] = 0.0f;
        return;
    }
    float v;
    if (g_vis_layer == 0) v = h2f(enc[g_vis_dim]);
    else if (g_vis_layer == 1) v = h2f(h[g_vis_dim]);
    else {
        uint16_t rin[32], h1[64], h2o[64];
        dense(dW1, 16, 64, h, rin, false);
        sh_one(cc[4], cc[5], cc[6], rin + 16);
        if (g_vis_layer == 2) v = h2f(rin[g_vis_dim]);
        else {
            dense(rW0, 64, 32, rin, h1, true);
            if (g_vis_layer == 3) v = h2f(h1[g_vis_dim]);
            else { dense(rW1, 64, 64, h1, h2o, true); v = h2f(h2o[g_vis_dim]); }
        }
    }
    cc[0] = std::max(-v, 0.0f); cc[1] = std::max(v, 0.0f); cc[2] = 0.0f;
    cc[3] = 1.0f; cc[4] = 1.0f; cc[5] = 1.0f; cc[6] = 1.0f;
}
/* one sample; coords = NerfCoordinate {pos(3), dt, dir(3)} (nerf_device.cuh:176-202);
 * out16 = the 16 fp16 outputs of the rgb network with row 3 replaced by density (extract_density) */
void network_one(const orc_model* m, const Grid& g, const float* coord, uint16_t* out16) {
    const uint16_t* dW0 = m->params;           /* density W0 [64][32] */
    const uint16_t* dW1 = dW0 + 64 * 32;       /* density W1 [16][64] */
    const uint16_t* rW0 = m->params + 3072;    /* rgb W0 [64][32] */
    const uint16_t* rW1 = rW0 + 64 * 32;       /* rgb W1 [64][64] */
    const uint16_t* rW2 = rW1 + 64 * 64;       /* rgb W2 [16][64] */
    uint16_t enc[32], h[64], h2[64], rgb_in[32], out[16];
    encode_one(g, coord, enc);
    dense(dW0, 64, 32, enc, h, true);
    dense(dW1, 16, 64, h, rgb_in, false);       /* density_network_output = rgb_network_input rows 0..15 */
    sh_one(coord[4], coord[5], coord[6], rgb_in + 16);
    dense(rW0, 64, 32, rgb_in, h, true);
    dense(rW1, 64, 64, h, h2, true);
    dense(rW2, 16, 64, h2, out, false);
    out[3] = rgb_in[0];                          /* extract_density: nerf_network.h:132-138 */
    std::memcpy(out16, out, sizeof(out));
}

/* ------------------------------------------------------------------------- */
/* BVH: triangle_bvh.cu:165-319 (traversal), 615-718 (build)                   */
/* ------------------------------------------------------------------------- */
struct Tri { V3 a, b, c; };
struct Node { BBox bb; int left, right; };
inline float tri_intersect(const Tri& tr, V3 ro, V3 rd) { /* triangle.cuh:45-59 */
    V3 v1v0 = tr.b - tr.a, v2v0 = tr.c - tr.a, rov0 = ro - tr.a;
    V3 n = cross(v1v0, v2v0);
    V3 q = cross(rov0, rd);
    float d = 1.0f / dot(rd, n);
    float u = d * -dot(q, v2v0);
    float v = d * dot(q, v1v0);
    float t = d * -dot(n, rov0);
    if (u < 0.0f || u > 1.0f || v < 0.0f || (u + v) > 1.0f || t < 0.0f) t = std::numeric_limits<float>::max();
    return t;
}
inline V3 tri_normal(const Tri& t) { return normalize(cross(t.b - t.a, t.c - t.a)); }
inline V3 tri_centroid(const Tri& t) { return (t.a + t.b + t.c) / 3.0f; }
inline float tri_centroid_axis(const Tri& t, int axis) { return (t.a[axis] + t.b[axis] + t.c[axis]) / 3; }
inline M3 tri_perturb(const Tri& t) { /* triangle.cuh:164-170 */
    V3 N = tri_normal(t);
    V3 T = normalize(tri_centroid(t) - t.a);
    V3 B = cross(T, N);
    return {{T, B, N}};
}
struct Object {
    const float* nodes;
    const Tri* tris;
    M3 rot; V3 pos; float scale; int mat_id;
    M3 world_to_obj; /* (I/scale) * inverse(rot) -- hoisted, same float ops (triangle_bvh.cu:313-319) */
};
inline Node load_node(const float* p, int idx) {
    const float* n = p + 8 * idx;
    Node r;
    r.bb.min = v3(n[0], n[1], n[2]);
    r.bb.max = v3(n[3], n[4], n[5]);
    std::memcpy(&r.left, &n[6], 4);
    std::memcpy(&r.right, &n[7], 4);
    return r;
}
/* ray_intersect_nodes_f<2>: triangle_bvh.cu:263-307 */
std::pair<int, float> ray_intersect_nodes(V3 ro, V3 rd, const float* nodes, const Tri* tris) {
    int stack[32];
    int count = 0;
    stack[count++] = 0;
    float mint = MAX_DEPTH;
    int shortest = -1;
    const V3 y = v3(1.0f / rd.x, 1.0f / rd.y, 1.0f / rd.z);
    while (count > 0) {
        int idx = stack[--count];
        Node node = load_node(nodes, idx);
        if (node.left < 0) {
            int end = -node.right - 1;
            for (int i = -node.left - 1; i < end; ++i) {
                float t = tri_intersect(tris[i], ro, rd);
                if (t < mint) { mint = t; shortest = i; }
            }
        } else {
            struct DI { float dist; int idx; } ch[2];
            /* BoundingBox::ray_intersect(...).x (triangle_bvh.cu:296-298): IEEE division as written, or the product's
             * multiply by the per-ray reciprocal */
            for (int i = 0; i < 2; ++i) {
                const BBox& bb = load_node(nodes, node.left + i).bb;
                ch[i] = {g_literal ? bb_ray_intersect(bb, ro, rd).x : bvh_box_entry(bb, ro, y), node.left + i};
            }
            if (ch[0].dist < ch[1].dist) std::swap(ch[0], ch[1]); /* sorting_network<2>: descending */
            for (int i = 0; i < 2; ++i)
                if (ch[i].dist < mint) {
                    if (count >= 31) std::fprintf(stderr, "WARNING TOO BIG\n");
                    stack[count++] = ch[i].idx;
                }
        }
    }
    return {shortest, mint};
}
std::pair<int, float> ray_intersect_object(V3 ro, V3 rd, const Object& o) {
    V3 oro = mul(o.world_to_obj, ro - o.pos);
    V3 ord = mul(o.world_to_obj, rd);
    return ray_intersect_nodes(oro, ord, o.nodes, o.tris);
}
Object make_object(const orc_object& s) {
    Object o;
    o.nodes = s.nodes;
    o.tris = (const Tri*)s.tris;
    o.rot = m3_load(s.rot);
    o.pos = v3(s.pos[0], s.pos[1], s.pos[2]);
    o.scale = s.scale;
    o.mat_id = s.mat_id;
    M3 msc = {{v3(1.0f / s.scale, 0.0f / s.scale, 0.0f / s.scale), v3(0.0f / s.scale, 1.0f / s.scale, 0.0f / s.scale),
               v3(0.0f / s.scale, 0.0f / s.scale, 1.0f / s.scale)}};
    o.world_to_obj = mulm(msc, inverse(o.rot));
    return o;
}
struct HitRecord {
    V3 pos = v3s(0.0f), normal = v3s(0.0f);
    M3 perturb = {{v3(1, 0, 0), v3(0, 1, 0), v3(0, 0, 1)}};
    float t = MAX_DEPTH;
    int material_idx = -1, object_idx = -1;
    bool front_face = true;
};
/* sng::depth_test_world: synerfgine/common.cu:36-48 */
float depth_test_world(V3 origin, V3 dir, const std::vector<Object>& objs, int& out_obj) {
    float depth = MAX_DEPTH;
    V3 off = origin + dir * MIN_DEPTH;
    for (size_t c = 0; c < objs.size(); ++c) {
        auto r = ray_intersect_object(off, dir, objs[c]);
        if (r.second < depth && r.second > MIN_DEPTH) { out_obj = (int)c; depth = r.second; }
    }
    return depth;
}
/* sng::depth_test_world (+HitRecord): synerfgine/common.cu:50-67 */
float depth_test_world_hit(V3 origin, V3 dir, const std::vector<Object>& objs, int& out_obj, HitRecord& h) {
    V3 off = origin + dir * MIN_DEPTH;
    for (size_t c = 0; c < objs.size(); ++c) {
        const Object& obj = objs[c];
        auto r = ray_intersect_object(off, dir, obj);
        if (r.second < h.t && r.second > MIN_DEPTH) {
            out_obj = (int)c;
            h.t = r.second;
            h.material_idx = obj.mat_id;
            h.normal = mul(obj.rot, tri_normal(obj.tris[r.first]));
            h.perturb = tri_perturb(obj.tris[r.first]);
            h.object_idx = (int)c;
        }
    }
    h.pos = origin + h.t * dir;
    h.front_face = dot(dir, h.normal) < 0.0f;
    return h.t;
}
/* sng::depth_test_nerf (full_d form): synerfgine/common.cu:69-83 */
float depth_test_nerf_fd(float full_d, uint32_t n_steps, float cone, V3 src, V3 L, V3 invL, const Volume& vol, uint32_t min_mip, uint32_t max_mip) {
    float s = 0.0f;
    for (uint32_t j = 0; j < n_steps; ++j) {
        s = if_unoccupied_advance_to_next_occupied_voxel(s, cone, src, L, invL, vol.bitfield, min_mip, max_mip, vol);
        if (s >= full_d) { s = full_d; break; }
        s += calc_dt(s, cone);
    }
    return s;
}
/* sng::depth_test_nerf (src,dst form): synerfgine/common.cu:85-102 */
float depth_test_nerf_sd(uint32_t n_steps, float cone, V3 src, V3 dst, const Volume& vol, uint32_t min_mip, uint32_t max_mip) {
    float full_d = length(dst - src);
    V3 L = normalize(dst - src);
    V3 invL = v3(1.0f / L.x, 1.0f / L.y, 1.0f / L.z);
    return depth_test_nerf_fd(full_d, n_steps, cone, src, L, invL, vol, min_mip, max_mip);
}

/* sRGB: common_device.cuh:35-70 */
/* x^n as the GPU's pow_small_int (mesh.hip) forms it: binary exponentiation for integer n in
 * [0, 4096] (the Phong exponents and shadow intensities of every reference scene), std::pow
 * otherwise.  The reference builds with --use_fast_math, so its powf is __powf (exp2(n log2 x),
 * coarser than either); both GPU and oracle use this form, so they agree bit for bit. */
inline float pow_small_int(float x, float n) {
    if (std::floor(n) == n && n >= 0.0f && n <= 4096.0f) {
        uint32_t e = (uint32_t)n;
        float r = 1.0f, b = x;
        while (e) {
            if (e & 1u) r *= b;
            b *= b;
            e >>= 1;
        }
        return r;
    }
    return std::pow(x, n);
}
/* pow(x, n) of the render path's Phong term and shadow masks: powf as the text writes it (literal mode), or the
 * product's pow_small_int */
inline float pow_src(float x, float n) { return g_literal ? std::pow(x, n) : pow_small_int(x, n); }
inline float srgb_to_linear(float s) { return s <= 0.04045f ? s / 12.92f : std::pow((s + 0.055f) / 1.055f, 2.4f); }
inline float linear_to_srgb(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * std::pow(l, 0.41666f) - 0.055f; }

Volume make_volume(const orc_volume* v) {
    Volume vol;
    vol.render_aabb = {v3(v->render_aabb_min[0], v->render_aabb_min[1], v->render_aabb_min[2]), v3(v->render_aabb_max[0], v->render_aabb_max[1], v->render_aabb_max[2])};
    vol.train_aabb = {v3(v->train_aabb_min[0], v->train_aabb_min[1], v->train_aabb_min[2]), v3(v->train_aabb_max[0], v->train_aabb_max[1], v->train_aabb_max[2])};
    vol.to_local = m3_load(v->render_aabb_to_local);
    vol.to_local_identity = m3_is_identity(vol.to_local);
    vol.cone = v->cone_angle_constant;
    vol.max_mip = v->max_mip;
    vol.min_transmittance = v->min_transmittance;
    vol.bitfield = v->bitfield;
    return vol;
}

/* glm-style quat round trip used by get_xform_given_rolling_shutter
 * (common_device.cuh:361-368) with start == end and pixel_t == 0 [tcnn quat, unvendored] */
struct Quat { float x, y, z, w; };
Quat quat_from_m3(const M3& m0) {
    auto m = [&](int i, int j) { return m0.c[i][j]; };
    float fx = m(0, 0) - m(1, 1) - m(2, 2), fy = m(1, 1) - m(0, 0) - m(2, 2), fz = m(2, 2) - m(0, 0) - m(1, 1), fw = m(0, 0) + m(1, 1) + m(2, 2);
    int bi = 0;
    float fb = fw;
    if (fx > fb) { fb = fx; bi = 1; }
    if (fy > fb) { fb = fy; bi = 2; }
    if (fz > fb) { fb = fz; bi = 3; }
    float bv = std::sqrt(fb + 1.0f) * 0.5f;
    float mult = 0.25f / bv;
    switch (bi) {
        case 0: return {(m(1, 2) - m(2, 1)) * mult, (m(2, 0) - m(0, 2)) * mult, (m(0, 1) - m(1, 0)) * mult, bv};
        case 1: return {bv, (m(0, 1) + m(1, 0)) * mult, (m(2, 0) + m(0, 2)) * mult, (m(1, 2) - m(2, 1)) * mult};
        case 2: return {(m(0, 1) + m(1, 0)) * mult, bv, (m(1, 2) + m(2, 1)) * mult, (m(2, 0) - m(0, 2)) * mult};
        default: return {(m(2, 0) + m(0, 2)) * mult, (m(1, 2) + m(2, 1)) * mult, bv, (m(0, 1) - m(1, 0)) * mult};
    }
}
M3 rolling_shutter_rotation(const M3& rot) {
    Quat q = quat_from_m3(rot);
    /* slerp(q, q, 0) */
    float cos_theta = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
    Quat s;
    if (cos_theta > 1.0f - std::numeric_limits<float>::epsilon()) {
        s = {q.x * (1.0f - 0.0f) + q.x * 0.0f, q.y * (1.0f - 0.0f) + q.y * 0.0f, q.z * (1.0f - 0.0f) + q.z * 0.0f, q.w * (1.0f - 0.0f) + q.w * 0.0f};
    } else {
        float angle = std::acos(cos_theta);
        float s0 = std::sin((1.0f - 0.0f) * angle), s1 = std::sin(0.0f * angle), sa = std::sin(angle);
        s = {(s0 * q.x + s1 * q.x) / sa, (s0 * q.y + s1 * q.y) / sa, (s0 * q.z + s1 * q.z) / sa, (s0 * q.w + s1 * q.w) / sa};
    }
    float len = std::sqrt(s.x * s.x + s.y * s.y + s.z * s.z + s.w * s.w);
    s = {s.x / len, s.y / len, s.z / len, s.w / len};
    float qxx = s.x * s.x, qyy = s.y * s.y, qzz = s.z * s.z, qxz = s.x * s.z, qxy = s.x * s.y, qyz = s.y * s.z;
    float qwx = s.w * s.x, qwy = s.w * s.y, qwz = s.w * s.z;
    M3 r;
    r.c[0][0] = 1.0f - 2.0f * (qyy + qzz); r.c[0][1] = 2.0f * (qxy + qwz); r.c[0][2] = 2.0f * (qxz - qwy);
    r.c[1][0] = 2.0f * (qxy - qwz); r.c[1][1] = 1.0f - 2.0f * (qxx + qzz); r.c[1][2] = 2.0f * (qyz + qwx);
    r.c[2][0] = 2.0f * (qxz + qwy); r.c[2][1] = 2.0f * (qyz - qwx); r.c[2][2] = 1.0f - 2.0f * (qxx + qyy);
    return r;
}

/* get_xform_given_rolling_shutter (common_device.cuh:361-368) for start != end: slerp(q0, q1, t) with
 * the short-way negation and the mix branch near cos 1, normalize, to_mat3 [tcnn quat, unvendored] */
M3 shutter_rotation(Quat a, Quat b, float t) {
    float cos_theta = a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
    if (cos_theta < 0.0f) { b = {-b.x, -b.y, -b.z, -b.w}; cos_theta = -cos_theta; }
    Quat s;
    if (cos_theta > 1.0f - std::numeric_limits<float>::epsilon()) {
        s = {a.x * (1.0f - t) + b.x * t, a.y * (1.0f - t) + b.y * t, a.z * (1.0f - t) + b.z * t, a.w * (1.0f - t) + b.w * t};
    } else {
        float angle = std::acos(cos_theta);
        float s0 = std::sin((1.0f - t) * angle), s1 = std::sin(t * angle), sa = std::sin(angle);
        s = {(s0 * a.x + s1 * b.x) / sa, (s0 * a.y + s1 * b.y) / sa, (s0 * a.z + s1 * b.z) / sa, (s0 * a.w + s1 * b.w) / sa};
    }
    float len = std::sqrt(s.x * s.x + s.y * s.y + s.z * s.z + s.w * s.w);
    s = {s.x / len, s.y / len, s.z / len, s.w / len};
    float qxx = s.x * s.x, qyy = s.y * s.y, qzz = s.z * s.z, qxz = s.x * s.z, qxy = s.x * s.y, qyz = s.y * s.z;
    float qwx = s.w * s.x, qwy = s.w * s.y, qwz = s.w * s.z;
    M3 r;
    r.c[0][0] = 1.0f - 2.0f * (qyy + qzz); r.c[0][1] = 2.0f * (qxy + qwz); r.c[0][2] = 2.0f * (qxz - qwy);
    r.c[1][0] = 2.0f * (qxy - qwz); r.c[1][1] = 1.0f - 2.0f * (qxx + qzz); r.c[1][2] = 2.0f * (qyz + qwx);
    r.c[2][0] = 2.0f * (qxz + qwy); r.c[2][1] = 2.0f * (qyz - qwx); r.c[2][2] = 1.0f - 2.0f * (qxx + qyy);
    return r;
}

/* View::camera1 / rolling_shutter (testbed.h:1032,1042): orc_set_motion_blur */
static bool g_has_cam1 = false;
static float g_cam1[12], g_rs[4] = {0.0f, 0.0f, 0.0f, 1.0f};
/* Lens (common.h:188-205): the render lens (Testbed::Nerf::render_lens with render_with_lens_distortion,
 * testbed_nerf.cu:2504; orc_set_render_lens) and the training images' lenses (orc_set_train_lens) */
struct OrcLens { int32_t mode = 0; float params[7] = {}; };
static OrcLens g_render_lens;
static std::vector<OrcLens> g_train_lens;

/* opencv_lens_distortion_delta (common_device.cuh:250-266) */
static void opencv_lens_distortion_delta(const float* extra_params, float u, float v, float* du, float* dv) {
    const float k1 = extra_params[0];
    const float k2 = extra_params[1];
    const float p1 = extra_params[2];
    const float p2 = extra_params[3];
    const float u2 = u * u;
    const float uv = u * v;
    const float v2 = v * v;
    const float r2 = u2 + v2;
    const float radial = k1 * r2 + k2 * r2 * r2;
    *du = u * radial + 2.0f * p1 * uv + p2 * (r2 + 2.0f * u2);
    *dv = v * radial + 2.0f * p2 * uv + p1 * (r2 + 2.0f * v2);
}
/* opencv_fisheye_lens_distortion_delta (common_device.cuh:268-292) */
static void opencv_fisheye_lens_distortion_delta(const float* extra_params, float u, float v, float* du, float* dv) {
    const float k1 = extra_params[0], k2 = extra_params[1], k3 = extra_params[2], k4 = extra_params[3];
    const float r = std::sqrt(u * u + v * v);
    if (r > (float)std::numeric_limits<double>::epsilon()) {
        const float theta = std::atan(r);
        const float theta2 = theta * theta;
        const float theta4 = theta2 * theta2;
        const float theta6 = theta4 * theta2;
        const float theta8 = theta4 * theta4;
        const float thetad = theta * (1.0f + k1 * theta2 + k2 * theta4 + k3 * theta6 + k4 * theta8);
        *du = u * thetad / r - u;
        *dv = v * thetad / r - v;
    } else {
        *du = 0.0f;
        *dv = 0.0f;
    }
}
/* iterative_lens_undistortion (common_device.cuh:294-330); mat2 J column-major, tcnn inverse(mat2) as 1/det x adjugate */
template <typename F>
static void iterative_lens_undistortion(const float* params, float* u, float* v, F distortion_fun) {
    const uint32_t kNumIterations = 100;
    const float kMaxStepNorm = 1e-10f;
    const float kRelStepSize = 1e-6f;
    float J[2][2];
    const V2 x0 = {*u, *v};
    V2 x = {*u, *v};
    V2 dx, dx_0b, dx_0f, dx_1b, dx_1f;
    for (uint32_t i = 0; i < kNumIterations; ++i) {
        const float step0 = std::max(std::numeric_limits<float>::epsilon(), std::abs(kRelStepSize * x.x));
        const float step1 = std::max(std::numeric_limits<float>::epsilon(), std::abs(kRelStepSize * x.y));
        distortion_fun(params, x.x, x.y, &dx.x, &dx.y);
        distortion_fun(params, x.x - step0, x.y, &dx_0b.x, &dx_0b.y);
        distortion_fun(params, x.x + step0, x.y, &dx_0f.x, &dx_0f.y);
        distortion_fun(params, x.x, x.y - step1, &dx_1b.x, &dx_1b.y);
        distortion_fun(params, x.x, x.y + step1, &dx_1f.x, &dx_1f.y);
        J[0][0] = 1 + (dx_0f.x - dx_0b.x) / (2 * step0);
        J[1][0] = (dx_1f.x - dx_1b.x) / (2 * step1);
        J[0][1] = (dx_0f.y - dx_0b.y) / (2 * step0);
        J[1][1] = 1 + (dx_1f.y - dx_1b.y) / (2 * step1);
        const float d = 1.0f / (J[0][0] * J[1][1] - J[1][0] * J[0][1]);
        const float inv[2][2] = {{d * J[1][1], -d * J[0][1]}, {-d * J[1][0], d * J[0][0]}};
        const V2 r = {x.x + dx.x - x0.x, x.y + dx.y - x0.y};
        const V2 step_x = {inv[0][0] * r.x + inv[1][0] * r.y, inv[0][1] * r.x + inv[1][1] * r.y};
        x.x -= step_x.x;
        x.y -= step_x.y;
        if (step_x.x * step_x.x + step_x.y * step_x.y < kMaxStepNorm) break;
    }
    *u = x.x;
    *v = x.y;
}
/* uv_to_ray's direction (common_device.cuh:403-447; identity foveation, no mask / distortion map); false = Ray::invalid() */
static bool uv_to_ray_dir(const OrcLens& lens, V2 uv, int W, int H, V2 focal, V2 screen_center, V3* dir) {
    const float PI_ = 3.14159265358979323846f;
    if (lens.mode == 2) {   /* f_theta_undistortion (370-384) */
        const V2 d = {uv.x - screen_center.x, uv.y - screen_center.y};
        const float xpix = d.x * lens.params[5];
        const float ypix = d.y * lens.params[6];
        const float norm = std::sqrt(xpix * xpix + ypix * ypix);
        const float alpha = lens.params[0] + norm * (lens.params[1] + norm * (lens.params[2] + norm * (lens.params[3] + norm * lens.params[4])));
        float sin_alpha = std::sin(alpha), cos_alpha = std::cos(alpha);
        if (cos_alpha <= std::numeric_limits<float>::min() || norm == 0.f) return false;
        sin_alpha *= 1.f / norm;
        *dir = v3(sin_alpha * xpix, sin_alpha * ypix, cos_alpha);
        return true;
    } else if (lens.mode == 3) {   /* latlong_to_dir (386-393) */
        const float theta = (uv.y - 0.5f) * PI_;
        const float phi = (uv.x - 0.5f) * PI_ * 2.0f;
        const float st = std::sin(theta), ct = std::cos(theta), sp = std::sin(phi), cp = std::cos(phi);
        *dir = v3(sp * ct, st, cp * ct);
        return true;
    } else if (lens.mode == 5) {   /* equirectangular_to_dir (395-401) */
        const float ct = (uv.y - 0.5f) * 2.0f;
        const float st = std::sqrt(std::max(1.0f - ct * ct, 0.0f));
        const float phi = (uv.x - 0.5f) * PI_ * 2.0f;
        const float sp = std::sin(phi), cp = std::cos(phi);
        *dir = v3(sp * st, ct, cp * st);
        return true;
    }
    *dir = v3((uv.x - screen_center.x) * (float)W / focal.x, (uv.y - screen_center.y) * (float)H / focal.y, 1.0f);
    if (lens.mode == 1) iterative_lens_undistortion(lens.params, &dir->x, &dir->y, opencv_lens_distortion_delta);
    else if (lens.mode == 4) iterative_lens_undistortion(lens.params, &dir->x, &dir->y, opencv_fisheye_lens_distortion_delta);
    return true;
}

/* Testbed::Nerf::glow_mode / glow_y_cutoff (testbed.h:870-871): orc_set_glow */
static int g_glow_mode = 0;
static float g_glow_y_cutoff = 0.0f;

/* composite_kernel_nerf's glow visualisation (testbed_nerf.cu:638-734): adds to rgb, may scale weight */
static void glow_term(V3 pos, V3 cam_pos, V3& rgb, float& weight) {
    const int glow_mode = g_glow_mode;
    const float glow_y_cutoff = g_glow_y_cutoff;
    float glow = 0.f;
    const bool green_grid = glow_mode & 1, green_cutline = glow_mode & 2, mask_to_alpha = glow_mode & 4;
    const bool radial_mode = glow_mode & 8, grid_mode = glow_mode & 16;
    float dist;
    if (radial_mode) {
        dist = length(pos - cam_pos);
        dist = std::min(dist, (4.5f - pos.y) * 0.333f);
    } else {
        dist = pos.y;
    }
    if (grid_mode) {
        glow = 1.f / std::max(1.f, dist);
    } else {
        float y = glow_y_cutoff - dist;
        float mask = 0.f;
        if (y > 0.f) {
            y *= 80.f;
            mask = std::min(1.f, y);
            if (green_cutline) glow += std::max(0.f, 1.f - std::fabs(1.f - y)) * 4.f;
            if (y > 1.f) y = 1.f - (y - 1.f) * 0.05f;
            if (green_grid) glow += std::max(0.f, y / std::max(1.f, dist));
        }
        if (mask_to_alpha) weight *= mask;
    }
    if (glow > 0.f) {
        float line = 0.f;
        const float sc[4] = {1.f, 2.f, 4.f, 8.f};
        for (int q = 0; q < 4; ++q) {   /* pos.y, pos.x, pos.z at frequencies 2, 4, 8, 16 (in the reference's order) */
            const float m = 2.f * sc[q];
            line += std::max(0.f, std::cos(pos.y * m * 3.141592653589793f * 16.f) - 0.975f);
            line += std::max(0.f, std::cos(pos.x * m * 3.141592653589793f * 16.f) - 0.975f);
            line += std::max(0.f, std::cos(pos.z * m * 3.141592653589793f * 16.f) - 0.975f);
        }
        if (grid_mode) {
            glow = glow * line * 15.f;
            rgb.y = glow; rgb.z = glow * 0.5f; rgb.x = glow * 0.25f;
        } else {
            glow = glow * glow * 0.25f + glow * line * 15.f;
            rgb.y += glow; rgb.z += glow * 0.5f; rgb.x += glow * 0.25f;
        }
    }
}

struct Payload { V3 origin, dir; float t, max_weight; uint32_t idx; uint16_t n_steps; bool alive; };
struct RayState { V4 rgba; float depth; Payload p; };

}  // namespace

/* =========================================================================== */
/* C API                                                                        */
/* =========================================================================== */
extern "C" {

uint32_t orc_morton3D(uint32_t x, uint32_t y, uint32_t z) { return morton3D(x, y, z); }
uint32_t orc_morton3D_invert(uint32_t x) { return morton3D_invert(x); }
uint32_t orc_sobol(uint32_t index, uint32_t dim) { return sobol(index, dim); }
float orc_ld_random_val(uint32_t index, uint32_t seed, uint32_t dim) { return ld_random_val(index, seed, dim); }
void orc_ld_random_pixel_offset(uint32_t spp, float out[2]) { V2 o = ld_random_pixel_offset(spp); out[0] = o.x; out[1] = o.y; }
uint16_t orc_float_to_half(float f) { return f2h(f); }
float orc_half_to_float(uint16_t h) { return h2f(h); }

void orc_xorwow_init(uint64_t seed, uint64_t subsequence, uint64_t offset, uint32_t state[6]) { xorwow_init(seed, subsequence, offset, state); }
void orc_xorwow_init_many(uint64_t seed, uint32_t n, uint32_t* states) {
    /* init_rand_state: curand_init(PT_SEED, idx, 0) (synerfgine/common.cu:22-26) */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) xorwow_init(seed, (uint64_t)i, 0, states + 6 * i);
}
uint32_t orc_xorwow_next(uint32_t state[6]) { return xorwow_next(state); }
float orc_curand_uniform(uint32_t state[6]) { return curand_uniform(state); }
void orc_xorwow_jump_steps_naive(uint32_t st[6], uint64_t steps) { for (uint64_t i = 0; i < steps; ++i) xorwow_next(st); }
void orc_xorwow_jump_matrix(uint32_t st[6], uint32_t log2_steps) {
    /* 0..63: M^(2^k) from step_pow; 67..98: the subsequence tables M^(2^67 * 2^(k-67)) */
    const XorwowTables& T = xorwow_tables();
    if (log2_steps < 64) gf2_apply(T.step_pow[log2_steps], st, st);
    else if (log2_steps >= 67 && log2_steps < 99) gf2_apply(T.seq_pow[log2_steps - 67], st, st);
    else return;
    if (log2_steps < 32) st[5] += (uint32_t)((1ull << log2_steps) * 362437ull);   /* 2^k * 362437 == 0 mod 2^32 for k >= 32 */
}

uint32_t orc_grid_level_table(const orc_model* m, uint32_t* offsets, uint32_t* resolutions) {
    Grid g = make_grid(m);
    for (uint32_t i = 0; i <= g.L; ++i) offsets[i] = g.offsets[i];
    for (uint32_t i = 0; i < g.L; ++i) resolutions[i] = g.res[i];
    return g.offsets[g.L];
}
uint32_t orc_n_params(const orc_model* m) { return 3072 + 7168 + make_grid(m).offsets[m->n_levels] * m->n_features; }

void orc_hashgrid_encode(const orc_model* m, const float* coords, uint32_t stride, uint32_t n, uint16_t* out) {
    Grid g = make_grid(m);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) encode_one(g, coords + (size_t)i * stride, out + (size_t)i * g.L * g.F);
}
void orc_sh_encode(const float* coords, uint32_t stride, uint32_t dir_offset, uint32_t n, uint16_t* out) {
    for (uint32_t i = 0; i < n; ++i) {
        const float* c = coords + (size_t)i * stride + dir_offset;
        sh_one(c[0], c[1], c[2], out + 16 * (size_t)i);
    }
}
void orc_nerf_inference(const orc_model* m, const float* coords, uint32_t stride, uint32_t n, uint16_t* out) {
    Grid g = make_grid(m);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) network_one(m, g, coords + (size_t)i * stride, out + 16 * (size_t)i);
}

/* update_density_grid_mean_and_bitfield: testbed_nerf.cu:3212-3229,
 * grid_to_bitfield 285-309, bitfield_max_pool 311-332 */
void orc_density_grid_to_bitfield(const uint16_t* grid_f16, uint32_t max_cascade, uint8_t* bf, float* mean_out) {
    const uint32_t N = NERF_GRID_N_CELLS;
    std::vector<float> grid((size_t)N * (max_cascade + 1));
    for (size_t i = 0; i < grid.size(); ++i) grid[i] = h2f(grid_f16[i]);
    double sum = 0.0;
    for (uint32_t i = 0; i < N; ++i) sum += (double)(std::fmax(grid[i], 0.f) / N);
    float mean = (float)sum;
    if (mean_out) *mean_out = mean;
    float thresh = std::min(NERF_MIN_OPTICAL_THICKNESS, mean);
    uint32_t n_elements = N / 8 * NERF_CASCADES, n_nonzero = N / 8 * (max_cascade + 1);
    for (uint32_t i = 0; i < n_elements; ++i) {
        if (i >= n_nonzero) { bf[i] = 0; continue; }
        uint8_t bits = 0;
        for (uint8_t j = 0; j < 8; ++j) bits |= grid[i * 8 + j] > thresh ? ((uint8_t)1 << j) : 0;
        bf[i] = bits;
    }
    for (uint32_t level = 1; level < NERF_CASCADES; ++level) {
        const uint8_t* prev = bf + (size_t)N / 8 * (level - 1);
        uint8_t* next = bf + (size_t)N / 8 * level;
        for (uint32_t i = 0; i < N / 64; ++i) {
            uint8_t bits = 0;
            for (uint8_t j = 0; j < 8; ++j) bits |= prev[i * 8 + j] > 0 ? ((uint8_t)1 << j) : 0;
            uint32_t x = morton3D_invert(i >> 0) + NERF_GRIDSIZE / 8;
            uint32_t y = morton3D_invert(i >> 1) + NERF_GRIDSIZE / 8;
            uint32_t z = morton3D_invert(i >> 2) + NERF_GRIDSIZE / 8;
            next[morton3D(x, y, z)] |= bits;
        }
    }
}

/* Testbed::render_nerf_with_buffers (testbed_nerf.cu:2467-2613) with
 * NerfTracer::init_rays_from_camera (2037-2120) and trace_alt (2128-2277). */
/* ngp = 0: SyNeRFgine's trace_alt + composite_kernel_nerf_alt + extract_from_payload + normals.
 * ngp = 1: instant-NGP's NerfTracer::trace (2279-2401) + composite_kernel_nerf (577-788) +
 *          shade_kernel_nerf (1788-1828): depth at the max-weight sample, no payload.t reset,
 *          render modes AO / Shade / Positions / Depth / Cost / EncodingVis. */
static void render_nerf_impl(const orc_model* m, const orc_volume* vdesc, const orc_camera* c, int ngp, int render_mode, float depth_scale,
                             float* frame_rgba, float* frame_depth, float* positions, float* normals, orc_nerf_stats* stats) {
    Volume vol = make_volume(vdesc);
    Grid g = make_grid(m);
    const int W = c->res[0], H = c->res[1];
    const uint32_t n_px = (uint32_t)W * H;
    M43 cam = m43_load(c->camera);
    /* get_xform_given_rolling_shutter({camera0, camera1}, rolling_shutter, uv, motionblur_time), testbed_nerf.cu:1895 */
    const Quat q0 = quat_from_m3(m3_of(cam));
    M43 cam1 = g_has_cam1 ? m43_load(g_cam1) : cam;
    const Quat q1 = quat_from_m3(m3_of(cam1));
    const V3 pos1 = cam1.c[3];
    V2 focal = {c->focal[0], c->focal[1]};
    V2 sc = {c->screen_center[0], c->screen_center[1]};
    V3 cam_fwd = cam.c[2], cam_pos = cam.c[3];
    if (stats) std::memset(stats, 0, sizeof(*stats));

    /* init_rays_with_payload_kernel_nerf: testbed_nerf.cu:1855-1970 */
    std::vector<RayState> rays(n_px);
    V2 pixel_offset = ld_random_pixel_offset(c->snap_to_pixel_centers ? 0 : c->spp);
#pragma omp parallel for schedule(static)
    for (int64_t idx = 0; idx < (int64_t)n_px; ++idx) {
        int x = (int)(idx % W), y = (int)(idx / W);
        RayState& r = rays[idx];
        r.rgba = {0, 0, 0, 0};
        r.depth = 0.0f; /* cudaMemsetAsync(m_rays[0].depth, 0) 2103 */
        Payload& p = r.p;
        p.max_weight = 0.0f;
        frame_depth[idx] = MAX_DEPTH;
        V2 uv = {((float)x + pixel_offset.x) / (float)W, ((float)y + pixel_offset.y) / (float)H};
        /* uv_to_ray (common_device.cuh:403-470) with identity foveation, the render lens, no parallax, aperture 0, near 0 */
        V3 dir;
        const bool valid = uv_to_ray_dir(g_render_lens, uv, W, H, focal, sc, &dir);
        const float pixel_t = g_rs[0] + g_rs[1] * uv.x + g_rs[2] * uv.y + g_rs[3] * ld_random_val(c->spp, (uint32_t)idx * 72239731u);
        dir = mul(shutter_rotation(q0, q1, pixel_t), dir);
        V3 origin = cam_pos + (pos1 - cam_pos) * pixel_t;
        p.origin = origin;
        if (!valid) { p.alive = false; p.dir = normalize(dir); p.idx = (uint32_t)idx; continue; }   /* !ray.is_valid() (1919-1923) */
        frame_rgba[4 * idx + 0] = 0.0f; frame_rgba[4 * idx + 1] = 0.0f; frame_rgba[4 * idx + 2] = 0.0f; /* rgb only */
        dir = normalize(dir);
        float t = std::fmax(bb_ray_intersect(vol.render_aabb, to_local(vol, origin), to_local(vol, dir)).x, 0.0f) + 1e-6f;
        p.origin = origin;
        if (!bb_contains(vol.render_aabb, to_local(vol, origin + dir * t))) { p.alive = false; p.dir = dir; p.idx = (uint32_t)idx; continue; }
        p.dir = dir; p.t = t; p.idx = (uint32_t)idx; p.n_steps = 0; p.alive = true;
        /* advance_pos_nerf: testbed_nerf.cu:334-363 */
        V3 idir = v3(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
        float cone = vol.cone; /* calc_cone_angle returns the constant (nerf_device.cuh:370-377) */
        float tt = advance_n_steps(p.t, cone, ld_random_val(c->spp, p.idx * 786433u));
        tt = if_unoccupied_advance_to_next_occupied_voxel(tt, cone, origin, dir, idir, vol.bitfield, 0, vol.max_mip, vol);
        if (tt >= MAX_DEPTH) p.alive = false;
        else p.t = tt;
    }
    for (uint32_t i = 0; i < n_px; ++i) { positions[3 * i] = positions[3 * i + 1] = positions[3 * i + 2] = 0.0f; normals[3 * i] = normals[3 * i + 1] = normals[3 * i + 2] = 0.0f; }

    /* trace_alt: double-buffered wavefront, testbed_nerf.cu:2155-2277 */
    std::vector<RayState> current, hit;
    std::vector<RayState>* src = &rays;
    std::vector<float> coords;
    std::vector<uint16_t> outs;
    uint32_t i_step = 1, iter = 0;
    uint32_t n_alive = n_px;
    const uint32_t target = c->target_n_queries ? c->target_n_queries : 2u * 1024u * 1024u;
    while (i_step < MARCH_ITER) {
        /* compact_kernel_nerf 1830-1853 (order: stable, deterministic) */
        current.clear();
        for (uint32_t i = 0; i < n_alive; ++i) {
            const RayState& r = (*src)[i];
            if (r.p.alive) current.push_back(r);
            else if (r.rgba.w > 0.001f) hit.push_back(r);
        }
        n_alive = (uint32_t)current.size();
        if (n_alive == 0) break;
        uint32_t n_steps = wavefront_steps(n_alive, target);
        if (stats && iter < 64) { stats->alive_per_iter[iter] = n_alive; stats->steps_per_iter[iter] = n_steps; }
        ++iter;
        /* generate_next_nerf_network_inputs 790-837; slot i + j*n_alive */
        coords.assign((size_t)n_alive * n_steps * 7, 0.0f);
        uint64_t real = 0;
#pragma omp parallel for schedule(static) reduction(+ : real)
        for (int64_t i = 0; i < (int64_t)n_alive; ++i) {
            Payload& p = current[i].p;
            V3 o = p.origin, d = p.dir, idir = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
            float t = p.t;
            uint32_t j = 0;
            bool exhausted = false;
            for (; j < n_steps; ++j) {
                t = if_unoccupied_advance_to_next_occupied_voxel(t, vol.cone, o, d, idir, vol.bitfield, 0, vol.max_mip, vol);
                if (t >= MAX_DEPTH) { p.n_steps = (uint16_t)j; exhausted = true; break; }
                float dt = calc_dt(t, vol.cone);
                V3 wp = warp_position(o + d * t, vol.train_aabb);
                V3 wd = warp_direction(d);
                float* cc = &coords[((size_t)i + (size_t)j * n_alive) * 7];
                cc[0] = wp.x; cc[1] = wp.y; cc[2] = wp.z; cc[3] = warp_dt(dt); cc[4] = wd.x; cc[5] = wd.y; cc[6] = wd.z;
                t += dt;
            }
            if (!exhausted) { p.t = t; p.n_steps = (uint16_t)n_steps; }
            real += exhausted ? j : n_steps;
        }
        if (stats) { stats->n_samples += real; stats->n_slots += wavefront_elements(n_alive, n_steps); }
        /* inference_mixed_precision on the real slots (stale slots do not affect results) */
        outs.assign((size_t)n_alive * n_steps * 4, 0);
#pragma omp parallel for schedule(dynamic, 256)
        for (int64_t s = 0; s < (int64_t)n_alive * n_steps; ++s) {
            uint32_t i = (uint32_t)(s % n_alive), j = (uint32_t)(s / n_alive);
            if (j >= current[i].p.n_steps) continue;
            uint16_t o16[16];
            network_one(m, g, &coords[(size_t)s * 7], o16);
            std::memcpy(&outs[(size_t)s * 4], o16, 8);
            if (ngp && (render_mode == 2 || render_mode == 10)) probe_one(m, g, &coords[(size_t)s * 7], render_mode);
        }
        /* composite_kernel_nerf_alt 476-575 */
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)n_alive; ++i) {
            RayState& r = current[i];
            Payload& p = r.p;
            V4 lr = r.rgba;
            float ld = r.depth;
            uint32_t actual = p.n_steps, j = 0;
            for (; j < actual; ++j) {
                const uint16_t* o = &outs[((size_t)i + (size_t)j * n_alive) * 4];
                const float* cc = &coords[((size_t)i + (size_t)j * n_alive) * 7];
                V3 pos = unwarp_position(v3(cc[0], cc[1], cc[2]), vol.train_aabb);
                float T = 1.f - lr.w;
                float dt = unwarp_dt(cc[3]);
                float alpha = 1.f - det_expf(-det_expf(h2f(o[3])) * dt);
                float weight = alpha * T;
                V3 rgb = v3(logistic(h2f(o[0])), logistic(h2f(o[1])), logistic(h2f(o[2])));
                if (ngp && g_glow_mode) glow_term(pos, cam_pos, rgb, weight);
                if (ngp) {
                    if (render_mode == 2) {                                                                /* Normals */
                        const float dd = det_expf(std::min(std::max(h2f(o[3]), -15.0f), 15.0f));  /* network_to_density_derivative */
                        rgb = normalize(v3(cc[0], cc[1], cc[2]) * -dd);
                    } else if (render_mode == 3) rgb = (pos - 0.5f) / 2.0f + 0.5f;                         /* Positions */
                    else if (render_mode == 10) rgb = v3(cc[0], cc[1], cc[2]);                             /* EncodingVis */
                    else if (render_mode == 4) rgb = v3s(dot(cam_fwd, pos - p.origin) * depth_scale);      /* Depth */
                    else if (render_mode == 0) rgb = v3s(alpha);                                           /* AO */
                }
                lr.x += rgb.x * weight; lr.y += rgb.y * weight; lr.z += rgb.z * weight; lr.w += weight;
                if (ngp) {
                    if (weight > p.max_weight) { p.max_weight = weight; ld = dot(cam_fwd, pos - cam_pos); }
                } else {
                    ld = dot(cam_fwd, pos - cam_pos);
                    if (weight > p.max_weight) p.max_weight = weight;
                }
                if (lr.w > (1.0f - vol.min_transmittance)) {
                    float a = lr.w;
                    lr.x /= a; lr.y /= a; lr.z /= a; lr.w /= a;
                    break;
                }
            }
            if (j < n_steps) { p.alive = false; p.n_steps = (uint16_t)(j + i_step); }
            r.rgba = lr;
            r.depth = ld;
            if (!ngp) p.t = ld / dot(cam_fwd, p.dir);   /* composite_kernel_nerf_alt:574; trace keeps generate's t */
        }
        src = &current;
        std::vector<RayState> tmp = current; /* next compaction reads this buffer */
        rays.swap(tmp);
        src = &rays;
        i_step += n_steps;
    }
    if (stats) { stats->n_iterations = iter; stats->n_hit = (uint32_t)hit.size(); }

    if (ngp) {
        /* shade_kernel_nerf 1788-1828 (gbuffer_hard_edges = false, train_in_linear_colors = false) */
        for (const RayState& r : hit) {
            const Payload& p = r.p;
            V4 tmp = r.rgba;
            if (render_mode == 6) { float col = (float)p.n_steps / 128; tmp = {col, col, col, 1.0f}; }   /* Cost */
            if (render_mode == 1) { tmp.x = srgb_to_linear(tmp.x); tmp.y = srgb_to_linear(tmp.y); tmp.z = srgb_to_linear(tmp.z); }
            float* fb = &frame_rgba[4 * (size_t)p.idx];
            fb[0] = tmp.x + fb[0] * (1.0f - tmp.w);
            fb[1] = tmp.y + fb[1] * (1.0f - tmp.w);
            fb[2] = tmp.z + fb[2] * (1.0f - tmp.w);
            fb[3] = tmp.w + fb[3] * (1.0f - tmp.w);
            if (tmp.w > 0.2f) frame_depth[p.idx] = r.depth;
        }
        return;
    }
    /* extract_from_payload 1578-1612 (Shade mode) */
    for (const RayState& r : hit) {
        const Payload& p = r.p;
        V3 orig_pos = cam_pos + p.dir * p.t;
        float* fb = &frame_rgba[4 * (size_t)p.idx];
        V4 tmp = {srgb_to_linear(r.rgba.x), srgb_to_linear(r.rgba.y), srgb_to_linear(r.rgba.z), r.rgba.w};
        fb[0] = tmp.x + fb[0] * (1.0f - tmp.w);
        fb[1] = tmp.y + fb[1] * (1.0f - tmp.w);
        fb[2] = tmp.z + fb[2] * (1.0f - tmp.w);
        fb[3] = tmp.w + fb[3] * (1.0f - tmp.w);
        positions[3 * p.idx + 0] = orig_pos.x; positions[3 * p.idx + 1] = orig_pos.y; positions[3 * p.idx + 2] = orig_pos.z;
        if (tmp.w > 0.2f) frame_depth[p.idx] = r.depth;
    }

    /* write_normals_to_buffer 1523-1576 */
    static const int OFF[9][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}, {2, 0}, {0, 2}, {-2, 0}, {0, -2}, {1, 0}};
#pragma omp parallel for schedule(static)
    for (int64_t idx = 0; idx < (int64_t)n_px; ++idx) {
        int x = (int)(idx % W), y = (int)(idx / W);
        V3 pos = v3(positions[3 * idx], positions[3 * idx + 1], positions[3 * idx + 2]);
        float factor = 0.0f;
        V3 N = v3s(0.0f);
        for (int t = 0; t < 8; ++t) {
            int tx = x + OFF[t + 1][0], ty = y + OFF[t + 1][1], bx = x + OFF[t][0], by = y + OFF[t][1];
            if (tx >= W || tx < 0 || ty >= H || ty < 0 || bx >= W || bx < 0 || by >= H || by < 0) continue;
            const float* pt = &positions[3 * ((size_t)ty * W + tx)];
            const float* pb = &positions[3 * ((size_t)by * W + bx)];
            V3 T = v3(pt[0], pt[1], pt[2]) - pos;
            V3 B = v3(pb[0], pb[1], pb[2]) - pos;
            N = N + normalize(cross(normalize(T), B)); /* sng::get_normal, synerfgine/common.cuh:55-57 */
            factor += 1.0f;
        }
        N = factor == 0.0f ? N : N / factor;
        V3 n = normalize(N);
        normals[3 * idx] = n.x; normals[3 * idx + 1] = n.y; normals[3 * idx + 2] = n.z;
    }
}

/* shade_nerf_shadows (testbed_nerf.cu:2628-2677) -> shade_with_shadow (1702-1786)
 * -> shadow_for_px (1614-1700).  The neighbourhood's light samples draw from the
 * centre pixel's own RNG stream (the reference shares neighbour states racily,
 * SURVEY Appendix A.5); identical to the reference for kernel_size/2 == 0. */
/* 1: shadow_for_px's light samples advance the NEIGHBOUR's XORWOW state, as the reference's rand_state[idx]
 * does (testbed_nerf.cu:1635,1649: idx is the neighbour's pixel), with the pixels serialised in index order --
 * one race-free interleaving of what the reference's threads do concurrently (orc_set_shadow_rng_mode) */
static int g_shadow_rng_neighbour = 0;
void orc_shade_nerf_shadows(const orc_volume* vdesc, const int32_t res[2], float* frame_rgba, const float* positions, const float* normals,
                            const orc_object* objd, uint32_t n_objs, const orc_light* lights, uint32_t n_lights,
                            uint32_t* rng, float nerf_shadow_intensity, float thr, int32_t kernel_size) {
    Volume vol = make_volume(vdesc);
    std::vector<Object> objs;
    for (uint32_t i = 0; i < n_objs; ++i) objs.push_back(make_object(objd[i]));
    const int W = res[0], H = res[1];
    const int r = kernel_size / 2;
    const uint32_t n_steps = MAX_STEPS_INBETWEEN_COMPACTION;
    const int neighbour_rng = g_shadow_rng_neighbour;
#pragma omp parallel for schedule(dynamic, 64) if (!neighbour_rng)
    for (int64_t idx = 0; idx < (int64_t)W * H; ++idx) {
        int x = (int)(idx % W), y = (int)(idx / W);
        float sum = 0.0f;
        int blend = 0;
        uint32_t* const st_centre = rng + 6 * idx;
        for (int i = -r; i <= r; ++i)
            for (int j = -r; j <= r; ++j) {
                int fx = x + i, fy = y + j;
                if (fx < 0 || fy < 0 || fx >= W || fy >= H) continue;
                size_t t = (size_t)fy * W + fx;
                uint32_t* st = neighbour_rng ? rng + 6 * t : st_centre;
                V3 pos = v3(positions[3 * t], positions[3 * t + 1], positions[3 * t + 2]);
                V3 nrm = v3(normals[3 * t], normals[3 * t + 1], normals[3 * t + 2]);
                float overall = 1.0f;
                for (uint32_t li = 0; li < n_lights; ++li) {
                    const orc_light& L = lights[li];
                    V3 lp = v3(L.pos[0], L.pos[1], L.pos[2]);
                    if (L.type == 0) {
                        /* Light::sample (light.cuh:71-77) */
                        float ox = fractf(curand_uniform(st)), oy = fractf(curand_uniform(st)), oz = fractf(curand_uniform(st));
                        V3 lpos = lp + v3(ox, oy, oz) * L.size * 1.0f;
                        V3 l = normalize(lpos - pos);
                        float full_d = length(lpos - pos);
                        int hit = -1;
                        float syn_depth = depth_test_world(pos, l, objs, hit);
                        float syn_mask = syn_depth / full_d;
                        overall = std::min(overall, pow_src(syn_mask, nerf_shadow_intensity));
                        V3 fract_offset = full_d * thr * lpos;
                        float nerf_depth = std::min(full_d, depth_test_nerf_sd(n_steps, vol.cone, pos + fract_offset, lpos, vol, 0, vol.max_mip));
                        /* (full_d * (1.0 - thr)) is a double expression (1664) */
                        double mask = (double)(nerf_depth * (1.0f - std::min(L.intensity, 0.0f))) / ((double)full_d * (1.0 - (double)thr));
                        overall = (float)std::fmin((double)overall, mask);
                    } else {
                        V3 l = normalize(lp - pos);
                        /* min(1.0, overall + min(0.0, dot(l, n)) * intensity): double (1677) */
                        double v = (double)overall + std::fmin(0.0, (double)dot(l, nrm)) * (double)L.intensity;
                        overall = (float)std::fmin(1.0, v);
                    }
                }
                sum += overall;
                ++blend;
            }
        sum /= (float)blend;
        sum = pow_src(sum, nerf_shadow_intensity);
        float* rgba = &frame_rgba[4 * idx];
        rgba[0] = srgb_to_linear(rgba[0]) * sum;
        rgba[1] = srgb_to_linear(rgba[1]) * sum;
        rgba[2] = srgb_to_linear(rgba[2]) * sum;
    }
}

/* TriangleBvhWithBranchingFactor<2>::build: triangle_bvh.cu:615-692 */
int32_t orc_bvh_build(float* trisf, uint32_t n_tris, uint32_t ppl, float* nodes_out, uint32_t cap) {
    std::vector<Tri> tris((Tri*)trisf, (Tri*)trisf + n_tris);
    std::vector<Node> nodes;
    auto bb_of = [&](std::vector<Tri>::iterator b, std::vector<Tri>::iterator e) {
        BBox bb;
        bb.min = bb.max = b->a;
        for (auto it = b; it != e; ++it) {
            bb.min = vmin3(bb.min, it->a); bb.max = vmax3(bb.max, it->a);
            bb.min = vmin3(bb.min, it->b); bb.max = vmax3(bb.max, it->b);
            bb.min = vmin3(bb.min, it->c); bb.max = vmax3(bb.max, it->c);
        }
        return bb;
    };
    nodes.push_back({});
    nodes.front().bb = bb_of(tris.begin(), tris.end());
    struct BuildNode { int node_idx; std::vector<Tri>::iterator begin, end; };
    std::stack<BuildNode> st;
    st.push({0, tris.begin(), tris.end()});
    while (!st.empty()) {
        BuildNode curr = st.top();
        st.pop();
        size_t node_idx = curr.node_idx;
        BuildNode children[2];
        children[0].begin = curr.begin;
        children[0].end = curr.end;
        int n_children = 1;
        while (n_children < 2) {
            for (int i = n_children - 1; i >= 0; --i) {
                auto& child = children[i];
                V3 mean = v3s(0.0f);
                for (auto it = child.begin; it != child.end; ++it) mean = mean + tri_centroid(*it);
                mean = mean / (float)std::distance(child.begin, child.end);
                V3 var = v3s(0.0f);
                for (auto it = child.begin; it != child.end; ++it) { V3 d = tri_centroid(*it) - mean; var = var + d * d; }
                var = var / (float)std::distance(child.begin, child.end);
                float mv = vmax(var);
                int axis = var.x == mv ? 0 : (var.y == mv ? 1 : 2);
                auto mid = child.begin + std::distance(child.begin, child.end) / 2;
                std::nth_element(child.begin, mid, child.end, [&](const Tri& a, const Tri& b) { return tri_centroid_axis(a, axis) < tri_centroid_axis(b, axis); });
                children[i * 2].begin = children[i].begin;
                children[i * 2 + 1].end = children[i].end;
                children[i * 2].end = children[i * 2 + 1].begin = mid;
            }
            n_children *= 2;
        }
        nodes[node_idx].left = (int)nodes.size();
        for (int i = 0; i < 2; ++i) {
            auto& child = children[i];
            child.node_idx = (int)nodes.size();
            nodes.push_back({});
            nodes.back().bb = bb_of(child.begin, child.end);
            if ((uint32_t)std::distance(child.begin, child.end) <= ppl) {
                nodes.back().left = -(int)std::distance(tris.begin(), child.begin) - 1;
                nodes.back().right = -(int)std::distance(tris.begin(), child.end) - 1;
            } else {
                st.push(child);
            }
        }
        nodes[node_idx].right = (int)nodes.size();
    }
    if (nodes.size() > cap) return -1;
    for (size_t i = 0; i < nodes.size(); ++i) {
        float* n = nodes_out + 8 * i;
        n[0] = nodes[i].bb.min.x; n[1] = nodes[i].bb.min.y; n[2] = nodes[i].bb.min.z;
        n[3] = nodes[i].bb.max.x; n[4] = nodes[i].bb.max.y; n[5] = nodes[i].bb.max.z;
        std::memcpy(&n[6], &nodes[i].left, 4);
        std::memcpy(&n[7], &nodes[i].right, 4);
    }
    std::memcpy(trisf, tris.data(), n_tris * sizeof(Tri));
    return (int32_t)nodes.size();
}

void orc_depth_test_world(const orc_object* objd, uint32_t n_objs, const float* o, const float* d, uint32_t n, float* t_out, int32_t* obj_out) {
    std::vector<Object> objs;
    for (uint32_t i = 0; i < n_objs; ++i) objs.push_back(make_object(objd[i]));
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        int hit = -1;
        t_out[i] = depth_test_world(v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]), objs, hit);
        obj_out[i] = hit;
    }
}

/* sng::init_rays_with_payload_kernel_nerf: synerfgine/raytracer.cu:59-99 */
void orc_mesh_init_rays(const orc_camera* c, float* origins, float* dirs, float* acc_rgba, float* acc_depth) {
    const int W = c->res[0], H = c->res[1];
    M43 cam = m43_load(c->camera);
    M3 rot = m3_of(cam);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            size_t idx = (size_t)y * W + x;
            V2 uv = {(float)x / (float)W, (float)y / (float)H};
            V3 dir = v3((uv.x - c->screen_center[0]) * (float)W / c->focal[0], (uv.y - c->screen_center[1]) * (float)H / c->focal[1], 1.0f);
            dir = mul(rot, dir);
            dir = normalize(dir);
            origins[3 * idx] = cam.c[3].x; origins[3 * idx + 1] = cam.c[3].y; origins[3 * idx + 2] = cam.c[3].z;
            dirs[3 * idx] = dir.x; dirs[3 * idx + 1] = dir.y; dirs[3 * idx + 2] = dir.z;
            acc_rgba[4 * idx] = 0.0f; acc_rgba[4 * idx + 1] = 0.0f; acc_rgba[4 * idx + 2] = 0.0f; acc_rgba[4 * idx + 3] = 1.0f;
            acc_depth[idx] = MAX_DEPTH;
        }
}

}  // extern "C"

namespace {
/* sng::cone_random(orig, perturb_frame, longi, latid): synerfgine/common.cuh:33-36 */
inline V3 cone_random_frame(V3 orig, const M3& frame, float longi, float latid) {
    V3 off = v3(std::cos(longi) * std::sin(latid), std::sin(longi) * std::sin(latid), std::cos(longi));
    return orig + mul(frame, off);
}
/* sng::cone_random(orig, up, longi, latid): synerfgine/common.cuh:37-48 */
inline V3 cone_random_up(V3 orig, V3 up, float longi, float latid) {
    V3 N = normalize(orig);
    V3 B = normalize(cross(N, up));
    V3 T = cross(B, N);
    M3 frame = {{T, B, N}};
    V3 off = v3(std::sin(longi) * std::cos(latid), std::sin(longi) * std::sin(latid), std::cos(longi));
    return orig + mul(frame, off);
}
inline V3 reflect(V3 i, V3 n) { return 2.0f * dot(i, n) * n - i; }
struct SampledRay { V3 pos = v3s(0.0f), dir = v3s(0.0f); float pdf = 0.0f, attenuation = 1.0f; };
/* Material::local_color (material.cuh:96-98) */
inline V3 local_color(const orc_material& m, V3 L, V3 N, V3 R, V3 V, const orc_light& light) {
    float a = std::max(0.0f, dot(L, N));
    V3 kd = v3(m.kd[0], m.kd[1], m.kd[2]), ks = v3(m.ks[0], m.ks[1], m.ks[2]);
    return a * kd * light.intensity + pow_src(std::max(0.0f, dot(R, V)), m.n) * ks;
}
/* sng::shade_object: synerfgine/raytracer.cu:6-57 */
V4 shade_object(V3 wi, SampledRay& ray, uint32_t shadow_count, HitRecord& hit, const orc_light* lights, uint32_t n_lights,
                const std::vector<Object>& objs, const orc_material* mats, uint32_t n_steps, float cone, const Volume& vol,
                uint32_t min_mip, uint32_t max_mip, uint32_t* st, float& out_nerf_shadow, bool no_shadow, float syn_shadow_factor) {
    if (hit.material_idx < 0) return {0, 0, 0, 0};
    const orc_material& mat = mats[hit.material_idx];
    V3 color = v3s(0.0f);
    for (uint32_t l = 0; l < n_lights; ++l) {
        const orc_light& light = lights[l];
        V3 lp = v3(light.pos[0], light.pos[1], light.pos[2]);
        for (uint32_t s = 0; s < shadow_count; ++s) {
            float ox = fractf(curand_uniform(st)), oy = fractf(curand_uniform(st)), oz = fractf(curand_uniform(st));
            V3 lpos = lp + v3(ox, oy, oz) * light.size * 1.0f;
            V3 L = lpos - hit.pos;
            float full_dist = length(L);
            L = normalize(L);
            if (light.type == 0) {
                V3 invL = v3(1.0f / L.x, 1.0f / L.y, 1.0f / L.z);
                int obj_hit = -1;
                float syn_shadow = no_shadow ? 1.0f : depth_test_world(hit.pos, L, objs, obj_hit);
                /* full_d = syn_shadow + 1.0 is a double expression bound to const float& */
                float nerf_shadow = no_shadow ? 1.0f : depth_test_nerf_fd((float)((double)syn_shadow + 1.0), n_steps, cone, hit.pos, L, invL, vol, min_mip, max_mip);
                out_nerf_shadow = std::min(nerf_shadow / full_dist, out_nerf_shadow);
                float shadow = std::min(std::min(nerf_shadow, syn_shadow), full_dist);
                float mask = smoothstep(shadow / full_dist);
                mask = pow_src(mask, syn_shadow_factor);
                V3 R = reflect(L, hit.normal);
                V3 V = normalize(-wi);
                color = color + local_color(mat, L, hit.normal, R, V, light) * mask;
            } else {
                V3 R = reflect(L, hit.normal);
                V3 V = normalize(-wi);
                color = color + local_color(mat, L, hit.normal, R, V, light);
            }
        }
    }
    color = color / (float)shadow_count;
    color = color + v3(mat.ka[0], mat.ka[1], mat.ka[2]);
    /* Material::scatter(hit, wi, ray, rand) (material.cuh:112-123) */
    ray.pos = hit.pos;
    if (mat.type == 0 || mat.type == 1) {
        float spec = mat.type == 0 ? PI_F / 2 : mat.spec_angle;
        ray.dir = reflect(-wi, hit.normal);
        float longi = curand_uniform(st) * spec;
        float latid = (float)((double)curand_uniform(st) * 2.0 * (double)PI_F); /* double expression */
        ray.dir = cone_random_frame(hit.normal, hit.perturb, longi, latid);
        ray.pdf = 1.0f / std::max(1.0f, spec * 2.0f);
        ray.attenuation *= mat.rg;
    }
    return {color.x, color.y, color.z, 1.0f};
}
}  // namespace

extern "C" {

/* sng::raytrace: synerfgine/raytracer.cu:101-218, every ImgBufferType (raytracer.cuh:20-30) */
void orc_raytrace(const orc_volume* vdesc, const float* camera, const orc_frame_params* P,
                  const orc_object* objd, uint32_t n_objs, const orc_light* lights, uint32_t n_lights,
                  const orc_material* mats, uint32_t n_mats, const float* origins, const float* dirs, uint32_t n,
                  uint32_t* rng, float* acc_rgba, float* acc_depth) {
    (void)n_mats;
    Volume vol = make_volume(vdesc);
    std::vector<Object> objs;
    for (uint32_t i = 0; i < n_objs; ++i) objs.push_back(make_object(objd[i]));
    M43 cam = m43_load(camera);
    const V3 up_vec = cam.c[0];
    const float lens = P->lens_angle_constant;
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint32_t* st = rng + 6 * i;
        V3 src_p = v3(origins[3 * i], origins[3 * i + 1], origins[3 * i + 2]);
        V3 src_d = v3(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        V3 shade = v3s(0.0f), normal = v3s(0.0f), view_pos = v3s(0.0f), next_pos = v3s(0.0f), view_dir = v3s(0.0f), next_dir = v3s(0.0f);
        float nerf_shadow = 1.0f;
        for (uint32_t spp = 0; spp < P->light_samples; ++spp) {
            SampledRay ray;
            float longi = curand_uniform(st) * lens;
            /* lens ? 0.0 : curand_uniform * 2.0 * PI -- second draw only when lens == 0 */
            float latid = lens != 0.0f ? 0.0f : (float)((double)curand_uniform(st) * 2.0 * (double)PI_F);
            ray.pos = src_p;
            ray.dir = cone_random_up(src_d, up_vec, longi, latid);
            ray.pdf = 1.0f / (float)P->path_trace_depth;
            ray.attenuation = 1.0f;
            V3 shade_s = v3s(0.0f);
            for (uint32_t bounce = 0; bounce < P->path_trace_depth; ++bounce) {
                V3 sp = ray.pos, sd = ray.dir;
                HitRecord hit;
                int hit_obj = -1;
                depth_test_world_hit(sp, sd, objs, hit_obj, hit);
                if (!bounce) { normal = normal + hit.normal; view_pos = view_pos + sp; view_dir = view_dir + sd; next_pos = next_pos + hit.pos; }
                if (hit_obj < 0) break;
                SampledRay next;
                V4 color = shade_object(sd, next, P->shadow_iters, hit, lights, n_lights, objs, mats, P->shadow_steps, vol.cone, vol, 0,
                                        vol.max_mip, st, nerf_shadow, !P->shadow_on_virtual_obj, P->syn_shadow_factor);
                shade_s = shade_s + v3(color.x, color.y, color.z) * ray.pdf * ray.attenuation;
                if (!bounce) next_dir = next_dir + next.dir;
                ray = next;
            }
            shade = shade + shade_s;
        }
        float weight = (float)P->light_samples;
        view_pos = view_pos / weight; view_dir = view_dir / weight; next_pos = next_pos / weight;
        next_dir = next_dir / weight; normal = normal / weight; shade = shade / weight;
        float depth = dot(src_d, next_pos - src_p);
        acc_depth[i] = depth;
        V3 curr = v3(acc_rgba[4 * i], acc_rgba[4 * i + 1], acc_rgba[4 * i + 2]);
        /* vec3_to_col (common.cu:300-302) */
        auto to_col = [](V3 v) { return v * 0.5f + v3s(0.5f); };
        V3 out;
        switch (P->rt_buffer_type) {   /* raytracer.cu:189-216 */
        case 1: out = length(next_pos - view_pos) + MIN_DEPTH > MAX_DEPTH ? v3s(0.0f) : to_col(normalize(next_pos)); break;   /* NextOrigin */
        case 2: out = to_col(normalize(view_pos)); break;   /* SrcOrigin */
        case 3: out = to_col(next_dir); break;              /* NextDirection */
        case 4: out = to_col(view_dir); break;              /* SrcDirection */
        case 5: out = to_col(normal); break;                /* Normal */
        case 6: out = v3s(depth); break;                    /* Depth */
        case 7: out = v3s(nerf_shadow); break;              /* NerfShadow */
        default:                                            /* Final */
            if (dot(curr, curr) > 0.001f) shade = shade * 0.5f + curr * 0.5f;
            out = shade;
            break;
        }
        acc_rgba[4 * i] = out.x; acc_rgba[4 * i + 1] = out.y; acc_rgba[4 * i + 2] = out.z;
    }
}

/* sng_tonemap: synerfgine/common.cu:186-243 (ETonemapCurve, common.h:113: 0 Identity, 1 ACES, 2 Hable, 3 Reinhard) */
V3 sng_tonemap(V3 x, int curve) {
    if (curve == 0) return x;
    x = v3(std::max(x.x, 0.0f), std::max(x.y, 0.0f), std::max(x.z, 0.0f));
    float k0, k1, k2, k3, k4, k5;
    if (curve == 1) {   /* ACES approximation, pre-exposure cancelled into the constants */
        k0 = 0.6f * 0.6f * 2.51f;
        k1 = 0.6f * 0.03f;
        k2 = 0.0f;
        k3 = 0.6f * 0.6f * 2.43f;
        k4 = 0.6f * 0.59f;
        k5 = 0.14f;
    } else if (curve == 2) {   /* Hable, white point 11.2, white scale and exposure bias folded in */
        const float A = 0.15f, B = 0.50f, C = 0.10f, D = 0.20f, E = 0.02f, F = 0.30f;
        k0 = A * F - A * E;
        k1 = C * B * F - B * E;
        k2 = 0.0f;
        k3 = A * F;
        k4 = B * F;
        k5 = D * F * F;
        const float W = 11.2f;
        const float nom = k0 * (W * W) + k1 * W + k2;
        const float denom = k3 * (W * W) + k4 * W + k5;
        const float white_scale = denom / nom;
        k0 = 4.0f * k0 * white_scale;
        k1 = 2.0f * k1 * white_scale;
        k2 = k2 * white_scale;
        k3 = 4.0f * k3;
        k4 = 2.0f * k4;
    } else {   /* Reinhard on luminance */
        const float Y = 0.2126f * x.x + 0.7152f * x.y + 0.0722f * x.z;
        return x * (1.f / (Y + 1.0f));
    }
    const V3 sq = x * x;
    const V3 nom = sq * k0 + x * k1 + k2;
    const V3 denom = sq * k3 + x * k4 + k5;
    return v3(nom.x / denom.x, nom.y / denom.y, nom.z / denom.z);
}

/* sng::overlay_nerf: synerfgine/raytracer.cu:220-258 */
void orc_overlay(const orc_frame_params* P, const float* syn_rgba, const float* syn_depth, const float* nerf_rgba, const float* nerf_depth,
                 float* final_rgba, float* final_depth) {
    const int W = P->mesh_res[0], H = P->mesh_res[1], s = P->syn_px_scale;
    const int nW = W / s;
    const int n_nerf = P->nerf_res[0] * P->nerf_res[1];
    float e = std::pow(2.0f, P->exposure);
    const float qnan = std::numeric_limits<float>::quiet_NaN();
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int sid = x + y * W;
            int nid = (x / s) + (y / s) * nW;
            float* f = &final_rgba[4 * (size_t)sid];
            final_depth[sid] = syn_depth[sid];
            if (nid >= n_nerf) {
                if (g_literal) { f[0] = f[1] = f[2] = f[3] = qnan; continue; }   /* the reference reads past the buffer */
                nid = n_nerf - 1;                                               /* the product clamps */
            }
            const float* sr = &syn_rgba[4 * (size_t)sid];
            const float* nr = &nerf_rgba[4 * (size_t)nid];
            float sdepth = syn_depth[sid], ndepth = nerf_depth[nid];
            const float* use = (!P->show_nerf || sdepth - P->rt_depth_offset < ndepth) ? sr : nr;
            V3 rgb = sng_tonemap(v3(use[0] * e, use[1] * e, use[2] * e), P->tonemap_curve);
            f[0] = rgb.x; f[1] = rgb.y; f[2] = rgb.z;
            if (P->srgb_output) for (int k = 0; k < 3; ++k) f[k] = linear_to_srgb(f[k]);
            f[3] = use[3];
        }
}

/* Engine::frame (synerfgine/engine.cu:352-433): raytrace -> NeRF render (+ shadows) -> overlay.
 * The mesh layer is re-initialised (camera reset semantics, raytracer.cu:327-336). */
static float *g_gbuf_pos = nullptr, *g_gbuf_nrm = nullptr;
void orc_set_gbuffer_out(float* positions, float* normals) {
    g_gbuf_pos = positions;
    g_gbuf_nrm = normals;
}
void orc_render_frame(const orc_model* m, const orc_volume* v, const orc_camera* nerf_cam, const orc_camera* mesh_cam,
                      const orc_frame_params* P, const orc_object* objs, uint32_t n_objs, const orc_light* lights, uint32_t n_lights,
                      const orc_material* mats, uint32_t n_mats, uint32_t* nerf_rng, uint32_t* mesh_rng,
                      float* final_rgba, float* final_depth, float* nerf_rgba, float* nerf_depth, orc_nerf_stats* stats) {
    size_t n_mesh = (size_t)mesh_cam->res[0] * mesh_cam->res[1];
    size_t n_nerf = (size_t)nerf_cam->res[0] * nerf_cam->res[1];
    std::vector<float> o(3 * n_mesh), d(3 * n_mesh), acc(4 * n_mesh), accd(n_mesh);
    orc_mesh_init_rays(mesh_cam, o.data(), d.data(), acc.data(), accd.data());
    if (P->show_virtual_obj)
        orc_raytrace(v, mesh_cam->camera, P, objs, n_objs, lights, n_lights, mats, n_mats, o.data(), d.data(), (uint32_t)n_mesh, mesh_rng, acc.data(), accd.data());
    if (P->show_nerf) {
        std::vector<float> pos(3 * n_nerf), nrm(3 * n_nerf);
        orc_render_nerf(m, v, nerf_cam, nerf_rgba, nerf_depth, pos.data(), nrm.data(), stats);
        if (g_gbuf_pos) std::memcpy(g_gbuf_pos, pos.data(), pos.size() * sizeof(float));   /* the NeRF G-buffer (A10c) */
        if (g_gbuf_nrm) std::memcpy(g_gbuf_nrm, nrm.data(), nrm.size() * sizeof(float));
        if (P->shadow_on_nerf)
            orc_shade_nerf_shadows(v, nerf_cam->res, nerf_rgba, pos.data(), nrm.data(), objs, n_objs, lights, n_lights, nerf_rng,
                                   P->nerf_shadow_intensity, P->nerf_on_nerf_shadow_threshold, P->nerf_kernel_size);
    }
    orc_overlay(P, acc.data(), accd.data(), nerf_rgba, nerf_depth, final_rgba, final_depth);
}

void orc_set_visualization(int32_t layer, int32_t dim) {
    g_vis_layer = layer;
    g_vis_dim = dim;
}
void orc_set_motion_blur(const float* camera1, const float* rolling_shutter) {
    g_has_cam1 = camera1 != nullptr;
    if (camera1) std::memcpy(g_cam1, camera1, sizeof(g_cam1));
    const float rs0[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    std::memcpy(g_rs, rolling_shutter ? rolling_shutter : rs0, sizeof(g_rs));
}
void orc_set_shadow_rng_mode(int32_t neighbour) { g_shadow_rng_neighbour = neighbour; }
void orc_set_render_lens(const orc_lens* lens) {
    g_render_lens = OrcLens{};
    if (lens) { g_render_lens.mode = lens->mode; std::memcpy(g_render_lens.params, lens->params, sizeof(g_render_lens.params)); }
}
int32_t orc_uv_to_ray_dir(const orc_lens* lens, const float* uv, int32_t W, int32_t H, const float* focal, const float* screen_center, float* dir) {
    OrcLens l;
    if (lens) { l.mode = lens->mode; std::memcpy(l.params, lens->params, sizeof(l.params)); }
    V3 d;
    const bool ok = uv_to_ray_dir(l, V2{uv[0], uv[1]}, W, H, V2{focal[0], focal[1]}, V2{screen_center[0], screen_center[1]}, &d);
    dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
    return ok ? 1 : 0;
}
void orc_lens_distortion_delta(const orc_lens* lens, float u, float v, float* du, float* dv) {
    if (lens->mode == 4) opencv_fisheye_lens_distortion_delta(lens->params, u, v, du, dv);
    else opencv_lens_distortion_delta(lens->params, u, v, du, dv);
}
void orc_set_train_lens(const orc_lens* lenses, uint32_t n) {
    g_train_lens.assign(n, OrcLens{});
    for (uint32_t i = 0; i < n; ++i) { g_train_lens[i].mode = lenses[i].mode; std::memcpy(g_train_lens[i].params, lenses[i].params, sizeof(lenses[i].params)); }
}
void orc_set_glow(int32_t mode, float y_cutoff) {
    g_glow_mode = mode;
    g_glow_y_cutoff = y_cutoff;
}
void orc_set_mlp_accum(int32_t mode, int32_t chunk) {
    g_mlp_accum = mode;
    g_mlp_chunk = chunk > 0 ? chunk : 16;
}

void orc_set_num_threads(int32_t n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int32_t orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

}  // extern "C"

void orc_render_nerf(const orc_model* m, const orc_volume* v, const orc_camera* c, float* frame_rgba, float* frame_depth, float* positions,
                     float* normals, orc_nerf_stats* stats) {
    render_nerf_impl(m, v, c, 0, 1, 1.0f, frame_rgba, frame_depth, positions, normals, stats);
}
void orc_render_nerf_ngp(const orc_model* m, const orc_volume* v, const orc_camera* c, int32_t render_mode, float depth_scale, float* frame_rgba,
                         float* frame_depth, orc_nerf_stats* stats) {
    const int W = c->res[0], H = c->res[1];
    std::vector<float> pos((size_t)W * H * 3), nrm((size_t)W * H * 3);
    render_nerf_impl(m, v, c, 1, render_mode, depth_scale, frame_rgba, frame_depth, pos.data(), nrm.data(), stats);
}

/* ---- online training ------------------------------------------------------- */
namespace {
/* tcnn pcg32 (random.h, after M. O'Neill's PCG32 / W. Jakob's pcg32.h) [tcnn, unvendored] */
struct OrcPcg32 {
    uint64_t state, inc;
    uint32_t next_uint() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31));
    }
    float next_float() {
        union { uint32_t u; float f; } x;
        x.u = (next_uint() >> 9) | 0x3f800000u;
        return x.f - 1.0f;
    }
    void advance(uint64_t delta) {
        uint64_t cur_mult = 0x5851f42d4c957f2dULL, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
        while (delta > 0) {
            if (delta & 1) { acc_mult *= cur_mult; acc_plus = acc_plus * cur_mult + cur_plus; }
            cur_plus = (cur_mult + 1) * cur_plus;
            cur_mult *= cur_mult;
            delta /= 2;
        }
        state = acc_mult * state + acc_plus;
    }
};
/* mip_from_dt (nerf_device.cuh:450-460) */
inline uint32_t mip_from_dt(float dt, V3 pos, uint32_t max_cascade) {
    uint32_t mip = mip_from_pos(pos, max_cascade);
    dt *= 2 * NERF_GRIDSIZE;
    if (dt < 1.0f) return mip;
    int exponent;
    std::frexp(dt, &exponent);
    return (uint32_t)std::min(std::max((int)mip, exponent), (int)max_cascade);
}
}  // namespace

extern "C" {
void orc_train_generate(const orc_volume* vdesc, const orc_train_images* im, uint64_t rng_state, uint64_t rng_inc, uint32_t n_rays,
                        uint32_t max_per_ray, uint32_t* numsteps, float* rays, float* coords) {
    const Volume vol = make_volume(vdesc);
    const BBox aabb = vol.train_aabb;
    for (uint32_t i = 0; i < n_rays; ++i) {
        numsteps[i] = 0;
        /* image_idx without a CDF (nerf_device.cuh:598) */
        const uint32_t img = ((i * (uint32_t)im->n) / n_rays) % (uint32_t)im->n;
        OrcPcg32 rng{rng_state, rng_inc};
        rng.advance((uint64_t)i * 16);   /* N_MAX_RANDOM_SAMPLES_PER_RAY (nerf_device.cuh:40) */
        /* nerf_random_image_pos_training with snap_to_pixel_centers (nerf_device.cuh:553-576; testbed.h:794) */
        float ux = rng.next_float();
        float uy = rng.next_float();
        int px = std::min(std::max((int)(ux * (float)im->w), 0), im->w - 1), py = std::min(std::max((int)(uy * (float)im->h), 0), im->h - 1);
        V2 uv = {((float)px + 0.5f) / (float)im->w, ((float)py + 0.5f) / (float)im->h};
        /* read_rgba < 0: masked texel (common_device.cuh:803-835) */
        int tx = std::min(std::max((int)(uv.x * (float)im->w), 0), im->w - 1), ty = std::min(std::max((int)(uv.y * (float)im->h), 0), im->h - 1);
        const uint8_t* tex = im->rgba + (((size_t)img * im->h + ty) * im->w + tx) * 4;
        if (tex[0] == 0xFF && tex[1] == 0x00 && tex[2] == 0xFF && tex[3] == 0x00) continue;
        (void)rng.next_float();   /* motionblur_time */
        /* get_xform_given_rolling_shutter (common_device.cuh:361-368), then uv_to_ray with the image's lens (403-470);
         * an invalid ray is {xform[3], xform[2]} (testbed_nerf.cu:901-903) */
        const float* xf = im->xforms + 12 * (size_t)img;
        const M43 cam = m43_load(xf);
        const M3 rot = rolling_shutter_rotation(m3_of(cam));
        const float* fo = im->focal + 2 * (size_t)img;
        const float* pp = im->pp + 2 * (size_t)img;
        const OrcLens lens = img < g_train_lens.size() ? g_train_lens[img] : OrcLens{};
        V3 dir;
        if (uv_to_ray_dir(lens, uv, im->w, im->h, V2{fo[0], fo[1]}, V2{pp[0], pp[1]}, &dir)) dir = mul(rot, dir);
        else dir = rot.c[2];
        const V3 o = cam.c[3];
        const V3 dn = normalize(dir);
        V2 tminmax = bb_ray_intersect(aabb, o, dn);
        const float cone = vol.cone;   /* calc_cone_angle returns the constant (nerf_device.cuh:370-377) */
        tminmax.x = std::fmax(tminmax.x, 0.0f);
        const float startt = advance_n_steps(tminmax.x, cone, rng.next_float());
        const V3 idir = v3(1.0f / dn.x, 1.0f / dn.y, 1.0f / dn.z);
        uint32_t j = 0;
        float t = startt;
        V3 pos;
        float* co = coords + (size_t)i * max_per_ray * 7;
        const V3 wd = warp_direction(dn);
        while (bb_contains(aabb, pos = o + t * dn) && j < NERF_STEPS) {
            const float dt = calc_dt(t, cone);
            const uint32_t mip = mip_from_dt(dt, pos, vol.max_mip);
            if (density_grid_occupied_at(pos, vol.bitfield, mip)) {
                if (j < max_per_ray) {
                    const V3 wp = warp_position(pos, aabb);
                    float* c = co + (size_t)j * 7;
                    c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(dt); c[4] = wd.x; c[5] = wd.y; c[6] = wd.z;
                }
                ++j;
                t += dt;
            } else {
                t = advance_to_next_voxel(t, cone, pos, dn, idir, mip);
            }
        }
        numsteps[i] = j;
        float* r = rays + 6 * (size_t)i;
        r[0] = o.x; r[1] = o.y; r[2] = o.z; r[3] = dir.x; r[4] = dir.y; r[5] = dir.z;
    }
}

void orc_train_adam_ema(uint64_t n, uint32_t n_matrix, float lr, float beta1, float beta2, float eps, float l2_reg, float loss_scale,
                        float ema_decay, uint32_t ema_step, float* master, const float* grads, float* m1, float* m2, uint32_t* steps,
                        float* ema) {
    const float deb_old = 1.0f - std::pow(ema_decay, (float)ema_step), deb_new = 1.0f - std::pow(ema_decay, (float)(ema_step + 1));
    for (uint64_t i = 0; i < n; ++i) {
        /* tcnn adam_step (optimizers/adam.h) [unvendored] */
        float gradient = grads[i] / loss_scale;
        if (i < n_matrix || gradient != 0.0f) {
            const float w = master[i];
            if (i < n_matrix) gradient += l2_reg * w;
            const float gsq = gradient * gradient;
            const float fm = m1[i] = beta1 * m1[i] + (1.0f - beta1) * gradient;
            const float sm = m2[i] = beta2 * m2[i] + (1.0f - beta2) * gsq;
            const uint32_t step = ++steps[i];
            float l = lr;
            l *= std::sqrt(1.0f - std::pow(beta2, (float)step)) / (1.0f - std::pow(beta1, (float)step));
            const float eff = l / (std::sqrt(sm) + eps);
            master[i] = w - eff * fm;
        }
        /* tcnn EmaOptimizer (optimizers/average.h): debiased exponential moving average of the weights */
        ema[i] = (ema[i] * ema_decay * deb_old + master[i] * (1.0f - ema_decay)) / deb_new;
    }
}
}  // extern "C"

/* ---- scene animation ---------------------------------------------------------- */
namespace {
struct OrcCam { V3 c[4]; float scale; V3 up; };
inline V3 orc_look_at(const OrcCam& k) { return k.c[3] + k.c[2] * k.scale; }                       /* testbed.cu:405-407 */
inline void orc_set_look_at(OrcCam& k, V3 pos) { k.c[3] = k.c[3] + (pos - orc_look_at(k)); }     /* testbed.cu:409-411 */
inline void orc_set_scale(OrcCam& k, float scale) {                                               /* testbed.cu:413-417 */
    V3 prev = orc_look_at(k);
    k.c[3] = (k.c[3] - prev) * (scale / k.scale) + prev;
    k.scale = scale;
}
inline void orc_set_view_dir(OrcCam& k, V3 dir) {                                                 /* testbed.cu:419-425 */
    V3 old = orc_look_at(k);
    k.c[0] = normalize(cross(dir, k.up));
    k.c[1] = normalize(cross(dir, k.c[0]));
    k.c[2] = normalize(dir);
    orc_set_look_at(k, old);
}
}  // namespace

extern "C" {
void orc_camera_set_view(float cam[12], float* scale, const float up[3], const float view[3], const float at[3], float zoom) {
    OrcCam k;
    for (int i = 0; i < 4; ++i) k.c[i] = v3(cam[3 * i], cam[3 * i + 1], cam[3 * i + 2]);
    k.scale = *scale;
    k.up = v3(up[0], up[1], up[2]);
    orc_set_view_dir(k, v3(view[0], view[1], view[2]));
    orc_set_look_at(k, v3(at[0], at[1], at[2]));
    orc_set_scale(k, zoom);
    for (int i = 0; i < 4; ++i) { cam[3 * i] = k.c[i].x; cam[3 * i + 1] = k.c[i].y; cam[3 * i + 2] = k.c[i].z; }
    *scale = k.scale;
}
void orc_animation_play(float cam[12], float* scale, const float up[3], const orc_keyframe* keys, uint32_t n_keys, int32_t total_frames,
                        int32_t playing, float anim_speed, orc_light_anim* lights, uint32_t n_lights, orc_object_anim* objs, uint32_t n_objs,
                        uint32_t n_frames, float* cams_out, float* light_pos_out, float* obj_pos_out) {
    OrcCam k;
    for (int i = 0; i < 4; ++i) k.c[i] = v3(cam[3 * i], cam[3 * i + 1], cam[3 * i + 2]);
    k.scale = *scale;
    k.up = v3(up[0], up[1], up[2]);
    /* CamPath(config) (cam_path.cuh:97-115): frames_between_keyframes = total_frames / max(n - 1, 1) */
    int frames_between = total_frames / std::max((int)n_keys - 1, 1);
    if (frames_between < 1) frames_between = 1;
    int current_frame = 0;
    const bool enable = anim_speed > 0.0f;   /* m_enable_animations (engine.cu:43-46) */
    for (uint32_t f = 0; f < n_frames; ++f) {
        /* CamPath::update -> advance_frame -> set_to_frame (cam_path.cuh:117-135) */
        if (playing && n_keys >= 2) {
            current_frame += 1;
            int current_keyframe = current_frame / frames_between;
            uint32_t next = (uint32_t)current_keyframe + 1;
            if (next >= n_keys) { current_frame = 0; current_keyframe = 0; next = 1; }
            const orc_keyframe& a = keys[current_keyframe];
            const orc_keyframe& b = keys[next];
            /* CamKeyframe::interpolate (cam_path.cuh:30-39) */
            float t = (float)(current_frame % frames_between) / (float)frames_between;
            float invk = (float)(1.0 - (double)t);
            V3 view = invk * v3(a.view[0], a.view[1], a.view[2]) + t * v3(b.view[0], b.view[1], b.view[2]);
            orc_set_view_dir(k, view);
            V3 at = invk * v3(a.at[0], a.at[1], a.at[2]) + t * v3(b.at[0], b.at[1], b.at[2]);
            orc_set_look_at(k, at);
            orc_set_scale(k, invk * a.zoom + t * b.zoom);
        }
        if (enable) {
            /* update_world_objects (engine.cu:87-98): VirtualObject::next_frame (virtual_object.cuh:53-64) */
            for (uint32_t i = 0; i < n_objs; ++i) {
                orc_object_anim& o = objs[i];
                if (o.angle == 0.0f) continue;
                const V3 ax = v3(o.axis[0], o.axis[1], o.axis[2]);
                const float cost = std::cos(o.angle * anim_speed);
                const float sint = std::sin(o.angle * anim_speed);
                /* tcnn mat3 from 9 scalars: column-major, written as in the reference (3rd column uses ax.z*ax.y) */
                const float m[9] = {cost + ax.x * ax.x * (1.0f - cost), ax.x * ax.y * (1.0f - cost) - ax.z * sint, ax.x * ax.z * (1.0f - cost) + ax.y * sint,
                                    ax.x * ax.y * (1.0f - cost) + ax.z * sint, cost + ax.y * ax.y * (1.0f - cost), ax.y * ax.z * (1.0f - cost) - ax.x * sint,
                                    ax.z * ax.y * (1.0f - cost) - ax.y * sint, ax.z * ax.y * (1.0f - cost) + ax.x * sint, cost + ax.z * ax.z * (1.0f - cost)};
                const M3 next = m3_load(m);
                const M3 rot = m3_load(o.rot);
                V3 p = v3(o.pos[0], o.pos[1], o.pos[2]);
                const V3 centre = v3(o.centre[0], o.centre[1], o.centre[2]);
                p = mul(next, mul(rot, p - centre)) + centre;
                o.pos[0] = p.x; o.pos[1] = p.y; o.pos[2] = p.z;
            }
            /* Light::next_frame (light.cuh:39-49) */
            for (uint32_t i = 0; i < n_lights; ++i) {
                orc_light_anim& l = lights[i];
                if (!l.on || l.step == 0.0f) continue;
                float nr = l.ratio + l.step;
                if (nr > 1.0 || nr < 0.0) { l.step = -l.step; nr = l.ratio + l.step; }
                l.ratio = nr;
            }
        }
        for (int i = 0; i < 4; ++i) { cams_out[12 * f + 3 * i] = k.c[i].x; cams_out[12 * f + 3 * i + 1] = k.c[i].y; cams_out[12 * f + 3 * i + 2] = k.c[i].z; }
        for (uint32_t i = 0; i < n_lights; ++i) {
            const orc_light_anim& l = lights[i];
            float* q = light_pos_out + 3 * ((size_t)f * n_lights + i);
            if (l.on) {
                const V3 p = (1.0f - l.ratio) * v3(l.start[0], l.start[1], l.start[2]) + l.ratio * v3(l.end[0], l.end[1], l.end[2]);
                q[0] = p.x; q[1] = p.y; q[2] = p.z;
            } else {
                q[0] = l.start[0]; q[1] = l.start[1]; q[2] = l.start[2];
            }
        }
        for (uint32_t i = 0; i < n_objs; ++i)
            for (int d = 0; d < 3; ++d) obj_pos_out[3 * ((size_t)f * n_objs + i) + d] = objs[i].pos[d];
    }
    for (int i = 0; i < 4; ++i) { cam[3 * i] = k.c[i].x; cam[3 * i + 1] = k.c[i].y; cam[3 * i + 2] = k.c[i].z; }
    *scale = k.scale;
}
}  // extern "C"

/* ---- display stage (main.frag) ------------------------------------------------------ */
namespace {
struct Tex4 { float r, g, b, a; };
/* texture(sampler2D, uv) with GL_LINEAR + GL_REPEAT; textureProjOffset adds the texel offset in texel space */
Tex4 gl_texture(const float* img, int W, int H, float u, float v, int ox = 0, int oy = 0) {
    const float x = u * (float)W - 0.5f + (float)ox, y = v * (float)H - 0.5f + (float)oy;
    const float fx0 = std::floor(x), fy0 = std::floor(y);
    const float ax = x - fx0, ay = y - fy0;
    int x0 = (int)fx0 % W, y0 = (int)fy0 % H;
    if (x0 < 0) x0 += W;
    if (y0 < 0) y0 += H;
    const int x1 = x0 + 1 == W ? 0 : x0 + 1, y1 = y0 + 1 == H ? 0 : y0 + 1;
    const float* a = img + 4 * ((size_t)y0 * W + x0);
    const float* b = img + 4 * ((size_t)y0 * W + x1);
    const float* c = img + 4 * ((size_t)y1 * W + x0);
    const float* d = img + 4 * ((size_t)y1 * W + x1);
    const float w00 = (1.0f - ax) * (1.0f - ay), w10 = ax * (1.0f - ay), w01 = (1.0f - ax) * ay, w11 = ax * ay;
    float o[4];
    for (int k = 0; k < 4; ++k) o[k] = a[k] * w00 + b[k] * w10 + c[k] * w01 + d[k] * w11;
    return {o[0], o[1], o[2], o[3]};
}
inline float gl_luma(float r, float g, float b) { return r * 0.299f + g * 0.587f + b * 0.114f; }   /* dot(rgb, vec3(0.299, 0.587, 0.114)) */
}  // namespace

extern "C" void orc_display(const float* rgba, int32_t W, int32_t H, int32_t OW, int32_t OH, const float clear[3], uint8_t* out) {
#pragma omp parallel for schedule(static)
    for (int row = 0; row < OH; ++row)
        for (int x = 0; x < OW; ++x) {
            /* main(): tex_coords = UVs, y flipped, unwarp = identity without foveation */
            const int ygl = OH - 1 - row;
            const float u = ((float)x + 0.5f) / (float)OW;
            const float v = 1.0f - ((float)ygl + 0.5f) / (float)OH;
            /* fxaa(tex, fragCoord, resolution) */
            const float ivx = 1.0f / (float)OW, ivy = 1.0f / (float)OH;
            const Tex4 nw = gl_texture(rgba, W, H, u, v, -1, 1), ne = gl_texture(rgba, W, H, u, v, 1, 1);
            const Tex4 sw = gl_texture(rgba, W, H, u, v, -1, -1), se = gl_texture(rgba, W, H, u, v, 1, -1);
            const Tex4 tc = gl_texture(rgba, W, H, u, v);
            const float lNW = gl_luma(nw.r, nw.g, nw.b), lNE = gl_luma(ne.r, ne.g, ne.b), lSW = gl_luma(sw.r, sw.g, sw.b), lSE = gl_luma(se.r, se.g, se.b);
            const float lM = gl_luma(tc.r, tc.g, tc.b);
            const float lmin = std::fmin(lM, std::fmin(std::fmin(lNW, lNE), std::fmin(lSW, lSE)));
            const float lmax = std::fmax(lM, std::fmax(std::fmax(lNW, lNE), std::fmax(lSW, lSE)));
            float dx = -((lNW + lNE) - (lSW + lSE));
            float dy = ((lNW + lSW) - (lNE + lSE));
            const float reduce = std::fmax((lNW + lNE + lSW + lSE) * (0.25f * (1.0f / 8.0f)), 1.0f / 128.0f);   /* FXAA_REDUCE_MUL / _MIN */
            const float rcp_min = 1.0f / (std::fmin(std::fabs(dx), std::fabs(dy)) + reduce);
            dx = std::fmin(8.0f, std::fmax(-8.0f, dx * rcp_min)) * ivx;   /* FXAA_SPAN_MAX */
            dy = std::fmin(8.0f, std::fmax(-8.0f, dy * rcp_min)) * ivy;
            const float k1 = 1.0f / 3.0f - 0.5f, k2 = 2.0f / 3.0f - 0.5f;
            const Tex4 a1 = gl_texture(rgba, W, H, u + dx * k1, v + dy * k1), a2 = gl_texture(rgba, W, H, u + dx * k2, v + dy * k2);
            const float A[3] = {0.5f * (a1.r + a2.r), 0.5f * (a1.g + a2.g), 0.5f * (a1.b + a2.b)};
            const Tex4 b1 = gl_texture(rgba, W, H, u + dx * -0.5f, v + dy * -0.5f), b2 = gl_texture(rgba, W, H, u + dx * 0.5f, v + dy * 0.5f);
            const float B[3] = {A[0] * 0.5f + 0.25f * (b1.r + b2.r), A[1] * 0.5f + 0.25f * (b1.g + b2.g), A[2] * 0.5f + 0.25f * (b1.b + b2.b)};
            const float lB = gl_luma(B[0], B[1], B[2]);
            const float* C = (lB < lmin || lB > lmax) ? A : B;
            const float ia = 1.0f - tc.a;
            uint8_t* o = out + 3 * ((size_t)row * OW + x);
            for (int k = 0; k < 3; ++k) {
                float f = C[k] + clear[k] * ia;
                f = std::fmin(std::fmax(f, 0.0f), 1.0f);
                o[k] = (uint8_t)(int)(f * 255.0f + 0.5f);
            }
        }
}

extern "C" void orc_wavefront_schedule(const uint32_t* n_alive, uint32_t n, uint32_t target, uint32_t* n_steps, uint64_t* n_elements) {
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t a = n_alive[i];
        n_steps[i] = a ? wavefront_steps(a, target ? target : 2u * 1024u * 1024u) : 0u;
        n_elements[i] = a ? wavefront_elements(a, n_steps[i]) : 0u;
    }
}

extern "C" void orc_set_literal(int32_t on) { g_literal = on ? 1 : 0; }
