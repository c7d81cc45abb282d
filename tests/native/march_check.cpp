// Host-side checks of the product's exact fast paths (synerfgine_amd/csrc/sng_math.h), compiled
// by tests/test_host_fastpaths.py with hipcc as plain host code (no GPU needed):
//   1. div_by(x, d, RN(1/d)) == x / d bit for bit (random pairs + a sweep of t / MIN_STEP);
//   2. advance_to_occupied_linear == the general advance_to_occupied (nerf_device.cuh:462-495) on
//      cone == 0, max_mip == 0 volumes for random rays through a random occupancy grid;
//   3. aabb_entry_fast == aabb_entry for random boxes and rays, and for degenerate boxes / on-plane origins.
#include "sng_math.h"
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
using namespace sng;
static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static bool same(float a, float b) { return bits(a) == bits(b) || (a != a && b != b); }

int main() {
    std::mt19937 g(7);
    long bad_div = 0, n_div = 0;
    {
        std::uniform_real_distribution<float> E(-30.f, 30.f), S(0.f, 1.f);
        for (int i = 0; i < 4000000; ++i) {
            float x = std::ldexp(S(g) + 0.5f, (int)E(g)) * (g() & 1 ? 1.f : -1.f);
            float d = std::ldexp(S(g) + 0.5f, (int)E(g)) * (g() & 1 ? 1.f : -1.f);
            volatile float y = 1.0f / d;
            ++n_div;
            if (!same(div_by(x, d, y), x / d)) ++bad_div;
        }
        float t = 1e-6f;
        for (int i = 0; i < 4000000; ++i, t = std::nextafter(t, 1e9f) * 1.0000037f) {
            ++n_div;
            if (!same(div_by(t, MIN_STEP, INV_MIN_STEP), t / MIN_STEP)) ++bad_div;
        }
    }
    // occupancy grid (Morton bitfield + its linear copy)
    std::vector<uint8_t> bf(GRID_CELLS / 8 * N_CASCADES, 0);
    for (uint32_t z = 0; z < 128; ++z)
        for (uint32_t y = 0; y < 128; ++y)
            for (uint32_t x = 0; x < 128; ++x) {
                float dx = x - 64.f, dy = y - 60.f, dz = z - 70.f;
                bool occ = (dx * dx + dy * dy + dz * dz < 1600.f && ((x / 4 + y / 4 + z / 4) % 3 == 0)) || (g() % 1000 == 0);
                if (occ) { uint32_t m = morton3D(x, y, z); bf[m >> 3] |= 1u << (m & 7); }
            }
    std::vector<uint32_t> occ(GRID_CELLS / 32, 0);
    for (uint32_t w = 0; w < GRID_CELLS / 32; ++w) {
        uint32_t z = w / (128 * 4), y = (w / 4) % 128, x0 = (w % 4) * 32, b = 0;
        for (uint32_t k = 0; k < 32; ++k) { uint32_t m = morton3D(x0 + k, y, z); b |= (uint32_t)((bf[m >> 3] >> (m & 7)) & 1) << k; }
        occ[w] = b;
    }
    Volume v{};
    v.render_aabb = {splat(0.f), splat(1.f)};
    v.train_aabb = v.render_aabb;
    v.to_local = {mk(1, 0, 0), mk(0, 1, 0), mk(0, 0, 1)};
    v.to_local_identity = 1;
    v.bitfield = bf.data();
    v.occ_linear = occ.data();
    std::uniform_real_distribution<float> U(-1, 1), U01(0, 1);
    long bad_march = 0, n_march = 0, n_samples = 0;
    for (int it = 0; it < 200000; ++it) {
        f3 o = (it % 3 == 0) ? mk(U01(g), U01(g), U01(g)) : mk(U(g) * 2.f + 0.5f, U(g) * 2.f + 0.5f, U(g) * 2.f + 0.5f);
        f3 d = normalize(mk(U(g), U(g), U(g)));
        if (it % 17 == 0) d.x = 0.f;
        if (it % 19 == 0) d = normalize(mk(0.f, 0.f, U(g)));
        const f3 idir = inv(d);
        float t0 = fmaxf(aabb_entry(v.render_aabb, o, d), 0.0f) + 1e-6f;
        float ta = t0, tb = t0;
        for (int s = 0; s < 12; ++s) {
            v.linear = 0;
            ta = advance_to_occupied(ta, 0.f, o, d, idir, 0, 0, v);
            tb = advance_to_occupied_linear(tb, o, d, idir, half_sign(d), v);
            ++n_march;
            if (!same(ta, tb)) { ++bad_march; break; }
            if (ta >= MAX_DEPTH) break;
            ++n_samples;
            const float dt = calc_dt(ta, 0.f);
            ta += dt; tb += dt;
        }
    }
    long bad_slab = 0, n_slab = 0;
    for (int it = 0; it < 2000000; ++it) {
        f3 a = mk(U(g), U(g), U(g)), b = mk(U(g), U(g), U(g));
        aabb box = {mk(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)), mk(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z))};
        f3 o = mk(U(g) * 3.f, U(g) * 3.f, U(g) * 3.f);
        f3 d = normalize(mk(U(g), U(g), U(g)));
        if (it % 7 == 0) d = d * 37.5f;
        if (!slab_fast_ok(o, d)) continue;
        ++n_slab;
        // bvh_box_entry's branch-free form equals the branchy one up to the sign of a zero result (callers only compare it)
        const float fa = aabb_entry_fast(box, o, inv(d)), fb = bvh_box_entry(box, o, inv(d));
        if (!(same(fa, fb) || (fa == 0.0f && fb == 0.0f))) ++bad_slab;
    }
    // degenerate slabs and origins on a slab plane: the equal-value cases of the swaps and early-outs
    for (int it = 0; it < 2000000; ++it) {
        const float q[5] = {-0.5f, 0.0f, 0.25f, 0.5f, 1.0f};
        f3 lo = mk(q[g() % 5], q[g() % 5], q[g() % 5]), hi = lo;
        if (g() & 1) hi.x = fmaxf(hi.x, q[g() % 5]);
        if (g() & 1) hi.y = fmaxf(hi.y, q[g() % 5]);
        if (g() & 1) hi.z = fmaxf(hi.z, q[g() % 5]);
        aabb box = {lo, hi};
        f3 o = mk(q[g() % 5], q[g() % 5], q[g() % 5]);
        if (g() & 1) o.x += U(g);
        f3 d = mk(q[g() % 5] + 0.125f * (float)(g() % 3), q[g() % 5] - 0.0625f, q[g() % 5] + 0.375f);
        if (d.x == 0.0f || d.y == 0.0f || d.z == 0.0f || !slab_fast_ok(o, d)) continue;
        ++n_slab;
        const float fa = aabb_entry_fast(box, o, inv(d)), fb = bvh_box_entry(box, o, inv(d));
        if (!(same(fa, fb) || (fa == 0.0f && fb == 0.0f))) ++bad_slab;
    }
    // sng_logf's f / (2 + f) as div_by(f, d, RN(1/d)): every f it can form (m in [0.5, 1), doubled below
    // 0.7071, f = m - 1), i.e. all 2^23 mantissas.  recip_rn is 1.0f / d on the host and bit-identical to
    // it on the device (tools/rcp_check.hip), so this covers the device form too.
    long bad_log = 0, n_log = 0;
    for (uint32_t u = 0x3F000000u; u < 0x3F800000u; ++u) {
        float m;
        std::memcpy(&m, &u, 4);
        if (m < 0.707106769f) m = m * 2.0f;
        const float f = m - 1.0f, den = 2.0f + f;
        ++n_log;
        if (!same(div_by(f, den, recip_rn(den)), f / den)) ++bad_log;
    }
    // to_stepping_space's log branch: sng_logf(t) / log1p_c as div_by with RN(1 / log1p_c), for every t in
    // (at, bt] (strided by 7 ulps) at five cone angles.  Its quotients are IEEE whenever |sng_logf(t)| >= 2^-105
    // (below that the FMA remainder underflows); t != 1 gives |log t| >= 2^-25 and t == 1 gives 0 exactly.
    long bad_step = 0, n_step = 0;
    const float cones[5] = {1.0f / 1024.0f, 1.0f / 256.0f, 1.0f / 128.0f, 0.01f, 0.05f};
    for (float cone : cones) {
        const StepSpace k = step_space(cone);
        uint32_t u0, u1;
        std::memcpy(&u0, &k.at, 4);
        std::memcpy(&u1, &k.bt, 4);
        for (uint32_t u = u0 + 1; u <= u1; u += 7) {
            float t;
            std::memcpy(&t, &u, 4);
            ++n_step;
            const float x = sng_logf(t);
            if (!same(div_by(x, k.log1p_c, k.rlog1p_c), x / k.log1p_c) || !same(to_stepping_space(t, k), x / k.log1p_c)) ++bad_step;
        }
    }
    std::printf("{\"div\": [%ld, %ld], \"march\": [%ld, %ld, %ld], \"slab\": [%ld, %ld], \"logdiv\": [%ld, %ld], \"stepdiv\": [%ld, %ld]}\n", n_div,
                bad_div, n_march, n_samples, bad_march, n_slab, bad_slab, n_log, bad_log, n_step, bad_step);
    return (bad_div || bad_march || bad_slab || bad_log || bad_step) ? 1 : 0;
}
