// fused.hip -- ray-local NeRF wavefront: generate + field (hash grid + MLPs on MFMA) + composite
// in ONE persistent kernel.
//
// Why this is exact: trace_alt / trace pick n_steps = clamp(2^21 / n_alive, 1, 8) per iteration
// from the frame-wide alive count (testbed_nerf.cu:2189-2190).  Once n_alive * 8 <= 2^21 the
// count only shrinks, so every later iteration takes exactly 8 steps and a ray's samples, t
// resets, termination and MARCH_ITER cut-off depend on nothing but the ray itself (its k-th
// iteration has i = i0 + 8k).  From that point each wave can own 64 rays and advance each one
// through its iterations independently -- no grid-wide launch per iteration, no waiting for the
// frame's slowest ray, no sample buffers in HBM.  Per wave iteration:
//   generate : every lane marches up to 8 samples (flattened DDA loop), t's to LDS;
//   field    : the wave compacts its samples (wave scan) and evaluates them 16 at a time with
//              the same field_tile() as nerf_network_kernel, recomputing each sample's NerfCoordinate
//              with generate_kernel's float expressions, so outputs are bit-identical;
//   composite: every lane composites its samples exactly as composite_kernel, then either keeps
//              the ray, or retires it (extract_from_payload / shade_kernel_nerf) and refills the
//              lane from the ray queue.
// Statistics (alive / samples per iteration, hits) are gathered in LDS and flushed per block.
#include <algorithm>

#include "nerf_field.h"

namespace sng {

constexpr int FUSED_WAVES = 4;   // waves per workgroup

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_incl_scan_u(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t o = __shfl_up(v, off, 64);
        if (lane >= off) v += o;
    }
    return v;
}

template <int F, bool LIN>
__global__ __launch_bounds__(256) void nerf_fused_kernel(FusedArgs a) {
    __shared__ float ts_lds[FUSED_WAVES][MAX_STEPS_BETWEEN_COMPACTION][64];
    __shared__ float4 ray_lds[FUSED_WAVES][64][2];   // origin, dir of each lane's ray
    __shared__ uint16_t own_lds[FUSED_WAVES][64 * MAX_STEPS_BETWEEN_COMPACTION];
    __shared__ uint2 out_lds[FUSED_WAVES][64 * MAX_STEPS_BETWEEN_COMPACTION];
    __shared__ uint32_t hist_alive[64], hist_samples[64];
    __shared__ uint32_t blk_hit, blk_iter;
    __shared__ unsigned long long blk_samples, blk_reused;

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int g = lane >> 4, col = lane & 15;
    if (threadIdx.x < 64) { hist_alive[threadIdx.x] = 0; hist_samples[threadIdx.x] = 0; }
    if (threadIdx.x == 0) { blk_hit = 0; blk_iter = 0; blk_samples = 0; blk_reused = 0; }
    __syncthreads();

    const Volume& vol = a.vol;
    const CamDev& cam = a.cam;
    // continue where the per-iteration wavefront stopped: its alive buffer, step counter i and
    // iteration count (all 0-based iteration statistics continue at k0)
    const uint32_t n_rays = a.ctrl->n_alive[a.p];
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ctrl->fused_rays_in = n_rays;   // (host_render.cpp spec_adapt)
    // nothing left (the speculative rounds finished every ray), or not a tail after all (tail_prepare's check):
    // leave before the weight fragments are loaded
    if (n_rays == 0 || !a.ctrl->spec_ok) return;
    const uint32_t i_step0 = a.ctrl->i_step[a.p];
    const uint32_t k0 = a.ctrl->n_iter;
    // after speculative rounds each ray carries its own next iteration (RayBuf::kk)
    const bool kk_in = a.ctrl->spec_kk_valid[a.p] != 0u;
    const uint32_t base_k = a.ctrl->spec_base_k, base_istep = a.ctrl->spec_base_istep;
    const f3 wdiag = vol.train_aabb.hi - vol.train_aabb.lo;
    const StepSpace cone = LIN ? step_space(0.0f) : vol.ss;
    const h8* wfrag = reinterpret_cast<const h8*>(a.wfrag);
    const _Float16* grid = reinterpret_cast<const _Float16*>(a.grid_params);
    h8 W[20];
#pragma unroll
    for (int f = 0; f < 20; ++f) W[f] = wfrag[f * 64 + lane];

    bool has = false;
    f3 o = splat(0.0f), d = splat(1.0f);
    float t = 0.0f, depth = 0.0f, mw = 0.0f;
    float4 rgba = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    uint32_t idx = 0, k = 0, istep = 0;
    uint32_t my_hits = 0, my_iter = 0;
    bool loaded = false, left = false;   // the lane took a ray from the queue / retired its ray this trip
    unsigned long long my_samples = 0, my_reused = 0;
    // trace_alt boundary-sample cache (RayBuf::lt/lo): the previous iteration's last sample t and output
    float lt = 0.0f;
    uint2 lo = make_uint2(0u, 0u);

    while (true) {
        // ---- refill empty lanes from the ray queue (one atomic per wave)
        {
            const unsigned long long need = __ballot(!has && (uint32_t)lane < a.lanes);
            if (need) {
                const int leader = __ffsll((long long)need) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(a.work, (uint32_t)__popcll(need));
                base = __shfl(base, leader, 64);
                if (!has) {
                    const uint32_t r = base + (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
                    if (r < n_rays) {
                        const float4 ot = a.rays.o_t[r], di = a.rays.d_idx[r];
                        o = mk(ot.x, ot.y, ot.z);
                        t = ot.w;
                        d = mk(di.x, di.y, di.z);
                        idx = __float_as_uint(di.w);
                        rgba = a.rays.rgba[r];
                        depth = a.rays.depth[r];
                        mw = a.mode.ngp ? a.rays.mw[r] : 0.0f;
                        if (!a.mode.ngp) { lt = a.rays.lt[r].x; lo = a.rays.lo[r]; }
                        k = kk_in ? a.rays.kk[r] : k0;
                        loaded = true;
                        istep = kk_in ? base_istep + MAX_STEPS_BETWEEN_COMPACTION * (k - base_k) : i_step0;
                        has = true;
                    }
                }
            }
        }
        wave_add_keyed(a.ctrl->tail_live, k, 1, loaded);   // alive from its first tail iteration on (reference slots)
        loaded = false;
        if (!__ballot(has)) break;

        // ---- generate: up to 8 samples (generate_next_nerf_network_inputs, testbed_nerf.cu:790-837)
        uint32_t cnt = 0;
        bool reuse = false;
        const uint32_t n_steps = MAX_STEPS_BETWEEN_COMPACTION;
        if (has) {
            const f3 idir = inv(d);
            if constexpr (LIN) {
                const f3 hs = half_sign(d);
                OccCache oc;
                while (cnt < n_steps) {
                    const f3 pos = o + d * t;
                    if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) break;
                    if (occupied_linear_c(pos, vol.occ_linear, oc)) {
                        if (cnt == 0 && !a.mode.ngp && t == lt) reuse = true;
                        ts_lds[wv][cnt][lane] = t;
                        t += calc_dt(t, 0.0f);
                        ++cnt;
                    } else {
                        t = dda_step_linear(t, pos, idir, hs);
                    }
                }
            } else {
#pragma unroll 1
                while (cnt < n_steps) {   // flattened occ_step trips (generate_kernel)
                    if (occ_step(t, cone, o, d, idir, 0, vol.max_mip, vol)) {
                        if (t >= MAX_DEPTH) break;
                        ts_lds[wv][cnt][lane] = t;
                        t += calc_dt(t, cone);
                        ++cnt;
                    }
                }
                reuse = cnt > 0 && !a.mode.ngp && ts_lds[wv][0][lane] == lt;
            }
            ray_lds[wv][lane][0] = make_float4(o.x, o.y, o.z, 0.0f);
            ray_lds[wv][lane][1] = make_float4(d.x, d.y, d.z, 0.0f);
            if (k < 64) atomicAdd(&hist_alive[k], 1u);
            if (istep >= MARCH_ITER) cnt = 0;   // unreachable: `last` retires rays first
        }
        // the network evaluates only the samples not taken from the boundary cache
        const uint32_t ru = reuse ? 1u : 0u;
        const uint32_t ncnt = cnt - ru;
        const uint32_t incl = wave_incl_scan_u(ncnt, lane);
        const uint32_t total = __shfl(incl, 63, 64);
        const uint32_t sbase = incl - ncnt;
        for (uint32_t j = ru; j < cnt; ++j) own_lds[wv][sbase + j - ru] = (uint16_t)((lane << 3) | j);
        if (has && k < 64 && cnt) atomicAdd(&hist_samples[k], cnt);
        my_samples += cnt;
        my_reused += ru;
        wave_sync();

        // ---- field on the wave's samples, 16 per tile
        for (uint32_t tile = 0; tile * 16 < total; ++tile) {
            const uint32_t q = tile * 16 + (uint32_t)col;
            const bool valid = q < total;
            const uint32_t ow = own_lds[wv][valid ? q : 0];
            const uint32_t ol = ow >> 3, oj = ow & 7u;
            const float4 ro = ray_lds[wv][ol][0], rd = ray_lds[wv][ol][1];
            const float ts = ts_lds[wv][oj][ol];
            const f3 so = mk(ro.x, ro.y, ro.z), sd = mk(rd.x, rd.y, rd.z);
            const f3 wp = ((so + sd * ts) - vol.train_aabb.lo) / wdiag;   // generate_kernel's expressions
            const f3 wd = (sd + 1.0f) * 0.5f;
            f4v out, dens;
            field_tile<F, true>(W, a.levels, grid, g, wp.x, wp.y, wp.z, wd.x, wd.y, wd.z, out, dens);
            if (valid && g == 0) {
                const _Float16 r = (_Float16)out[0], gg = (_Float16)out[1], b = (_Float16)out[2], s = (_Float16)dens[0];
                out_lds[wv][q] = make_uint2((uint32_t)__builtin_bit_cast(uint16_t, r) | ((uint32_t)__builtin_bit_cast(uint16_t, gg) << 16),
                                            (uint32_t)__builtin_bit_cast(uint16_t, b) | ((uint32_t)__builtin_bit_cast(uint16_t, s) << 16));
            }
        }
        wave_sync();

        // ---- composite (composite_kernel_nerf_alt 476-575 / composite_kernel_nerf 577-788)
        if (has) {
            const bool last = istep + n_steps >= MARCH_ITER;
            uint32_t j = 0;
            uint2 last_raw = lo;
            for (; j < cnt; ++j) {
                const uint2 raw = (reuse && j == 0) ? lo : out_lds[wv][sbase + j - ru];
                last_raw = raw;
                const float ts = ts_lds[wv][j][lane];
                const f3 wp = ((o + d * ts) - vol.train_aabb.lo) / wdiag;
                const float cdt = warp_dt(calc_dt(ts, cone));
                const f3 pos = vol.train_aabb.lo + wp * wdiag;
                const float T = 1.f - rgba.w;
                const float dt = unwarp_dt(cdt);
                const float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x & 0xffffu));
                const float gg = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x >> 16));
                const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y & 0xffffu));
                const float s = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y >> 16));
                const float alpha = 1.f - sng_expf(-sng_expf(s) * dt);
                const float weight = alpha * T;
                f3 rgb = mk(logistic(r), logistic(gg), logistic(b));
                if (a.mode.ngp) {
                    if (a.mode.render_mode == 3) rgb = (pos - 0.5f) / 2.0f + 0.5f;
                    else if (a.mode.render_mode == 10) rgb = wp;
                    else if (a.mode.render_mode == 4) rgb = splat(dot(cam.c2, pos - o) * a.mode.depth_scale);
                    else if (a.mode.render_mode == 0) rgb = splat(alpha);
                }
                rgba.x += rgb.x * weight;
                rgba.y += rgb.y * weight;
                rgba.z += rgb.z * weight;
                rgba.w += weight;
                if (a.mode.ngp) {
                    if (weight > mw) { mw = weight; depth = dot(cam.c2, pos - cam.c3); }
                } else {
                    depth = dot(cam.c2, pos - cam.c3);
                }
                if (rgba.w > (1.0f - vol.min_transmittance)) {
                    const float aa = rgba.w;
                    rgba.x /= aa; rgba.y /= aa; rgba.z /= aa; rgba.w /= aa;
                    break;
                }
            }
            // trace_alt resets t to the last sample (574); trace keeps generate's t (836) -- in
            // the flattened march t already is generate's end value when all 8 steps were taken
            if (!a.mode.ngp) {
                t = depth / dot(cam.c2, d);
                if (cnt) { lt = ts_lds[wv][cnt - 1][lane]; lo = last_raw; }   // survivors composited all cnt samples
            }
            bool hit = false;
            if (j < n_steps) {
                hit = !last && rgba.w > 0.001f;
                has = false;
            } else if (last) {
                has = false;
            }
            if (!has && a.hint) a.hint[idx] = (uint8_t)min(k - base_k + 1u, 255u);   // the next frame's look-ahead (SpecArgs::hint)
            left = !has;   // alive up to iteration k
            if (hit) {
                if (a.mode.ngp) {
                    float4 tmp = rgba;
                    if (a.mode.render_mode == 6) { const float c6 = (float)(j + istep) / 128; tmp = make_float4(c6, c6, c6, 1.0f); }
                    if (a.mode.render_mode == 1) { tmp.x = srgb_to_linear(tmp.x); tmp.y = srgb_to_linear(tmp.y); tmp.z = srgb_to_linear(tmp.z); }
                    float4 fb = a.frame_rgba[idx];
                    fb = make_float4(tmp.x + fb.x * (1.0f - tmp.w), tmp.y + fb.y * (1.0f - tmp.w), tmp.z + fb.z * (1.0f - tmp.w),
                                     tmp.w + fb.w * (1.0f - tmp.w));
                    a.frame_rgba[idx] = fb;
                    if (tmp.w > 0.2f) a.frame_depth[idx] = depth;
                } else {
                    const f3 orig = cam.c3 + d * t;
                    float4 fb = a.frame_rgba[idx];
                    const float ta = rgba.w;
                    const float sr = srgb_to_linear(rgba.x), sg = srgb_to_linear(rgba.y), sb = srgb_to_linear(rgba.z);
                    fb = make_float4(sr + fb.x * (1.0f - ta), sg + fb.y * (1.0f - ta), sb + fb.z * (1.0f - ta), ta + fb.w * (1.0f - ta));
                    a.frame_rgba[idx] = fb;
                    a.positions[3 * idx + 0] = orig.x; a.positions[3 * idx + 1] = orig.y; a.positions[3 * idx + 2] = orig.z;
                    if (ta > 0.2f) a.frame_depth[idx] = depth;
                }
                ++my_hits;
            }
            my_iter = max(my_iter, k + 1);
            istep += n_steps;
            ++k;
        }
        wave_add_keyed(a.ctrl->tail_live, k, -1, left);   // k: one past the ray's last iteration
        left = false;
        wave_sync();
    }

    // ---- statistics
    atomicAdd(&blk_hit, my_hits);
    atomicMax(&blk_iter, my_iter);
    atomicAdd(&blk_samples, my_samples);
    if (my_reused) atomicAdd(&blk_reused, my_reused);
    __syncthreads();
    if (threadIdx.x < 64) {
        if (hist_alive[threadIdx.x]) atomicAdd(&a.ctrl->alive_hist[threadIdx.x], hist_alive[threadIdx.x]);
        if (hist_samples[threadIdx.x]) atomicAdd(&a.ctrl->samples_hist[threadIdx.x], hist_samples[threadIdx.x]);
    }
    if (threadIdx.x == 0) {
        atomicAdd(&a.ctrl->n_hit, blk_hit);
        atomicMax(&a.ctrl->n_iter, blk_iter);
        atomicAdd(&a.ctrl->total_samples, blk_samples);
        if (blk_reused) atomicAdd(&a.ctrl->reused_samples, blk_reused);
    }
}

// =============================================================================================
// trace_alt's one-step regime (OnestepArgs, sng_internal.h)
// =============================================================================================
//
// While the frame-wide alive count n exceeds target / 2, trace_alt takes n_steps = 1 per
// iteration (testbed_nerf.cu:2189-2190) and its t reset (574) sends every ray back to the point it
// has just sampled: iteration m samples s_m = adv(t_m) (if_unoccupied_advance_to_next_occupied_voxel,
// 824) and the compositor sets t_{m+1} = g(s_m) = depth(s_m) / dot(fwd, dir).  t -> g(adv(t)) is a
// fixed float map, so once a ray's start t repeats (t_m == t_{m-P}) its samples -- and their network
// outputs -- repeat with period P: the ray composites the same P (sample, output) pairs again and
// again until its opacity passes 1 - min_transmittance.  In C4 (2 M rays alive for ~1100 one-step
// iterations) nearly every ray is periodic after an iteration or two, with P = 1.
//
// Exactness needs the schedule, and under n_steps = 1 a ray's fate does not depend on the others:
//   pass 0 (speculative): each lane simulates its ray alone under n_steps = 1 until it leaves --
//          dies, finds no occupied sample, or reaches MARCH_ITER -- evaluating the field only for
//          samples the ray has not seen in its last 4 iterations; periodic rays finish in a closed
//          loop over their opacity alone.  The iteration each ray leaves at is histogrammed;
//   schedule: alive(k + m) = n_k - prefix(deaths); the regime lasts J iterations, J = the first m
//          whose alive count allows 2 steps (or 0 alive, or MARCH_ITER); the per-iteration statistics
//          are those the wavefront records;
//   pass 1 (final): the same simulation stopped at k + J with full compositing; rays leaving before
//          k + J are extracted exactly as composite_kernel does, survivors are appended to the next
//          ray buffer with their boundary-sample cache.
constexpr int OS_P = 4;   // longest orbit closed (start t's remembered)

// A wave's LDS: the closed-loop section's orbit entries and the field section's staging are used one
// after the other in each trip (a wave's LDS operations execute in order), so they share the bytes.
union OnestepWaveLds {
    struct {
        float4 cyc[OS_P][64];    // orbit entry: logistic rgb, alpha
        float4 cycd[OS_P][64];   // orbit entry: depth, sample t, raw output (2 x u32)
    } orbit;
    struct {
        float4 ray[64][2];
        float s[64];
        uint8_t own[64];
        uint2 out[64];
    } field;
};

// The regime evaluates the field for few samples (the march and the closed loops are the work), so
// the weight fragments live in LDS, not in 80 VGPRs: 3 waves per SIMD instead of 2 (LDS: 3 workgroups
// x (20 KiB weights + 4 x 8 KiB) per CU).
// True when a ray compositing (in float) samples of alpha <= amax from opacity w0 provably stays at or below
// `opaque` for n more iterations.  One iteration is w' = fl(w + fl(a fl(1 - w))); with t = 1 - w and u = 2^-24,
// t' >= t (1 - a (1 + u)^2) - (w + weight) u >= r t - 1.0001 u, so t_n >= r^n t_0 - 1.0001 n u; w passes
// `opaque` only when t falls below 1 - opaque.  Evaluated in double with relative margins far above its error.
__device__ __forceinline__ bool os_no_death(float w0, float amax, uint32_t n, float opaque) {
    const double u = 5.9604644775390625e-08;
    const double ar = (double)amax * (1.0 + 2.0 * u + u * u) * (1.0 + 1e-12);
    if (!(ar < 0.5)) return false;
    const double tn = (1.0 - (double)w0) * exp((double)n * log1p(-ar) * (1.0 + 1e-12)) * (1.0 - 1e-12) - 1.0001 * (double)n * u;
    return tn > (1.0 - (double)opaque) * (1.0 + 1e-9) + 1e-15;
}

template <int F, bool FINAL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void nerf_onestep_kernel(OnestepArgs a) {
    __shared__ OnestepWaveLds wl[FUSED_WAVES];
    __shared__ h8 sW[20 * 64];
#define ray_lds(w, l, k) wl[w].field.ray[l][k]
#define s_lds(w, l) wl[w].field.s[l]
#define own_lds(w, l) wl[w].field.own[l]
#define out_lds(w, l) wl[w].field.out[l]
#define cyc_lds(w, q, l) wl[w].orbit.cyc[q][l]
#define cycd_lds(w, q, l) wl[w].orbit.cycd[q][l]

    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int g = lane >> 4, col = lane & 15;
    const Volume& vol = a.vol;
    const CamDev& cam = a.cam;
    OnestepState* os = a.os;
    const uint32_t n_rays = os->n_local;
    const uint32_t istep0 = os->istep0;
    const uint32_t limit = FINAL ? os->J : os->H;   // iterations simulated (relative to k)
    const f3 wdiag = vol.train_aabb.hi - vol.train_aabb.lo;
    const StepSpace cone = vol.ss;
    const float opaque = 1.0f - vol.min_transmittance;
    const h8* wfrag = reinterpret_cast<const h8*>(a.wfrag);
    const _Float16* grid = reinterpret_cast<const _Float16*>(a.grid_params);
    for (int k = threadIdx.x; k < 20 * 64; k += blockDim.x) sW[k] = wfrag[k];
    __syncthreads();
    const LdsWeights W{sW, lane};
    const float qnan = __int_as_float(0x7fc00000);

    bool has = false, own = true;
    f3 o = splat(0.0f), d = splat(1.0f);
    float t = 0.0f, depth = 0.0f;
    float4 rgba = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    uint32_t idx = 0, m = 0;
    float th0 = qnan, th1 = qnan, th2 = qnan, th3 = qnan;   // start t of iterations m-1 .. m-4
    float sc0 = qnan, sc1 = qnan, sc2 = qnan, sc3 = qnan;   // their samples
    uint2 oc0 = make_uint2(0u, 0u), oc1 = oc0, oc2 = oc0, oc3 = oc0;   // and raw outputs
    uint32_t my_evals = 0, my_hits = 0;

    // a ray leaves at relative iteration mm (it is not alive at k + mm + 1)
    auto record = [&](uint32_t mm, bool nos) {
        atomicAdd(&a.deaths_local[mm], 1u);
        if (a.sched.global && own) atomicAdd(&a.deaths_sched[mm], 1u);
        if (nos) atomicAdd(&a.nosample[mm], 1u);
    };
    // composite_kernel's hit path for trace_alt (extract_from_payload, testbed_nerf.cu:1578-1612)
    auto extract = [&]() {
        const f3 orig = cam.c3 + d * t;
        float4 fb = a.frame_rgba[idx];
        const float ta = rgba.w;
        const float sr = srgb_to_linear(rgba.x), sg = srgb_to_linear(rgba.y), sb = srgb_to_linear(rgba.z);
        fb = make_float4(sr + fb.x * (1.0f - ta), sg + fb.y * (1.0f - ta), sb + fb.z * (1.0f - ta), ta + fb.w * (1.0f - ta));
        a.frame_rgba[idx] = fb;
        a.positions[3 * idx + 0] = orig.x; a.positions[3 * idx + 1] = orig.y; a.positions[3 * idx + 2] = orig.z;
        if (ta > 0.2f) a.frame_depth[idx] = depth;
        ++my_hits;
    };

    while (true) {
        // ---- refill empty lanes from the ray queue (one atomic per wave)
        {
            const unsigned long long need = __ballot(!has);
            if (need) {
                const int leader = __ffsll((long long)need) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&os->work[FINAL ? 1 : 0], (uint32_t)__popcll(need));
                base = __shfl(base, leader, 64);
                if (!has) {
                    const uint32_t r = base + (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
                    if (r < n_rays) {
                        const float4 ot = a.in.o_t[r], di = a.in.d_idx[r];
                        o = mk(ot.x, ot.y, ot.z);
                        t = ot.w;
                        d = mk(di.x, di.y, di.z);
                        idx = __float_as_uint(di.w);
                        own = !a.sched.global || (idx >= a.sched.own_lo && idx < a.sched.own_hi);
                        rgba = a.in.rgba[r];
                        depth = a.in.depth[r];
                        th0 = th1 = th2 = th3 = qnan;
                        sc0 = a.in.lt[r].x; sc1 = sc2 = sc3 = qnan;   // the wavefront's boundary-sample cache
                        oc0 = a.in.lo[r];
                        m = 0;
                        has = true;
                    }
                }
            }
        }
        if (!__ballot(has)) break;

        bool survivor = false;   // FINAL: alive at k + J -> next ray buffer
        // ---- rays at the end of the span, and periodic rays (closed loop, no field evaluations)
        if (has) {
            if (m >= limit) {   // pass 0: alive at the horizon (the schedule's span ends there)
                survivor = FINAL;
                has = false;
            } else {
                const int P = t == th0 ? 1 : t == th1 ? 2 : t == th2 ? 3 : t == th3 ? 4 : 0;
                if (P) {
                    // orbit entry q (0..P-1) = the sample of iteration m - P + q, used at m + q, m + q + P, ...
                    bool all_zero = true;
                    float amax = 0.0f;   // the orbit's largest alpha
#pragma unroll
                    for (int q = 0; q < OS_P; ++q) {
                        if (q < P) {
                            const int src = P - 1 - q;
                            const float sq = src == 0 ? sc0 : src == 1 ? sc1 : src == 2 ? sc2 : sc3;
                            const uint2 raw = src == 0 ? oc0 : src == 1 ? oc1 : src == 2 ? oc2 : oc3;
                            const float dt = unwarp_dt(warp_dt(calc_dt(sq, cone)));
                            const f3 wp = ((o + d * sq) - vol.train_aabb.lo) / wdiag;
                            const f3 pos = vol.train_aabb.lo + wp * wdiag;
                            const float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x & 0xffffu));
                            const float gg = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x >> 16));
                            const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y & 0xffffu));
                            const float s = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y >> 16));
                            const float alpha = 1.f - sng_expf(-sng_expf(s) * dt);
                            all_zero = all_zero && alpha == 0.0f;
                            amax = fmaxf(amax, alpha);
                            cyc_lds(wv, q, lane) = make_float4(logistic(r), logistic(gg), logistic(b), alpha);
                            cycd_lds(wv, q, lane) = make_float4(dot(cam.c2, pos - cam.c3), sq, __uint_as_float(raw.x), __uint_as_float(raw.y));
                        }
                    }
                    const float dfw = dot(cam.c2, d);
                    uint32_t q = 0;
                    if (all_zero) {
                        // weights are exactly 0: rgba never changes, depth is the last composited sample's
                        if (FINAL) {
                            q = (limit - 1u - m) % (uint32_t)P;
                            depth = cycd_lds(wv, q, lane).x;
                            t = depth / dfw;
                            survivor = istep0 + limit < MARCH_ITER;   // else dropped in MARCH_ITER's last iteration
                        }
                        // pass 0: never opaque; dropped at MARCH_ITER's last iteration, past every schedule decision
                    } else {
                        uint32_t x0 = m;
                        bool stuck = false;
                        // iterations x < xnl are not the march's last (istep0 + x + 1 < MARCH_ITER) and inside the span
                        const uint32_t xnl = min(limit, istep0 + 1u < MARCH_ITER ? MARCH_ITER - 1u - istep0 : 0u);
                        if (!FINAL && xnl > m && os_no_death(rgba.w, amax, xnl - m, opaque)) {
                            // pass 0 needs only the iteration the ray leaves at, and it provably passes no opacity
                            // threshold before xnl: it is dropped at the march's last iteration, or alive at the span's end
                            if (xnl < limit) record(xnl, false);
                            stuck = true;
                        } else if (P == 1) {
                            // the orbit's one entry in registers: the iterations that neither pass the opacity
                            // threshold nor are the march's last run here without LDS reads or bookkeeping; the
                            // loop below takes over from the same state at the first one that does (the same float
                            // operations in the same order, so the same values)
                            const float4 c = cyc_lds(wv, 0, lane);
                            float w = rgba.w, cr = rgba.x, cg = rgba.y, cb = rgba.z;
                            // four iterations per check: the opacity never decreases (weights are >= 0), so the
                            // fourth's <= threshold clears all four; a fixed point (w unchanged) persists, so the
                            // fourth equal to the third catches one reached inside the block (pass 0 stops there)
                            while (x0 + 4u <= xnl) {
                                const float w1 = w + c.w * (1.f - w);
                                const float w2 = w1 + c.w * (1.f - w1);
                                const float w3 = w2 + c.w * (1.f - w2);
                                const float k3 = c.w * (1.f - w3);
                                const float w4 = w3 + k3;
                                if (w4 > opaque) break;
                                if (FINAL) {
                                    const float k0 = c.w * (1.f - w), k1 = c.w * (1.f - w1), k2 = c.w * (1.f - w2);
                                    cr += c.x * k0; cg += c.y * k0; cb += c.z * k0;
                                    cr += c.x * k1; cg += c.y * k1; cb += c.z * k1;
                                    cr += c.x * k2; cg += c.y * k2; cb += c.z * k2;
                                    cr += c.x * k3; cg += c.y * k3; cb += c.z * k3;
                                }
                                x0 += 4u;
                                const bool fixed = w4 == w3;
                                w = w4;
                                if (!FINAL && fixed) { stuck = true; break; }
                            }
                            for (; !stuck && x0 < xnl; ++x0) {
                                const float weight = c.w * (1.f - w);
                                const float wn = w + weight;
                                if (wn > opaque) break;
                                if (FINAL) {
                                    cr += c.x * weight;
                                    cg += c.y * weight;
                                    cb += c.z * weight;
                                } else if (wn == w) {   // opacity unchanged over the orbit: it never changes again
                                    stuck = true;
                                    break;
                                }
                                w = wn;
                            }
                            rgba = make_float4(cr, cg, cb, w);
                        } else {
                            // P = 2..4: one whole orbit per check, its entries in registers (a lane whose orbit is
                            // longer would otherwise hold its wave in the LDS loop below for ~1,100 iterations); the
                            // orbit that passes the threshold is replayed by that loop from the state before it
                            float4 e0 = cyc_lds(wv, 0, lane), e1 = cyc_lds(wv, 1, lane), e2 = e1, e3 = e1;
                            if (P > 2) e2 = cyc_lds(wv, 2, lane);
                            if (P > 3) e3 = cyc_lds(wv, 3, lane);
                            float w = rgba.w, cr = rgba.x, cg = rgba.y, cb = rgba.z;
                            while (x0 + (uint32_t)P <= xnl) {
                                float wn = w, nr = cr, ng = cg, nb = cb;
                                auto step = [&](const float4& c) {
                                    const float weight = c.w * (1.f - wn);
                                    if (FINAL) { nr += c.x * weight; ng += c.y * weight; nb += c.z * weight; }
                                    wn += weight;
                                };
                                step(e0);
                                step(e1);
                                if (P > 2) step(e2);
                                if (P > 3) step(e3);
                                if (wn > opaque) break;   // opacity never decreases: the orbit's last value decides
                                x0 += (uint32_t)P;
                                const bool fixed = wn == w;   // unchanged over a whole orbit: never changes again
                                w = wn; cr = nr; cg = ng; cb = nb;
                                if (!FINAL && fixed) { stuck = true; break; }
                            }
                            rgba = make_float4(cr, cg, cb, w);
                        }
                        float wprev = rgba.w;
                        for (uint32_t x = x0; !stuck; ++x) {
                            if (x >= limit) {   // FINAL: alive at k + J
                                survivor = FINAL;
                                break;
                            }
                            const float4 cq = cyc_lds(wv, q, lane);
                            const bool last = istep0 + x + 1u >= MARCH_ITER;
                            const float T = 1.f - rgba.w;
                            const float weight = cq.w * T;
                            if (FINAL) {
                                rgba.x += cq.x * weight;
                                rgba.y += cq.y * weight;
                                rgba.z += cq.z * weight;
                            }
                            rgba.w += weight;
                            if (rgba.w > opaque) {
                                if (FINAL) {
                                    const float aa = rgba.w;
                                    rgba.x /= aa; rgba.y /= aa; rgba.z /= aa; rgba.w /= aa;
                                    depth = cycd_lds(wv, q, lane).x;
                                    t = depth / dfw;
                                    if (!last) extract();
                                } else {
                                    record(x, false);
                                }
                                break;
                            }
                            if (last) {   // survives its composite but the march ends: dropped
                                if (!FINAL) record(x, false);
                                break;
                            }
                            if (++q == (uint32_t)P) {
                                q = 0;
                                if (!FINAL) {   // opacity unchanged over a whole orbit: it never changes again
                                    if (rgba.w == wprev) break;
                                    wprev = rgba.w;
                                }
                            }
                        }
                        if (FINAL && survivor) {
                            // alive at k + J: the last composited sample is the orbit entry before q
                            const uint32_t ql = q == 0 ? (uint32_t)P - 1u : q - 1u;
                            depth = cycd_lds(wv, ql, lane).x;
                            t = depth / dfw;
                        }
                    }
                    if (FINAL && survivor) {
                        const uint32_t ql = (limit - 1u - m) % (uint32_t)P;
                        const float4 e = cycd_lds(wv, ql, lane);
                        sc0 = e.y;
                        oc0 = make_uint2(__float_as_uint(e.z), __float_as_uint(e.w));
                    }
                    has = false;
                }
            }
        }

        // ---- stepping rays: one iteration (generate one sample, field if unseen, composite)
        bool need = false;
        float s = 0.0f;
        uint2 out = make_uint2(0u, 0u);
        if (has) {
            const f3 idir = inv(d);
            if (vol.linear) {
                s = advance_to_occupied(t, vol.cone, o, d, idir, 0, vol.max_mip, vol);
            } else {
                s = t;
                while (!occ_step(s, cone, o, d, idir, 0, vol.max_mip, vol)) {}
            }
            if (s >= MAX_DEPTH) {
                // no occupied sample: the compositor sees cnt = 0 < n_steps and retires the ray
                const bool last = istep0 + m + 1u >= MARCH_ITER;
                if (FINAL) {
                    if (!last && rgba.w > 0.001f) extract();
                } else {
                    record(m, true);
                }
                has = false;
            } else if (s == sc0) out = oc0;
            else if (s == sc1) out = oc1;
            else if (s == sc2) out = oc2;
            else if (s == sc3) out = oc3;
            else need = true;
        }
        // ---- field on the wave's unseen samples, 16 per tile (generate_kernel's coordinate expressions)
        const unsigned long long nb = __ballot(need);
        if (nb) {
            const uint32_t total = (uint32_t)__popcll(nb);
            const uint32_t slot = (uint32_t)__popcll(nb & ((1ull << lane) - 1ull));
            if (need) {
                own_lds(wv, slot) = (uint8_t)lane;
                s_lds(wv, lane) = s;
                ray_lds(wv, lane, 0) = make_float4(o.x, o.y, o.z, 0.0f);
                ray_lds(wv, lane, 1) = make_float4(d.x, d.y, d.z, 0.0f);
            }
            wave_sync();
            for (uint32_t tile = 0; tile * 16 < total; ++tile) {
                const uint32_t q = tile * 16 + (uint32_t)col;
                const bool valid = q < total;
                const uint32_t ol = own_lds(wv, valid ? q : 0);
                const float4 ro = ray_lds(wv, ol, 0), rd = ray_lds(wv, ol, 1);
                const float ts = s_lds(wv, ol);
                const f3 so = mk(ro.x, ro.y, ro.z), sd = mk(rd.x, rd.y, rd.z);
                const f3 wp = ((so + sd * ts) - vol.train_aabb.lo) / wdiag;
                const f3 wd = (sd + 1.0f) * 0.5f;
                f4v fo, dens;
                field_tile<F>(W, a.levels, grid, g, wp.x, wp.y, wp.z, wd.x, wd.y, wd.z, fo, dens);
                if (valid && g == 0) {
                    const _Float16 r = (_Float16)fo[0], gg = (_Float16)fo[1], b = (_Float16)fo[2], sg = (_Float16)dens[0];
                    out_lds(wv, q) = make_uint2((uint32_t)__builtin_bit_cast(uint16_t, r) | ((uint32_t)__builtin_bit_cast(uint16_t, gg) << 16),
                                                (uint32_t)__builtin_bit_cast(uint16_t, b) | ((uint32_t)__builtin_bit_cast(uint16_t, sg) << 16));
                }
            }
            wave_sync();
            if (need) { out = out_lds(wv, slot); ++my_evals; }
            wave_sync();
        }
        // ---- composite the stepped sample (composite_kernel_nerf_alt 535-574 with n_steps = 1)
        if (has) {
            const bool last = istep0 + m + 1u >= MARCH_ITER;
            const float dt = unwarp_dt(warp_dt(calc_dt(s, cone)));
            const f3 wp = ((o + d * s) - vol.train_aabb.lo) / wdiag;
            const f3 pos = vol.train_aabb.lo + wp * wdiag;
            const float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(out.x & 0xffffu));
            const float gg = (float)__builtin_bit_cast(_Float16, (uint16_t)(out.x >> 16));
            const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(out.y & 0xffffu));
            const float sg = (float)__builtin_bit_cast(_Float16, (uint16_t)(out.y >> 16));
            const float T = 1.f - rgba.w;
            const float alpha = 1.f - sng_expf(-sng_expf(sg) * dt);
            const float weight = alpha * T;
            rgba.x += logistic(r) * weight;
            rgba.y += logistic(gg) * weight;
            rgba.z += logistic(b) * weight;
            rgba.w += weight;
            depth = dot(cam.c2, pos - cam.c3);
            const float t_start = t;
            t = depth / dot(cam.c2, d);
            if (rgba.w > opaque) {
                if (FINAL) {
                    const float aa = rgba.w;
                    rgba.x /= aa; rgba.y /= aa; rgba.z /= aa; rgba.w /= aa;
                    if (!last) extract();
                } else {
                    record(m, false);
                }
                has = false;
            } else if (last) {
                if (!FINAL) record(m, false);
                has = false;
            } else {
                th3 = th2; th2 = th1; th1 = th0; th0 = t_start;
                sc3 = sc2; sc2 = sc1; sc1 = sc0; sc0 = s;
                oc3 = oc2; oc2 = oc1; oc1 = oc0; oc0 = out;
                ++m;
            }
        }

        // ---- FINAL: survivors to the next ray buffer (one atomic per wave)
        if (FINAL) {
            const unsigned long long sv = __ballot(survivor);
            if (sv) {
                const int leader = __ffsll((long long)sv) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&a.ctrl->n_alive[a.p ^ 1], (uint32_t)__popcll(sv));
                base = __shfl(base, leader, 64);
                if (a.sched.global) {
                    const unsigned long long so = __ballot(survivor && own);
                    if (so && lane == leader) atomicAdd(&a.ctrl->n_owned[a.p ^ 1], (uint32_t)__popcll(so));
                }
                if (survivor) {
                    const uint32_t slot = base + (uint32_t)__popcll(sv & ((1ull << lane) - 1ull));
                    a.out.o_t[slot] = make_float4(o.x, o.y, o.z, t);
                    a.out.d_idx[slot] = make_float4(d.x, d.y, d.z, __uint_as_float(idx));
                    a.out.rgba[slot] = rgba;
                    a.out.depth[slot] = depth;
                    a.out.lt[slot] = make_float2(sc0, 0.0f);
                    a.out.lo[slot] = oc0;
                }
            }
        }
    }

    // ---- statistics
    if (my_evals) atomicAdd(&os->evals[FINAL ? 1 : 0], (unsigned long long)my_evals);
    if (FINAL) {
        if (my_hits) atomicAdd(&a.ctrl->n_hit, my_hits);
        // the schedule counted every regime sample as reused; the final pass's evaluations were not
        if (my_evals) atomicAdd(&a.ctrl->reused_samples, (unsigned long long)(-(long long)my_evals));
    }
}

#undef ray_lds
#undef s_lds
#undef own_lds
#undef out_lds
#undef cyc_lds
#undef cycd_lds

__global__ void onestep_begin_kernel(OnestepArgs a, uint32_t k, uint32_t horizon, int first) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ONESTEP_HIST; i += gridDim.x * blockDim.x) {
        a.deaths_local[i] = 0;
        a.deaths_sched[i] = 0;
        a.nosample[i] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const MarchCtrl* c = a.ctrl;
        OnestepState* os = a.os;
        os->k = k;
        os->istep0 = c->i_step[a.p];
        os->n_local = c->n_alive[a.p];
        os->n_sched = a.sched.global ? c->sched_alive[a.p] : c->n_alive[a.p];
        const uint32_t left = c->i_step[a.p] < MARCH_ITER ? MARCH_ITER - c->i_step[a.p] : 0u;
        os->H = left < horizon ? left : horizon;   // a regime longer than the horizon continues in a new segment
        os->J = 0;
        os->work[0] = 0; os->work[1] = 0;
        if (first) { os->evals[0] = 0; os->evals[1] = 0; }   // accumulated over the segments of a frame
    }
}

// alive(k + m) = n_k - sum_{x < m} deaths[x]; J = first m in [0, H) whose alive count is 0 or allows
// more than one step (H: MARCH_ITER).  Statistics as generate/composite record them per iteration.
// one 256-thread workgroup (a 1024-thread one waited ~0.5 ms for a free CU beside the raytracer's persistent grids)
constexpr uint32_t OS_SCHED_THREADS = 256;
__global__ __launch_bounds__(OS_SCHED_THREADS) void onestep_schedule_kernel(OnestepArgs a) {
    constexpr uint32_t CH = ONESTEP_HIST / OS_SCHED_THREADS;
    static_assert(ONESTEP_HIST % OS_SCHED_THREADS == 0, "histogram split");
    __shared__ uint32_t ps[OS_SCHED_THREADS], pl[OS_SCHED_THREADS];
    __shared__ uint32_t J_sh;
    __shared__ unsigned long long slots_sh, samp_sh;
    OnestepState* os = a.os;
    MarchCtrl* c = a.ctrl;
    const uint32_t H = os->H, k = os->k, tid = threadIdx.x;
    const uint32_t* ds = a.sched.global ? a.deaths_sched : a.deaths_local;
    const uint32_t b0 = tid * CH;
    uint32_t ss = 0, sl = 0;
    for (uint32_t x = 0; x < CH; ++x)
        if (b0 + x < H) { ss += ds[b0 + x]; sl += a.deaths_local[b0 + x]; }
    ps[tid] = ss; pl[tid] = sl;
    if (tid == 0) { J_sh = H; slots_sh = 0; samp_sh = 0; }
    __syncthreads();
    for (uint32_t off = 1; off < OS_SCHED_THREADS; off <<= 1) {   // inclusive Hillis-Steele scans
        const uint32_t vs = tid >= off ? ps[tid - off] : 0u, vl = tid >= off ? pl[tid - off] : 0u;
        __syncthreads();
        ps[tid] += vs; pl[tid] += vl;
        __syncthreads();
    }
    uint32_t alive_s = os->n_sched - (ps[tid] - ss);
    for (uint32_t x = 0; x < CH; ++x) {
        const uint32_t mm = b0 + x;
        if (mm >= H) break;
        if (alive_s == 0 || steps_for(alive_s, a.target) > 1) { atomicMin(&J_sh, mm); break; }
        alive_s -= ds[mm];
    }
    __syncthreads();
    const uint32_t J = J_sh;
    uint32_t alive_l = os->n_local - (pl[tid] - sl);
    unsigned long long slots = 0, samp = 0;
    for (uint32_t x = 0; x < CH; ++x) {
        const uint32_t mm = b0 + x;
        if (mm >= J) break;
        const uint32_t sm = alive_l - a.nosample[mm];
        slots += ((unsigned long long)alive_l + 255ull) / 256ull * 256ull;
        samp += sm;
        if (k + mm < 64) { c->alive_hist[k + mm] = alive_l; c->steps_hist[k + mm] = 1; c->samples_hist[k + mm] = sm; }
        if (c->log && k + mm < MARCH_LOG_CAP) { c->log[3 * (k + mm)] = alive_l; c->log[3 * (k + mm) + 1] = 1; c->log[3 * (k + mm) + 2] = sm; }
        if (k + mm < TAIL_LIVE_CAP) c->sched_hint[k + mm] = 1u;
        alive_l -= a.deaths_local[mm];
    }
    if (slots) atomicAdd(&slots_sh, slots);
    if (samp) atomicAdd(&samp_sh, samp);
    __syncthreads();
    if (tid == 0) {
        c->ref_slots += slots_sh;
        c->total_samples += samp_sh;
        c->reused_samples += samp_sh;   // the final pass subtracts its field evaluations
        c->n_iter = k + J;
        c->i_step[a.p ^ 1] = os->istep0 + J;
        c->n_alive[a.p ^ 1] = 0;
        c->n_owned[a.p ^ 1] = 0;
        c->n_samples[a.p ^ 1] = 0;
        c->n_reused[a.p ^ 1] = 0;
        os->J = J;
    }
}

void launch_onestep_begin(const OnestepArgs& a, uint32_t k, uint32_t horizon, int first, hipStream_t s) {
    hipLaunchKernelGGL(onestep_begin_kernel, dim3((ONESTEP_HIST + 255) / 256), dim3(256), 0, s, a, k, horizon, first);
}
void launch_onestep_schedule(const OnestepArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(onestep_schedule_kernel, dim3(1), dim3(OS_SCHED_THREADS), 0, s, a);
}
void launch_onestep_pass(const OnestepArgs& a, const NetworkDev& net, int final_pass, uint32_t n_rays_hint, hipStream_t s) {

    const uint32_t waves = (n_rays_hint + 63) / 64;
    const uint32_t blocks = std::max(1u, std::min((waves + FUSED_WAVES - 1) / FUSED_WAVES, (uint32_t)net.n_cus * 8));
    if (net.F == 4) {
        if (final_pass) hipLaunchKernelGGL((nerf_onestep_kernel<4, true>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
        else hipLaunchKernelGGL((nerf_onestep_kernel<4, false>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
    } else {
        if (final_pass) hipLaunchKernelGGL((nerf_onestep_kernel<2, true>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
        else hipLaunchKernelGGL((nerf_onestep_kernel<2, false>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
    }
}

__global__ void fused_prepare_kernel(MarchCtrl* ctrl, uint32_t* work) {
    // iterations from n_iter on take 8 steps each (the fused kernel's precondition)
    if (threadIdx.x < 64 && threadIdx.x >= ctrl->n_iter) ctrl->steps_hist[threadIdx.x] = MAX_STEPS_BETWEEN_COMPACTION;
    if (threadIdx.x == 0) *work = 0;
}

void launch_nerf_fused(const FusedArgs& a, const NetworkDev& net, uint32_t n_rays_hint, uint32_t max_blocks, hipStream_t s, bool prepare) {
    if (prepare) hipLaunchKernelGGL(fused_prepare_kernel, dim3(1), dim3(64), 0, s, a.ctrl, a.work);   // else launch_tail_prepare did it
    const uint32_t waves_needed = (n_rays_hint + a.lanes - 1) / a.lanes;
    const uint32_t cap = max_blocks ? max_blocks : (uint32_t)net.n_cus * 2;
    const uint32_t blocks = std::max(1u, std::min((waves_needed + FUSED_WAVES - 1) / FUSED_WAVES, cap));
    const bool lin = a.vol.linear != 0;
    if (net.F == 4) {
        if (lin) hipLaunchKernelGGL((nerf_fused_kernel<4, true>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
        else hipLaunchKernelGGL((nerf_fused_kernel<4, false>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
    } else {
        if (lin) hipLaunchKernelGGL((nerf_fused_kernel<2, true>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
        else hipLaunchKernelGGL((nerf_fused_kernel<2, false>), dim3(blocks), dim3(64 * FUSED_WAVES), 0, s, a);
    }
}

}  // namespace sng
