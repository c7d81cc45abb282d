// nerf.hip -- occupancy-grid ray marcher, wavefront compactor and compositor.
//
// Replaces NerfTracer::init_rays_from_camera / trace_alt (testbed_nerf.cu:2037-2277)
// and the kernels init_rays_with_payload_kernel_nerf (1855-1970), advance_pos_nerf
// (334-384), compact_kernel_nerf (1830-1853), generate_next_nerf_network_inputs
// (790-837), composite_kernel_nerf_alt (476-575), extract_from_payload (1578-1612),
// write_normals_to_buffer (1523-1576) and the bitfield build (285-332, 3212-3229).
//
// MI355X design: the host never reads n_alive between iterations.  Each
// iteration is three launches whose sizes come from a device control block:
//   generate  : marches up to n_steps occupied samples per alive ray, reserves a
//               contiguous sample range with one atomic per wave (wave scan), and
//               writes only REAL samples (no stale slots, no 256-padding);
//   network   : fused encode+MLP over exactly the reserved samples;
//   composite : front-to-back compositing, then in the same kernel either the
//               ray dies (extract_from_payload is applied directly to the frame
//               buffer) or it is appended to the next alive buffer (compaction
//               fused into the producer).
// n_steps = clamp(2^21 / n_alive, 1, 8) and the payload.t reset to the last
// sample (composite_kernel_nerf_alt:574) are reproduced exactly, so per-pixel
// results follow the reference's schedule.
#include <algorithm>

#include "sng_internal.h"
#include "sng_math.h"

namespace sng {

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t o = __shfl_up(v, off, 64);
        if (lane >= off) v += o;
    }
    return v;
}

// Block-aggregated append for blocks of NW waves: ONE returning atomic on `counter` per
// workgroup trip instead of one per wave (same-address atomics serialise at ~10 ns each, so a
// 2M-ray iteration with per-wave atomics spends ~0.3 ms on them alone).  Returns each lane's
// exclusive slot for its `v` entries; `a`/`b` are count-only flags summed into cnt_a/cnt_b
// (null: skipped).  Must be reached by every thread of the block.
template <int NW = 4>
__device__ __forceinline__ uint32_t block_append(uint32_t* counter, uint32_t v, uint32_t* cnt_a, bool a, uint32_t* cnt_b, bool b,
                                                 uint32_t* sh, int lane) {
    const int wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v, lane);
    const uint32_t na = (uint32_t)__popcll(__ballot(a)), nb = (uint32_t)__popcll(__ballot(b));
    if (lane == 63) sh[wave] = incl;
    if (lane == 0) { sh[NW + wave] = na; sh[2 * NW + wave] = nb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t sv = 0, sa = 0, sb = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) { const uint32_t t = sh[w]; sh[w] = sv; sv += t; sa += sh[NW + w]; sb += sh[2 * NW + w]; }
        sh[3 * NW] = sv ? atomicAdd(counter, sv) : 0u;
        if (cnt_a && sa) atomicAdd(cnt_a, sa);
        if (cnt_b && sb) atomicAdd(cnt_b, sb);
    }
    __syncthreads();
    const uint32_t r = sh[3 * NW] + sh[wave] + incl - v;
    __syncthreads();   // sh is reused by the next trip
    return r;
}

// ---------------------------------------------------------------------------
// init_rays_with_payload_kernel_nerf + advance_pos_nerf + first compaction
// ---------------------------------------------------------------------------
// BRICK: the march to the first occupied voxel reads the occupancy bricks staged in LDS (one copy per
// workgroup of a persistent grid striding over the pixels) with branch-free trips; otherwise one thread per
// pixel with the linear / cascaded marcher.
template <bool BRICK>
__global__ __launch_bounds__(256) void init_rays_kernel(NerfFrameArgs a, RayBuf out, MarchCtrl* ctrl, float4* __restrict__ frame_rgba,
                                                        float* __restrict__ frame_depth, float* __restrict__ positions,
                                                        float* __restrict__ normals, uint32_t n_threads) {
    extern __shared__ uint32_t occ_lds[];
    __shared__ uint32_t sh_app[16];
    if constexpr (BRICK) stage_occ_brick(occ_lds, a.vol.occ_brick, a.vol.occ_brick_words);
    const int lane = threadIdx.x & 63;
    const uint32_t n_band = (uint32_t)(a.row1 - a.row0) * (uint32_t)a.W;
    for (uint32_t base = blockIdx.x * 256u; base < n_threads; base += gridDim.x * 256u) {   // block-uniform trips
        const uint32_t t = base + threadIdx.x;
        bool alive = false;
        f3 origin = a.cam.c3, dir = splat(0.0f);
        float tt = 0.0f;
        uint32_t idx = 0;
        int x, y;
        bool in_band;
        x = (int)(t % (uint32_t)a.W);
        y = a.row0 + (int)(t / (uint32_t)a.W);
        in_band = t < n_band;
        if (in_band) {
            idx = (uint32_t)x + (uint32_t)a.W * (uint32_t)y;
            f2 off = ld_random_pixel_offset(a.snap ? 0u : a.spp);
            f2 uv = {((float)x + off.x) / (float)a.W, ((float)y + off.y) / (float)a.H};
            // get_xform_given_rolling_shutter (testbed_nerf.cu:1895, common_device.cuh:361-368)
            const float* rs = a.rolling_shutter;
            const float pixel_t = rs[0] + rs[1] * uv.x + rs[2] * uv.y + rs[3] * ld_random_val0(a.spp, idx * 72239731u);
            origin = a.cam.c3 + (a.pos1 - a.cam.c3) * pixel_t;
            // uv_to_ray (common_device.cuh:403-470): the frame's lens (Perspective unless render_with_lens_distortion),
            // no foveation / parallax / aperture
            f3 d;
            bool valid = true;
            if (a.lens.mode == LENS_PERSPECTIVE)
                d = mk((uv.x - a.screen_center.x) * (float)a.W / a.focal.x, (uv.y - a.screen_center.y) * (float)a.H / a.focal.y, 1.0f);
            else
                valid = lens_dir(a.lens, uv, a.screen_center, a.W, a.H, a.focal, d);
            d = mul(shutter_rotation(a.q0, a.q1, pixel_t), d);
            float4 fb = frame_rgba[idx];
            if (valid) { fb.x = 0.0f; fb.y = 0.0f; fb.z = 0.0f; }   // an invalid ray returns before the clear (1919-1923)
            if (a.reset) fb.w = 0.0f;
            frame_rgba[idx] = fb;
            frame_depth[idx] = MAX_DEPTH;
            positions[3 * idx + 0] = 0.0f; positions[3 * idx + 1] = 0.0f; positions[3 * idx + 2] = 0.0f;
            normals[3 * idx + 0] = 0.0f; normals[3 * idx + 1] = 0.0f; normals[3 * idx + 2] = 0.0f;
            dir = normalize(d);
            const Volume& v = a.vol;
            float t0 = fmaxf(aabb_entry(v.render_aabb, to_local(v, origin), to_local(v, dir)), 0.0f) + 1e-6f;
            if (valid && aabb_contains(v.render_aabb, to_local(v, origin + dir * t0))) {
                // advance_pos_nerf (testbed_nerf.cu:334-363)
                f3 idir = inv(dir);
                float t1 = advance_n_steps(t0, v.cone, ld_random_val0(a.spp, idx * 786433u));
                if constexpr (BRICK) {
                    // advance_to_occupied_linear through the LDS bricks, one DDA step per trip, no branch but the exits
                    const f3 hs = half_sign(dir);
                    // past t_last the line meets no occupied cell (path_last_occupied_t): the walk's end is known
                    const float t_last = path_last_occupied_t(origin, dir, idir, t1, occ_lds);
#pragma unroll 1
                    while (true) {
                        const f3 pos = origin + dir * t1;
                        const bool inside = (t1 < MAX_DEPTH) & (t1 <= t_last) & aabb_contains_nb(v.render_aabb, pos);
                        const bool occ = inside & occupied_brick_nb(pos, occ_lds);
                        const float tn = dda_step_linear(t1, pos, idir, hs);
                        if (!inside) { t1 = MAX_DEPTH; break; }
                        if (occ) break;
                        t1 = tn;
                    }
                } else {
                    t1 = advance_to_occupied(t1, v.cone, origin, dir, idir, 0, v.max_mip, v);
                }
                if (t1 < MAX_DEPTH) { alive = true; tt = t1; }
            }
        }
        const uint32_t slot = block_append(&ctrl->n_alive[0], alive ? 1u : 0u, a.sched.global ? &ctrl->n_owned[0] : nullptr,
                                           alive && idx >= a.sched.own_lo && idx < a.sched.own_hi, nullptr, false, sh_app, lane);
        if (alive) {
            out.o_t[slot] = make_float4(origin.x, origin.y, origin.z, tt);
            out.d_idx[slot] = make_float4(dir.x, dir.y, dir.z, __uint_as_float(idx));
            out.rgba[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // memset(m_rays[0].rgba) 2102
            out.depth[slot] = 0.0f;                                // memset(m_rays[0].depth) 2103
            if (a.mode.ngp) out.mw[slot] = 0.0f;                   // payload.max_weight = 0 (1964)
            else out.lt[slot] = make_float2(__int_as_float(0x7fc00000), 0.0f);   // no cached boundary sample yet
        }
    }
}

// ---------------------------------------------------------------------------
// generate_next_nerf_network_inputs (790-837), real samples only
// coords: NerfCoordinate AoS {warp(pos), warp_dt(dt), warp(dir)} (nerf_device.cuh:176-202)
// ---------------------------------------------------------------------------
//
// LIN (cone == 0, max_cascade == 0, the unit-cube scenes): the march is the exact linear
// specialisation (advance_to_occupied_linear) and the loop is NOT unrolled -- the sample
// distances of a ray go to LDS instead of 8 live registers, which keeps the kernel small
// and at high occupancy (the DDA walk is latency bound: many waves in flight hide the
// bitfield gathers).  The general path (cascades / cone stepping) keeps the unrolled form.
template <bool LIN, int THREADS = 256, bool BRICK = false>
__global__ __launch_bounds__(THREADS) void generate_kernel(Volume vol, RayBuf rays, MarchCtrl* ctrl, int p, uint32_t target, uint32_t iter,
                                                       float* __restrict__ coords, uint2* __restrict__ samp, int store_t, int global_sched) {
    __shared__ float ts_lds[MAX_STEPS_BETWEEN_COMPACTION * THREADS];
    extern __shared__ uint32_t occ_lds[];
    const uint32_t n_alive = ctrl->n_alive[p];
    const uint32_t n_sched = global_sched ? ctrl->sched_alive[p] : n_alive;   // Sched
    const uint32_t i_step = ctrl->i_step[p];
    const bool active = n_sched > 0 && i_step < MARCH_ITER;
    const uint32_t n_steps = active ? steps_for(n_sched, target) : 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctrl->n_alive[p ^ 1] = 0;
        ctrl->n_owned[p ^ 1] = 0;
        ctrl->i_step[p ^ 1] = i_step + n_steps;
        if (active) {
            if (iter < 64) { ctrl->alive_hist[iter] = n_alive; ctrl->steps_hist[iter] = n_steps; }
            if (ctrl->log && iter < MARCH_LOG_CAP) { ctrl->log[3 * iter] = n_alive; ctrl->log[3 * iter + 1] = n_steps; }
            if (iter < TAIL_LIVE_CAP) ctrl->sched_hint[iter] = (uint8_t)n_steps;
            ctrl->n_iter = iter + 1;
            ctrl->ref_slots += ((unsigned long long)n_alive * n_steps + 255ull) / 256ull * 256ull;
        }
    }
    if (!active) return;
    if constexpr (BRICK) {
        if (blockIdx.x * blockDim.x >= n_alive) return;
        stage_occ_brick(occ_lds, vol.occ_brick, vol.occ_brick_words);
    }
    const int lane = threadIdx.x & 63;
    const f3 wdiag = vol.train_aabb.hi - vol.train_aabb.lo;
    const StepSpace cone = LIN ? step_space(0.0f) : vol.ss;
    __shared__ uint32_t sh_app[3 * (THREADS / 64) + 1];
    // block-uniform trips (block_append syncs the block)
    for (uint32_t blk = blockIdx.x * blockDim.x; blk < n_alive; blk += gridDim.x * blockDim.x) {
        const uint32_t i = blk + threadIdx.x;
        uint32_t cnt = 0;
        bool reuse = false;
        f3 o = splat(0.0f), d = splat(1.0f);
        if (i < n_alive) {
            float4 ot = rays.o_t[i], di = rays.d_idx[i];
            o = mk(ot.x, ot.y, ot.z);
            d = mk(di.x, di.y, di.z);
            const f3 idir = inv(d);
            float t = ot.w;
            // trace_alt: the previous iteration's last sample (t and output) -- if this iteration's first
            // sample lands on the same t, its NerfCoordinate is bit-identical and so is the network output
            const float lt0 = store_t ? __int_as_float(0x7fc00000) : rays.lt[i].x;
            float tl = 0.0f;
            if constexpr (LIN && BRICK) {
                // the same loop through the LDS occupancy bricks, branch-free but for the exits; past t_last no
                // occupied cell is left on the ray (path_last_occupied_t), so the march ends there
                const f3 hs = half_sign(d);
                const float t_last = path_last_occupied_t(o, d, idir, t, occ_lds);
#pragma unroll 1
                while (cnt < n_steps) {
                    const f3 pos = o + d * t;
                    const bool inside = (t < MAX_DEPTH) & (t <= t_last) & aabb_contains_nb(vol.render_aabb, pos);
                    const bool occ = inside & occupied_brick_nb(pos, occ_lds);
                    const float tn = dda_step_linear(t, pos, idir, hs);
                    if (!inside) break;
                    if (occ) {
                        if (cnt == 0 && t == lt0) reuse = true;
                        ts_lds[cnt * THREADS + threadIdx.x] = t;
                        tl = t;
                        t += calc_dt(t, 0.0f);
                        ++cnt;
                    } else {
                        t = tn;
                    }
                }
            } else if constexpr (LIN) {
                // advance_to_occupied_linear + sample, flattened into ONE loop: each trip either
                // records a sample (occupied voxel) or takes one DDA step, so a lane's cost is its
                // own total step count instead of the wave's worst walk summed over all 8 samples.
                const f3 hs = half_sign(d);
                OccCache oc;
#pragma unroll 1
                while (cnt < n_steps) {
                    const f3 pos = o + d * t;
                    if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) break;
                    if (occupied_linear_c(pos, vol.occ_linear, oc)) {
                        if (cnt == 0 && t == lt0) reuse = true;
                        ts_lds[cnt * THREADS + threadIdx.x] = t;
                        tl = t;
                        t += calc_dt(t, 0.0f);
                        ++cnt;
                    } else {
                        t = dda_step_linear(t, pos, idir, hs);
                    }
                }
            } else {
                // cascades / cone stepping: the same flattened loop over occ_step trips
#pragma unroll 1
                while (cnt < n_steps) {
                    if (occ_step(t, cone, o, d, idir, 0, vol.max_mip, vol)) {
                        if (t >= MAX_DEPTH) break;
                        if (cnt == 0 && t == lt0) reuse = true;
                        ts_lds[cnt * THREADS + threadIdx.x] = t;
                        tl = t;
                        t += calc_dt(t, cone);
                        ++cnt;
                    }
                }
            }
            // NerfTracer::trace keeps generate's t (payload.t = t after n_steps samples, 836);
            // trace_alt overwrites it in the compositor
            if (store_t && cnt == n_steps) reinterpret_cast<float*>(rays.o_t + i)[3] = t;
            if (!store_t && cnt) rays.lt[i] = make_float2(lt0, tl);
        }
        const uint32_t ru = reuse ? 1u : 0u;
        const uint32_t base = block_append<THREADS / 64>(&ctrl->n_samples[p], cnt - ru, &ctrl->n_reused[p], reuse, nullptr, false, sh_app, lane);
        if (i < n_alive) {
            samp[i] = make_uint2(base, cnt | (ru << 31));
            const f3 wd = (d + 1.0f) * 0.5f;
#pragma unroll 1
            for (uint32_t j = ru; j < cnt; ++j) {
                const float t = ts_lds[j * THREADS + threadIdx.x];
                const float dt = calc_dt(t, cone);
                const f3 wp = ((o + d * t) - vol.train_aabb.lo) / wdiag;
                float* c = coords + (size_t)(base + j - ru) * 7;
                c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(dt); c[4] = wd.x; c[5] = wd.y; c[6] = wd.z;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// composite_kernel_nerf_alt (476-575) + compaction into the next buffer
// (compact_kernel_nerf 1830-1853) + extract_from_payload (1578-1612)
// ---------------------------------------------------------------------------
// composite_kernel_nerf's glow visualisation (testbed_nerf.cu:638-734): green grid lines / cut line
// below glow_y_cutoff; adds to rgb (grid_mode replaces it) and may scale the sample weight
__device__ __forceinline__ void glow_term(int glow_mode, float glow_y_cutoff, f3 pos, f3 cam_pos, f3& rgb, float& weight) {
    float glow = 0.f;
    const bool green_grid = glow_mode & 1, green_cutline = glow_mode & 2, mask_to_alpha = glow_mode & 4;
    const bool radial_mode = glow_mode & 8, grid_mode = glow_mode & 16;
    float dist;
    if (radial_mode) {
        dist = length(pos - cam_pos);
        dist = fminf(dist, (4.5f - pos.y) * 0.333f);
    } else {
        dist = pos.y;
    }
    if (grid_mode) {
        glow = 1.f / fmaxf(1.f, dist);
    } else {
        float y = glow_y_cutoff - dist;
        float mask = 0.f;
        if (y > 0.f) {
            y *= 80.f;
            mask = fminf(1.f, y);
            if (green_cutline) glow += fmaxf(0.f, 1.f - fabsf(1.f - y)) * 4.f;
            if (y > 1.f) y = 1.f - (y - 1.f) * 0.05f;
            if (green_grid) glow += fmaxf(0.f, y / fmaxf(1.f, dist));
        }
        if (mask_to_alpha) weight *= mask;
    }
    if (glow > 0.f) {
        float line = 0.f;
        for (int q = 0; q < 4; ++q) {   // y, x, z lines at 2, 4, 8, 16 x 16 periods per unit
            const float m = 2.f * (float)(1 << q);
            line += fmaxf(0.f, cosf(pos.y * m * 3.141592653589793f * 16.f) - 0.975f);
            line += fmaxf(0.f, cosf(pos.x * m * 3.141592653589793f * 16.f) - 0.975f);
            line += fmaxf(0.f, cosf(pos.z * m * 3.141592653589793f * 16.f) - 0.975f);
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

template <int THREADS>
__global__ __launch_bounds__(THREADS) void composite_kernel(Volume vol, CamDev cam, TraceMode mode, Sched sched, RayBuf in, RayBuf out, MarchCtrl* ctrl, int p,
                                                        uint32_t target, uint32_t iter, const float* __restrict__ coords, const uint2* __restrict__ samp,
                                                        const uint2* __restrict__ net_out, float4* __restrict__ frame_rgba,
                                                        float* __restrict__ frame_depth, float* __restrict__ positions) {
    const uint32_t n_alive = ctrl->n_alive[p];
    const uint32_t n_sched = sched.global ? ctrl->sched_alive[p] : n_alive;
    const uint32_t i_step = ctrl->i_step[p];
    const bool active = n_sched > 0 && i_step < MARCH_ITER;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (active) {
            ctrl->total_samples += ctrl->n_samples[p] + ctrl->n_reused[p];
            ctrl->net_samples += ctrl->n_samples[p];
            ctrl->reused_samples += ctrl->n_reused[p];
            if (iter < 64) ctrl->samples_hist[iter] = ctrl->n_samples[p] + ctrl->n_reused[p];
            if (ctrl->log && iter < MARCH_LOG_CAP) ctrl->log[3 * iter + 2] = ctrl->n_samples[p] + ctrl->n_reused[p];
        }
        ctrl->n_samples[p ^ 1] = 0;
        ctrl->n_reused[p ^ 1] = 0;
    }
    if (!active) return;
    const uint32_t n_steps = steps_for(n_sched, target);
    // the reference leaves the loop without another compaction once i >= MARCH_ITER
    const bool last = i_step + n_steps >= MARCH_ITER;
    const int lane = threadIdx.x & 63;
    const f3 diag = vol.train_aabb.hi - vol.train_aabb.lo;
    __shared__ uint32_t sh_app[3 * (THREADS / 64) + 1];
    for (uint32_t blk = blockIdx.x * blockDim.x; blk < n_alive; blk += gridDim.x * blockDim.x) {
        const uint32_t i = blk + threadIdx.x;
        bool survive = false, hit = false;
        float4 rgba = make_float4(0, 0, 0, 0), ot = rgba, di = rgba;
        float depth = 0.0f, mw = 0.0f;
        float2 lt = make_float2(0.0f, 0.0f);
        uint2 last_raw = make_uint2(0u, 0u);
        uint32_t death_step = 0;
        if (i < n_alive) {
            rgba = in.rgba[i];
            depth = in.depth[i];
            ot = in.o_t[i];
            di = in.d_idx[i];
            if (mode.ngp) mw = in.mw[i];
            else lt = in.lt[i];
            const uint2 sc = samp[i];
            const uint32_t cnt = sc.y & 0x7fffffffu, ru = sc.y >> 31;
            uint32_t j = 0;
            for (; j < cnt; ++j) {
                uint2 raw;
                f3 pos;
                float dt;
                const bool cached = ru && j == 0;
                const float* c = coords + (cached ? (size_t)0 : (size_t)sc.x + j - ru) * 7;   // c unused when cached (trace_alt)
                if (cached) {   // the cached boundary sample: generate_kernel's expressions on its t
                    raw = in.lo[i];
                    const f3 wp = ((mk(ot.x, ot.y, ot.z) + mk(di.x, di.y, di.z) * lt.x) - vol.train_aabb.lo) / diag;
                    pos = vol.train_aabb.lo + wp * diag;
                    dt = unwarp_dt(warp_dt(calc_dt(lt.x, vol.ss)));
                } else {
                    raw = net_out[sc.x + j - ru];
                    pos = vol.train_aabb.lo + mk(c[0], c[1], c[2]) * diag;
                    dt = unwarp_dt(c[3]);
                }
                last_raw = raw;
                const float T = 1.f - rgba.w;
                const float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x & 0xffffu));
                const float g = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x >> 16));
                const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y & 0xffffu));
                const float s = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y >> 16));
                const float alpha = 1.f - sng_expf(-sng_expf(s) * dt);
                float weight = alpha * T;
                f3 rgb = mk(logistic(r), logistic(g), logistic(b));
                if (mode.ngp && mode.glow_mode) glow_term(mode.glow_mode, mode.glow_y_cutoff, pos, cam.c3, rgb, weight);
                if (mode.ngp) {   // composite_kernel_nerf render modes (testbed_nerf.cu:709-723)
                    if (mode.render_mode == 2) {   // network_to_density_derivative (Exponential) x the density gradient
                        const float dd = sng_expf(fminf(fmaxf(s, -15.0f), 15.0f));
                        rgb = normalize(-dd * mk(c[0], c[1], c[2]));
                    } else if (mode.render_mode == 3) rgb = (pos - 0.5f) / 2.0f + 0.5f;
                    else if (mode.render_mode == 10) rgb = mk(c[0], c[1], c[2]);
                    else if (mode.render_mode == 4) rgb = splat(dot(cam.c2, pos - mk(ot.x, ot.y, ot.z)) * mode.depth_scale);
                    else if (mode.render_mode == 0) rgb = splat(alpha);
                }
                rgba.x += rgb.x * weight;
                rgba.y += rgb.y * weight;
                rgba.z += rgb.z * weight;
                rgba.w += weight;
                if (mode.ngp) {   // depth of the max-weight sample (738-742)
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
            const f3 dir = mk(di.x, di.y, di.z);
            if (!mode.ngp) ot.w = depth / dot(cam.c2, dir);   // payload.t reset (576); trace keeps generate's t
            if (j < n_steps) { hit = !last && rgba.w > 0.001f; death_step = j + i_step; }
            else survive = !last;
        }
        const uint32_t own_idx = __float_as_uint(di.w);
        const uint32_t slot = block_append<THREADS / 64>(&ctrl->n_alive[p ^ 1], survive ? 1u : 0u, &ctrl->n_hit, hit,
                                           sched.global ? &ctrl->n_owned[p ^ 1] : nullptr, survive && own_idx >= sched.own_lo && own_idx < sched.own_hi,
                                           sh_app, lane);
        if (survive) {
            out.o_t[slot] = ot;
            out.d_idx[slot] = di;
            out.rgba[slot] = rgba;
            out.depth[slot] = depth;
            if (mode.ngp) out.mw[slot] = mw;
            else { out.lt[slot] = make_float2(lt.y, 0.0f); out.lo[slot] = last_raw; }
        }
        if (hit && mode.ngp) {
            // shade_kernel_nerf (1788-1828), gbuffer_hard_edges = false, train_in_linear_colors = false
            const uint32_t idx = __float_as_uint(di.w);
            float4 tmp = rgba;
            if (mode.render_mode == 6) { const float col = (float)death_step / 128; tmp = make_float4(col, col, col, 1.0f); }
            if (mode.render_mode == 1) { tmp.x = srgb_to_linear(tmp.x); tmp.y = srgb_to_linear(tmp.y); tmp.z = srgb_to_linear(tmp.z); }
            float4 fb = frame_rgba[idx];
            fb = make_float4(tmp.x + fb.x * (1.0f - tmp.w), tmp.y + fb.y * (1.0f - tmp.w), tmp.z + fb.z * (1.0f - tmp.w), tmp.w + fb.w * (1.0f - tmp.w));
            frame_rgba[idx] = fb;
            if (tmp.w > 0.2f) frame_depth[idx] = depth;
        } else if (hit) {
            const uint32_t idx = __float_as_uint(di.w);
            const f3 dir = mk(di.x, di.y, di.z);
            const f3 orig = cam.c3 + dir * ot.w;
            float4 fb = frame_rgba[idx];
            const float ta = rgba.w;
            const float r = srgb_to_linear(rgba.x), g = srgb_to_linear(rgba.y), b = srgb_to_linear(rgba.z);
            fb = make_float4(r + fb.x * (1.0f - ta), g + fb.y * (1.0f - ta), b + fb.z * (1.0f - ta), ta + fb.w * (1.0f - ta));
            frame_rgba[idx] = fb;
            positions[3 * idx + 0] = orig.x; positions[3 * idx + 1] = orig.y; positions[3 * idx + 2] = orig.z;
            if (ta > 0.2f) frame_depth[idx] = depth;
        }
    }
}

// ---------------------------------------------------------------------------
// Speculative tail rounds (SpecArgs, sng_internal.h)
// ---------------------------------------------------------------------------
// Once n_alive * 8 <= target, every later iteration of trace_alt / trace takes exactly 8 steps
// (testbed_nerf.cu:2189-2190).  A ray that survives an iteration starts the next one at
// t = depth(last sample) / dot(fwd, dir) (composite_kernel_nerf_alt:574; trace keeps generate's t,
// 836), and generate_next_nerf_network_inputs advances from there through occupancy alone (821-835):
// the positions of a ray's next K iterations do not depend on any network output.  Only the
// termination test (A > 1 - min_transmittance, 561) and the end of the march (cnt < n_steps, 567) do.
//   spec_generate : each lane marches its ray K iterations ahead (K * 8 samples, the t reset applied
//                   between iterations with the compositor's float expressions), writes every sample's t
//                   to tbuf and the samples that are not an iteration's cached boundary sample as
//                   NerfCoordinates for ONE whole-GPU network launch;
//   network       : nerf_network_kernel over the round's samples;
//   spec_composite: replays the K iterations in order with composite_kernel's arithmetic, stops the ray
//                   where the wavefront would (extract / shade, or the MARCH_ITER drop) and appends the
//                   survivors with their boundary-sample cache.  Samples past a ray's end are discarded.
// K = clamp(budget / (8 n_alive), 1, kmax) from the device alive count bounds the discarded work.

// composite_kernel's per-sample step (476-565 / 577-742) on a sample at march distance ts
__device__ __forceinline__ bool spec_composite_sample(const Volume& vol, const CamDev& cam, const TraceMode& mode, f3 o, f3 d, f3 diag, float ts, uint2 raw,
                                                      float4& rgba, float& depth, float& mw) {
    const f3 wp = ((o + d * ts) - vol.train_aabb.lo) / diag;   // generate_kernel's coordinate
    const f3 pos = vol.train_aabb.lo + wp * diag;
    const float dt = unwarp_dt(warp_dt(calc_dt(ts, vol.ss)));
    const float T = 1.f - rgba.w;
    const float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x & 0xffffu));
    const float g = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x >> 16));
    const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y & 0xffffu));
    const float s = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y >> 16));
    const float alpha = 1.f - sng_expf(-sng_expf(s) * dt);
    const float weight = alpha * T;
    f3 rgb = mk(logistic(r), logistic(g), logistic(b));
    if (mode.ngp) {
        if (mode.render_mode == 3) rgb = (pos - 0.5f) / 2.0f + 0.5f;
        else if (mode.render_mode == 4) rgb = splat(dot(cam.c2, pos - o) * mode.depth_scale);
        else if (mode.render_mode == 0) rgb = splat(alpha);
    }
    rgba.x += rgb.x * weight;
    rgba.y += rgb.y * weight;
    rgba.z += rgb.z * weight;
    rgba.w += weight;
    if (mode.ngp) {
        if (weight > mw) { mw = weight; depth = dot(cam.c2, pos - cam.c3); }
    } else {
        depth = dot(cam.c2, pos - cam.c3);
    }
    if (rgba.w > (1.0f - vol.min_transmittance)) {
        const float aa = rgba.w;
        rgba.x /= aa; rgba.y /= aa; rgba.z /= aa; rgba.w /= aa;
        return true;
    }
    return false;
}

// Per-ray look-ahead (SpecArgs::k_policy): iterations a ray is marched ahead in a round, from the opacity it has
// reached -- about the 90th percentile of the iterations rays of that opacity still live (lego, C2 / C3 after
// the head: A < 0.05 -> 5, ..., A >= 0.95 -> 1; tools/tail_diag.py), so fewer samples past a ray's end are
// evaluated.  Any choice is exact: a ray that outlives its look-ahead continues in the next round.
__device__ __forceinline__ uint32_t spec_k_of(float A) {
    return A < 0.05f ? 5u : A < 0.2f ? 4u : A < 0.5f ? 3u : A < 0.8f ? 3u : A < 0.95f ? 2u : 1u;
}

// BRICK: the occupancy bricks are staged in LDS (dynamic shared memory) and the march loop makes no global
// load, so its per-sample t stores to tbuf are fire-and-forget (no load waits behind them).  Without the
// bricks (too many for the LDS budget) the loop reads the linear occupancy through a register word cache.
template <bool LIN, bool BRICK, int THREADS = 256>
__global__ __launch_bounds__(THREADS) void spec_generate_kernel(SpecArgs a) {
    extern __shared__ uint32_t occ_lds[];
    __shared__ uint32_t sh_app[3 * (THREADS / 64) + 1];
    MarchCtrl* ctrl = a.ctrl;
    if (!ctrl->spec_ok) return;   // not a tail (tail_prepare): touch nothing
    const int p = a.p;
    const uint32_t n_alive = ctrl->n_alive[p];
    const uint32_t istep0 = ctrl->i_step[p];
    const uint32_t base_k = ctrl->spec_base_k, base_istep = ctrl->spec_base_istep;
    const bool kk_in = ctrl->spec_kk_valid[p] != 0u;   // per-ray iteration indices (after a round), else all at base_k
    uint32_t K = 0;   // the round's look-ahead bound; a ray's own may be smaller (k_policy, MARCH_ITER)
    // i_step[p] after a round is its largest look-ahead's (istep0 + 8 K); rays that looked ahead less are behind it.
    // Every survivor of a round is below MARCH_ITER (its last iteration was not the `last` one), so with per-ray
    // indices the round runs whatever i_step[p] says, and each ray's own `left` bounds its look-ahead.
    if (n_alive > 0 && (kk_in || istep0 < MARCH_ITER)) {
        K = a.budget / (MAX_STEPS_BETWEEN_COMPACTION * n_alive);
        K = K < 1u ? 1u : (K > a.kmax ? a.kmax : K);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctrl->spec_K[p] = K;
        ctrl->spec_k0[p] = ctrl->n_iter;
        ctrl->n_alive[p ^ 1] = 0;
        ctrl->i_step[p ^ 1] = istep0 + MAX_STEPS_BETWEEN_COMPACTION * K;
        ctrl->spec_kk_valid[p ^ 1] = 1u;   // the compositor writes each survivor's next iteration index
    }
    if (K == 0 || blockIdx.x * THREADS >= n_alive) return;
    const Volume& vol = a.vol;
    if constexpr (BRICK) stage_occ_brick(occ_lds, vol.occ_brick, vol.occ_brick_words);
    const int lane = threadIdx.x & 63;
    const f3 wdiag = vol.train_aabb.hi - vol.train_aabb.lo;
    const f3 rwdiag = mk(recip_rn(wdiag.x), recip_rn(wdiag.y), recip_rn(wdiag.z));
    const StepSpace cone = LIN ? step_space(0.0f) : vol.ss;
    const float qnan = __int_as_float(0x7fc00000);
    for (uint32_t blk = blockIdx.x * THREADS; blk < n_alive; blk += gridDim.x * THREADS) {
        const uint32_t i = blk + threadIdx.x;
        uint32_t tot = 0, nnet = 0, n_it = 0, cnt_last = 0, rbits = 0;
        f3 o = splat(0.0f), d = splat(1.0f);
        if (i < n_alive) {
            const float4 ot = a.in.o_t[i], di = a.in.d_idx[i];
            o = mk(ot.x, ot.y, ot.z);
            d = mk(di.x, di.y, di.z);
            // this ray's iteration, trace_alt step counter and look-ahead
            const uint32_t k_i = kk_in ? a.in.kk[i] : base_k;
            const uint32_t istep_i = base_istep + MAX_STEPS_BETWEEN_COMPACTION * (k_i - base_k);
            const uint32_t left = istep_i < MARCH_ITER ? (MARCH_ITER - istep_i + MAX_STEPS_BETWEEN_COMPACTION - 1) / MAX_STEPS_BETWEEN_COMPACTION : 1u;
            uint32_t K_i = K < left ? K : left;
            // the ray's own end in the last frame, when it is still ahead: look exactly that far; otherwise the
            // opacity policy.  Any K is exact (the round's replay stops where the wavefront would).
            const uint32_t h = (a.hint && a.hint_read) ? (uint32_t)a.hint[__float_as_uint(di.w)] : 0u;   // relative to the tail's first iteration
            if (h != 0u && h - 1u >= k_i - base_k) K_i = min(K_i, h - (k_i - base_k));
            else if (a.k_policy) K_i = min(K_i, spec_k_of(a.in.rgba[i].w));
            const f3 idir = inv(d);
            const float dfw = dot(a.cam.c2, d);
            const float rdfw = recip_rn(dfw);   // x / dfw as div_by(x, dfw, rdfw): the IEEE quotient (Markstein), fewer ops
            float t = ot.w;
            float prev = a.mode.ngp ? qnan : a.in.lt[i].x;   // the previous iteration's last sample
            OccCache oc;
            float* tb = a.tbuf + i;
            const size_t tstride = n_alive;
            // ONE flattened loop over all K iterations: each trip is one DDA step or one sample, and an
            // iteration's end (8 samples, or the march leaving the volume) is handled inside the trip, so a
            // wave runs max(total trips of its lanes) trips, not the sum over iterations of each one's max
            uint32_t cnt = 0, it = 0;
            float first = qnan, tl = 0.0f;
            const f3 hs = half_sign(d);
            bool going = true;
            // the t reset only moves t back to the last sample, so one bound serves the whole round
            float t_last = 3.0e38f;
            if constexpr (LIN && BRICK) t_last = path_last_occupied_t(o, d, idir, fminf(t, prev == prev ? prev : t), occ_lds);
#pragma unroll 1
            while (going) {
                bool sample = false, stop = false;   // stop: this iteration's march ends with cnt < 8
                if constexpr (LIN && BRICK) {
                    // branch-free trip: both successors formed, the occupancy bit selects (lanes of a wave
                    // diverge between DDA steps and samples on nearly every trip)
                    const f3 pos = o + d * t;   // render_aabb_to_local is the identity (launch_spec_generate)
                    const bool inside = (t < MAX_DEPTH) & (t <= t_last) & aabb_contains_nb(vol.render_aabb, pos);
                    stop = !inside;
                    sample = inside & occupied_brick_nb(pos, occ_lds);
                    const float t_dda = dda_step_linear(t, pos, idir, hs);
                    if (!stop && !sample) t = t_dda;
                } else if constexpr (LIN) {
                    const f3 pos = o + d * t;
                    if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) {
                        stop = true;
                    } else {
                        if (occupied_linear_c(pos, vol.occ_linear, oc)) sample = true;
                        else t = dda_step_linear(t, pos, idir, hs);
                    }
                } else {
                    if (occ_step(t, cone, o, d, idir, 0, vol.max_mip, vol)) {
                        if (t >= MAX_DEPTH) stop = true;
                        else sample = true;
                    }
                }
                if (sample) {
                    *tb = t;
                    tb += tstride;
                    if (cnt == 0) first = t;
                    tl = t;
                    t += LIN ? calc_dt(t, 0.0f) : calc_dt(t, cone);
                    ++cnt;
                }
                if (stop || cnt == MAX_STEPS_BETWEEN_COMPACTION) {   // the iteration's samples are complete
                    const uint32_t ru = (!a.mode.ngp && cnt > 0 && first == prev) ? 1u : 0u;
                    rbits |= ru << it;
                    tot += cnt;
                    nnet += cnt - ru;
                    ++n_it;
                    cnt_last = cnt;
                    if (cnt < MAX_STEPS_BETWEEN_COMPACTION || it + 1 == K_i) {
                        going = false;   // the ray ends in this iteration, or the round's look-ahead does
                    } else {
                        prev = tl;
                        if (!a.mode.ngp) {   // the compositor's t reset (574) on the iteration's last sample
                            const f3 q = (o + d * tl) - vol.train_aabb.lo;
                            const f3 wp = mk(div_by(q.x, wdiag.x, rwdiag.x), div_by(q.y, wdiag.y, rwdiag.y), div_by(q.z, wdiag.z, rwdiag.z));
                            const f3 pos = vol.train_aabb.lo + wp * wdiag;
                            t = div_by(dot(a.cam.c2, pos - a.cam.c3), dfw, rdfw);
                        }
                        ++it;
                        cnt = 0;
                        first = qnan;
                    }
                }
            }
            // trace keeps generate's t (836): the survivors' next start
            if (a.mode.ngp && n_it == K_i && cnt_last == MAX_STEPS_BETWEEN_COMPACTION) reinterpret_cast<float*>(a.in.o_t + i)[3] = t;
        }
        const uint32_t base = block_append<THREADS / 64>(&ctrl->n_samples[p], nnet, nullptr, false, nullptr, false, sh_app, lane);
        if (i < n_alive) {
            a.samp[i] = make_uint2(base, n_it | (cnt_last << 5) | (rbits << 9));
            const f3 wd = (d + 1.0f) * 0.5f;
            uint32_t q = base;
            // the iteration's t's read back together, then its NerfCoordinates written
#pragma unroll 1
            for (uint32_t s0 = 0; s0 < tot; s0 += MAX_STEPS_BETWEEN_COMPACTION) {
                float tv[MAX_STEPS_BETWEEN_COMPACTION];
#pragma unroll
                for (uint32_t j = 0; j < MAX_STEPS_BETWEEN_COMPACTION; ++j)
                    if (s0 + j < tot) tv[j] = a.tbuf[(size_t)(s0 + j) * n_alive + i];
                const uint32_t j0 = ((rbits >> (s0 >> 3)) & 1u) ? 1u : 0u;   // cached boundary sample: no evaluation
#pragma unroll
                for (uint32_t j = 0; j < MAX_STEPS_BETWEEN_COMPACTION; ++j) {
                    if (j < j0 || s0 + j >= tot) continue;
                    const float ts = tv[j];
                    const f3 wp = ((o + d * ts) - vol.train_aabb.lo) / wdiag;
                    float* c = a.coords + (size_t)q * 7;
                    c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(calc_dt(ts, cone)); c[4] = wd.x; c[5] = wd.y; c[6] = wd.z;
                    ++q;
                }
            }
        }
    }
}

// composite_kernel's per-sample activations (nerf_device.cuh:204-264, testbed_nerf.cu:545-556) of one network
// sample, from its NerfCoordinate (warped position, warped dt) and raw fp16 output: {logistic rgb, alpha}
// and its depth dot(fwd, pos - cam).  The float expressions of spec_composite_sample, so the same bits.
__device__ __forceinline__ float4 spec_activate(const Volume& vol, const CamDev& cam, f3 wp, float wdt, uint2 raw, float& depth) {
    const f3 diag = vol.train_aabb.hi - vol.train_aabb.lo;
    const f3 pos = vol.train_aabb.lo + wp * diag;
    const float dt = unwarp_dt(wdt);
    const float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x & 0xffffu));
    const float g = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x >> 16));
    const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y & 0xffffu));
    const float sg = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y >> 16));
    depth = dot(cam.c2, pos - cam.c3);
    return make_float4(logistic(r), logistic(g), logistic(b), 1.f - sng_expf(-sng_expf(sg) * dt));
}

// Sample-parallel half of the compositor: one thread per network sample of the round forms its activations,
// so the per-ray compositing chain (spec_composite) is only the front-to-back accumulation.
__global__ __launch_bounds__(256) void spec_prepare_kernel(SpecArgs a) {
    const int p = a.p;
    if (!a.ctrl->spec_ok || a.ctrl->spec_K[p] == 0) return;
    const uint32_t n = a.ctrl->n_samples[p];
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < n; s += gridDim.x * 256) {
        const float* c = a.coords + (size_t)s * 7;
        float depth;
        a.pre[s] = spec_activate(a.vol, a.cam, mk(c[0], c[1], c[2]), c[3], a.net_out[s], depth);
        a.pre_depth[s] = depth;
    }
}

template <int THREADS = 256>
__global__ __launch_bounds__(THREADS) void spec_composite_kernel(SpecArgs a) {
    __shared__ uint32_t hist_alive[64], hist_samples[64];
    __shared__ uint32_t blk_hit, blk_iter;
    __shared__ unsigned long long blk_samples, blk_reused;
    __shared__ uint32_t sh_app[3 * (THREADS / 64) + 1];
    MarchCtrl* ctrl = a.ctrl;
    if (!ctrl->spec_ok) return;
    const int p = a.p;
    const uint32_t n_alive = ctrl->n_alive[p];
    const uint32_t K = ctrl->spec_K[p];
    const uint32_t base_k = ctrl->spec_base_k, base_istep = ctrl->spec_base_istep;
    const bool kk_in = ctrl->spec_kk_valid[p] != 0u;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (K) {
            ctrl->net_samples += ctrl->n_samples[p];
            ctrl->spec_evals += ctrl->n_samples[p];
        }
        if (a.round < 4) ctrl->spec_round_samples[a.round] = K ? ctrl->n_samples[p] : 0u;
        ctrl->n_samples[p ^ 1] = 0;
        ctrl->n_reused[p ^ 1] = 0;
    }
    if (K == 0) return;
    if (threadIdx.x < 64) { hist_alive[threadIdx.x] = 0; hist_samples[threadIdx.x] = 0; }
    if (threadIdx.x == 0) { blk_hit = 0; blk_iter = 0; blk_samples = 0; blk_reused = 0; }
    __syncthreads();
    const Volume& vol = a.vol;
    const CamDev& cam = a.cam;
    const TraceMode& mode = a.mode;
    const int lane = threadIdx.x & 63;
    const f3 diag = vol.train_aabb.hi - vol.train_aabb.lo;
    uint32_t my_hits = 0, my_iter = 0;
    unsigned long long my_samples = 0, my_reused = 0;
    for (uint32_t blk = blockIdx.x * THREADS; blk < n_alive; blk += gridDim.x * THREADS) {
        const uint32_t i = blk + threadIdx.x;
        bool survive = false, hit = false;
        float4 rgba = make_float4(0, 0, 0, 0), ot = rgba, di = rgba;
        float depth = 0.0f, mw = 0.0f, lt = 0.0f;
        uint2 lraw = make_uint2(0u, 0u);
        uint32_t death_step = 0, kk_next = 0, k_end = 0, live_in = 0, live_out = 0;
        bool live = false;
        if (i < n_alive) {
            rgba = a.in.rgba[i];
            depth = a.in.depth[i];
            ot = a.in.o_t[i];
            di = a.in.d_idx[i];
            if (mode.ngp) mw = a.in.mw[i];
            else { lt = a.in.lt[i].x; lraw = a.in.lo[i]; }
            const f3 o = mk(ot.x, ot.y, ot.z), d = mk(di.x, di.y, di.z);
            const uint2 sc = a.samp[i];
            const uint32_t n_it = sc.y & 31u, cnt_last = (sc.y >> 5) & 15u, rbits = sc.y >> 9;
            const uint32_t k0 = kk_in ? a.in.kk[i] : base_k;   // this ray's iteration and step counter at the round's start
            const uint32_t istep0 = base_istep + MAX_STEPS_BETWEEN_COMPACTION * (k0 - base_k);
            kk_next = k0 + n_it;
            uint32_t ob = sc.x, s = 0;
            bool ended = false;
            if (a.pre) {
                // activations precomputed per sample (spec_prepare).  The chain only accumulates; the next
                // iteration's {rgb, alpha} are loaded while this one composites.  A reused boundary sample is the
                // previous iteration's last one (same t, coordinate and output), so it reuses that activation;
                // the round's first is activated from the ray's cache.  The payload's depth sample is resolved
                // once at the ray's end of round (its t reset and extraction need nothing earlier).
                float4 pv[MAX_STEPS_BETWEEN_COMPACTION], pn[MAX_STEPS_BETWEEN_COMPACTION];
                float4 carry = make_float4(0, 0, 0, 0);
                float d_carry = 0.0f;
                if (rbits & 1u) {   // round start: the ray's cached boundary sample (lt, lraw)
                    const f3 wp = ((o + d * lt) - vol.train_aabb.lo) / diag;   // generate_kernel's coordinate of t = lt
                    carry = spec_activate(vol, cam, wp, warp_dt(calc_dt(lt, vol.ss)), lraw, d_carry);
                }
                auto load_it = [&](uint32_t it_, uint32_t ob_, float4* dst) {
                    const uint32_t cnt_ = it_ + 1 == n_it ? cnt_last : MAX_STEPS_BETWEEN_COMPACTION;
                    const uint32_t ru_ = (rbits >> it_) & 1u;
#pragma unroll
                    for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q)
                        if (q < cnt_ && !(ru_ && q == 0)) dst[q] = a.pre[ob_ + q - ru_];
                };
                if (n_it) load_it(0, ob, pv);
                int64_t dsel = -2;   // the depth sample: -2 none, -1 the round's cached boundary sample, else its network index
                uint32_t last_net = 0;
                for (uint32_t it = 0; it < n_it && !ended; ++it) {
                    const uint32_t cnt = it + 1 == n_it ? cnt_last : MAX_STEPS_BETWEEN_COMPACTION;
                    const uint32_t ru = (rbits >> it) & 1u;
                    const uint32_t istep = istep0 + MAX_STEPS_BETWEEN_COMPACTION * it;
                    const bool last = istep + MAX_STEPS_BETWEEN_COMPACTION >= MARCH_ITER;
                    if (k0 + it < 64) {
                        atomicAdd(&hist_alive[k0 + it], 1u);
                        if (cnt) atomicAdd(&hist_samples[k0 + it], cnt);
                    }
                    my_samples += cnt;
                    my_reused += ru;
                    my_iter = max(my_iter, k0 + it + 1);
                    const uint32_t ob0 = ob;
                    ob += cnt - ru;
                    if (it + 1 < n_it) load_it(it + 1, ob, pn);   // in flight while this iteration composites
                    if (ru) pv[0] = carry;
                    uint32_t j = 0;
#pragma unroll
                    for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) {
                        if (q >= cnt) break;
                        j = q + 1;
                        const float4 v = pv[q];
                        const float T = 1.f - rgba.w;
                        const float weight = v.w * T;
                        rgba.x += v.x * weight;
                        rgba.y += v.y * weight;
                        rgba.z += v.z * weight;
                        rgba.w += weight;
                        const int64_t sel = (ru && q == 0) ? (it == 0 ? -1 : (int64_t)last_net) : (int64_t)(ob0 + q - ru);
                        if (mode.ngp) {
                            if (weight > mw) { mw = weight; dsel = sel; }
                        } else {
                            dsel = sel;
                        }
                        if (rgba.w > (1.0f - vol.min_transmittance)) {
                            const float aa = rgba.w;
                            rgba.x /= aa; rgba.y /= aa; rgba.z /= aa; rgba.w /= aa;
                            j = q;
                            break;
                        }
                    }
                    if (j < MAX_STEPS_BETWEEN_COMPACTION) {
                        hit = !last && rgba.w > 0.001f;
                        death_step = j + istep;
                        ended = true;
                        k_end = k0 + it;
                    } else if (last) {
                        ended = true;
                        k_end = k0 + it;
                    } else {
                        carry = pv[MAX_STEPS_BETWEEN_COMPACTION - 1];   // the next iteration's boundary sample
                        last_net = ob - 1;                              // its network index (8 samples, at most 1 reused)
                        s += cnt;
#pragma unroll
                        for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) pv[q] = pn[q];
                    }
                }
                if (!ended && n_it) {   // survivor: the boundary cache of the next round (the last sample, evaluated)
                    lt = a.tbuf[(size_t)(s - 1) * n_alive + i];
                    lraw = a.net_out[last_net];
                }
                if (dsel >= 0) depth = a.pre_depth[dsel];
                else if (dsel == -1) depth = d_carry;
                if (!mode.ngp && n_it) ot.w = depth / dot(cam.c2, d);   // payload.t reset (574)
            }
            for (uint32_t it = 0; it < n_it && !ended && !a.pre; ++it) {
                const uint32_t cnt = it + 1 == n_it ? cnt_last : MAX_STEPS_BETWEEN_COMPACTION;
                const uint32_t ru = (rbits >> it) & 1u;
                const uint32_t istep = istep0 + MAX_STEPS_BETWEEN_COMPACTION * it;
                const bool last = istep + MAX_STEPS_BETWEEN_COMPACTION >= MARCH_ITER;
                if (k0 + it < 64) {
                    atomicAdd(&hist_alive[k0 + it], 1u);
                    if (cnt) atomicAdd(&hist_samples[k0 + it], cnt);
                }
                my_samples += cnt;
                my_reused += ru;
                my_iter = max(my_iter, k0 + it + 1);
                // the iteration's t's and outputs are loaded together, ahead of the compositing chain
                float tv[MAX_STEPS_BETWEEN_COMPACTION];
                uint2 rv[MAX_STEPS_BETWEEN_COMPACTION];
#pragma unroll
                for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) {
                    if (q < cnt) {
                        tv[q] = a.tbuf[(size_t)(s + q) * n_alive + i];
                        rv[q] = (ru && q == 0) ? lraw : a.net_out[ob + q - ru];
                    }
                }
                ob += cnt - ru;
                uint32_t j = 0;
                uint2 last_raw = lraw;
#pragma unroll
                for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) {
                    if (q >= cnt) break;
                    last_raw = rv[q];
                    j = q + 1;
                    if (spec_composite_sample(vol, cam, mode, o, d, diag, tv[q], rv[q], rgba, depth, mw)) { j = q; break; }
                }
                if (!mode.ngp) ot.w = depth / dot(cam.c2, d);   // payload.t reset (574)
                if (j < MAX_STEPS_BETWEEN_COMPACTION) {
                    hit = !last && rgba.w > 0.001f;
                    death_step = j + istep;
                    ended = true;
                    k_end = k0 + it;
                } else if (last) {
                    ended = true;
                    k_end = k0 + it;
                } else {
                    lt = tv[MAX_STEPS_BETWEEN_COMPACTION - 1];   // the boundary-sample cache of the next iteration
                    lraw = last_raw;
                    s += cnt;
                }
            }
            survive = !ended;
            if (ended && a.hint) a.hint[__float_as_uint(di.w)] = (uint8_t)min(k_end - base_k + 1u, 255u);
            if (n_it) {   // alive at iterations k0 .. (ended ? k_end : kk_next - 1): reference slots (tail_slots_kernel)
                live_in = k0;
                live_out = ended ? k_end + 1u : kk_next;
                live = true;
            }
        }
        wave_add_keyed(ctrl->tail_live, live_in, 1, live);
        wave_add_keyed(ctrl->tail_live, live_out, -1, live);
        const uint32_t slot = block_append<THREADS / 64>(&ctrl->n_alive[p ^ 1], survive ? 1u : 0u, nullptr, false, nullptr, false, sh_app, lane);
        if (survive) {
            a.out.o_t[slot] = ot;
            a.out.d_idx[slot] = di;
            a.out.rgba[slot] = rgba;
            a.out.depth[slot] = depth;
            if (mode.ngp) a.out.mw[slot] = mw;
            else { a.out.lt[slot] = make_float2(lt, 0.0f); a.out.lo[slot] = lraw; }
            a.out.kk[slot] = kk_next;
        }
        if (hit) {
            ++my_hits;
            const uint32_t idx = __float_as_uint(di.w);
            if (mode.ngp) {   // shade_kernel_nerf (1788-1828)
                float4 tmp = rgba;
                if (mode.render_mode == 6) { const float col = (float)death_step / 128; tmp = make_float4(col, col, col, 1.0f); }
                if (mode.render_mode == 1) { tmp.x = srgb_to_linear(tmp.x); tmp.y = srgb_to_linear(tmp.y); tmp.z = srgb_to_linear(tmp.z); }
                float4 fb = a.frame_rgba[idx];
                fb = make_float4(tmp.x + fb.x * (1.0f - tmp.w), tmp.y + fb.y * (1.0f - tmp.w), tmp.z + fb.z * (1.0f - tmp.w), tmp.w + fb.w * (1.0f - tmp.w));
                a.frame_rgba[idx] = fb;
                if (tmp.w > 0.2f) a.frame_depth[idx] = depth;
            } else {          // extract_from_payload (1578-1612)
                const f3 dir = mk(di.x, di.y, di.z);
                const f3 orig = cam.c3 + dir * ot.w;
                float4 fb = a.frame_rgba[idx];
                const float ta = rgba.w;
                const float r = srgb_to_linear(rgba.x), g = srgb_to_linear(rgba.y), b = srgb_to_linear(rgba.z);
                fb = make_float4(r + fb.x * (1.0f - ta), g + fb.y * (1.0f - ta), b + fb.z * (1.0f - ta), ta + fb.w * (1.0f - ta));
                a.frame_rgba[idx] = fb;
                a.positions[3 * idx + 0] = orig.x; a.positions[3 * idx + 1] = orig.y; a.positions[3 * idx + 2] = orig.z;
                if (ta > 0.2f) a.frame_depth[idx] = depth;
            }
        }
    }
    // statistics (the wavefront's per-iteration histograms, hits, composited / reused samples)
    atomicAdd(&blk_hit, my_hits);
    atomicMax(&blk_iter, my_iter);
    atomicAdd(&blk_samples, my_samples);
    if (my_reused) atomicAdd(&blk_reused, my_reused);
    __syncthreads();
    if (threadIdx.x < 64) {
        if (hist_alive[threadIdx.x]) atomicAdd(&ctrl->alive_hist[threadIdx.x], hist_alive[threadIdx.x]);
        if (hist_samples[threadIdx.x]) atomicAdd(&ctrl->samples_hist[threadIdx.x], hist_samples[threadIdx.x]);
    }
    if (threadIdx.x == 0) {
        if (blk_hit) atomicAdd(&ctrl->n_hit, blk_hit);
        if (blk_iter) atomicMax(&ctrl->n_iter, blk_iter);
        if (blk_samples) {
            atomicAdd(&ctrl->total_samples, blk_samples);
            atomicAdd(&ctrl->spec_exec, blk_samples - blk_reused);
        }
        if (blk_reused) atomicAdd(&ctrl->reused_samples, blk_reused);
    }
}

// the tail's per-iteration statistics: iterations from n_iter on take 8 steps each
__global__ void tail_prepare_kernel(MarchCtrl* ctrl, uint32_t* work, int p, uint32_t target, int global_sched) {
    // the tail is exact only if every remaining iteration takes 8 steps: n_alive * 8 <= target now (it only shrinks)
    const uint32_t n_sched = global_sched ? ctrl->sched_alive[p] : ctrl->n_alive[p];
    const bool ok = (uint64_t)n_sched * MAX_STEPS_BETWEEN_COMPACTION <= target;
    __syncthreads();
    if (threadIdx.x == 0) {
        ctrl->spec_ok = ok ? 1u : 0u;
        if (!ok) { ctrl->n_samples[0] = 0u; ctrl->n_samples[1] = 0u; }   // the queued network launches find nothing
    }
    if (!ok) return;
    if (threadIdx.x < 64 && threadIdx.x >= ctrl->n_iter) ctrl->steps_hist[threadIdx.x] = MAX_STEPS_BETWEEN_COMPACTION;
    if (threadIdx.x == 0) {
        if (work) *work = 0;
        ctrl->spec_base_k = ctrl->n_iter;        // the tail's first iteration ...
        ctrl->spec_base_istep = ctrl->i_step[p]; // ... and its step counter
        ctrl->spec_kk_valid[0] = 0u;
        ctrl->spec_kk_valid[1] = 0u;
    }
}

// ---------------------------------------------------------------------------
// Multi-step speculative rounds (MsrArgs, sng_internal.h)
// ---------------------------------------------------------------------------
// The round's shape from the frame-wide alive count at its first iteration: S_0 = that iteration's steps
// (only 2..7: 1 is the one-step regime's, 8 the tail's) and K iterations before MARCH_ITER, each with its own
// step count Sv[m].  K == 0: the round is a no-op (every msr kernel returns without touching state).
// The last frame's schedule (MarchCtrl::sched_hint, frame-wide, so every rank of a banded frame forms the same
// round) predicts the steps of the iterations ahead: when it agrees with S_0 the round follows it -- across step
// changes when `span` (MsrArgs), else while it stays S_0 -- in 2..7, up to kmax iterations and budget / n_sched
// samples per ray;
// otherwise the round assumes S_0 throughout (no hint: as far as the budget allows; a hint that disagrees: the
// schedule is near a change, 2 iterations).  Any guess is exact: msr_schedule commits the iterations whose
// frame-wide count takes the guessed steps, and the rest are marched again.
__device__ __forceinline__ uint32_t msr_shape(const MarchCtrl* c, uint32_t n_sched, uint32_t istep0, uint32_t target, uint32_t budget,
                                              uint32_t kmax, int span, uint8_t* Sv) {
    if (n_sched == 0 || istep0 >= MARCH_ITER) return 0u;
    const uint32_t s = steps_for(n_sched, target);
    if (s < 2 || s >= MAX_STEPS_BETWEEN_COMPACTION) return 0u;
    const uint32_t per_ray = budget / n_sched;   // samples per ray the round may generate
    const uint32_t k0 = c->n_iter;
    const uint32_t h = k0 < TAIL_LIVE_CAP ? c->sched_hint[k0] : 0u;
    uint32_t K = 0;
    if (h == s) {
        uint32_t istep = istep0, tot = 0;
        while (K < kmax && istep < MARCH_ITER) {
            const uint32_t sm = K == 0 ? s : (k0 + K < TAIL_LIVE_CAP ? (uint32_t)c->sched_hint[k0 + K] : 0u);
            if (sm < 2 || sm >= MAX_STEPS_BETWEEN_COMPACTION || (K > 0 && tot + sm > per_ray) || (!span && sm != s)) break;
            Sv[K++] = (uint8_t)sm;
            tot += sm;
            istep += sm;
        }
        return K;
    }
    uint32_t k = per_ray / s;
    k = k < 1u ? 1u : (k > kmax ? kmax : k);
    const uint32_t left = (MARCH_ITER - istep0 + s - 1) / s;   // iterations whose i is still < MARCH_ITER
    k = k < left ? k : left;
    if (h != 0u) k = k < 2u ? k : 2u;
    for (uint32_t m = 0; m < k; ++m) Sv[m] = (uint8_t)s;
    return k;
}

// composite_kernel's opacity step on one sample (spec_composite_sample's alpha and accumulation of .w)
__device__ __forceinline__ float msr_alpha(const Volume& vol, float ts, uint2 raw) {
    const float dt = unwarp_dt(warp_dt(calc_dt(ts, vol.ss)));
    const float s = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y >> 16));
    return 1.f - sng_expf(-sng_expf(s) * dt);
}

// every alive ray marched K iterations of S samples ahead (spec_generate_kernel's flattened loop and t reset
// with S in place of 8, one look-ahead for every ray)
template <bool LIN, int THREADS = 256>
__global__ __launch_bounds__(THREADS) void msr_generate_kernel(MsrArgs a) {
    __shared__ uint32_t sh_app[3 * (THREADS / 64) + 1];
    __shared__ uint8_t sh_S[MSR_KMAX];
    MarchCtrl* ctrl = a.ctrl;
    const int p = a.p;
    const uint32_t n_alive = ctrl->n_alive[p];
    const uint32_t n_sched = a.sched.global ? ctrl->sched_alive[p] : n_alive;
    if (threadIdx.x == 0) {
        uint8_t Sv[MSR_KMAX];
        const uint32_t K = msr_shape(ctrl, n_sched, ctrl->i_step[p], a.target, a.budget, a.kmax, a.span, Sv);
        sh_app[3 * (THREADS / 64)] = K;
        for (uint32_t m = 0; m < MSR_KMAX; ++m) sh_S[m] = m < K ? Sv[m] : (uint8_t)0;
        if (blockIdx.x == 0) {
            ctrl->msr_S[p] = K ? Sv[0] : 0u;
            ctrl->msr_K[p] = K;
            for (uint32_t m = 0; m < MSR_KMAX; ++m) ctrl->msr_Sv[p][m] = sh_S[m];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 4 * MSR_KMAX) a.hist[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t K = sh_app[3 * (THREADS / 64)];
    __syncthreads();   // sh_app is block_append's scratch below
    if (K == 0 || blockIdx.x * THREADS >= n_alive) return;
    const Volume& vol = a.vol;
    const int lane = threadIdx.x & 63;
    const f3 wdiag = vol.train_aabb.hi - vol.train_aabb.lo;
    const f3 rwdiag = mk(recip_rn(wdiag.x), recip_rn(wdiag.y), recip_rn(wdiag.z));
    const StepSpace cone = LIN ? step_space(0.0f) : vol.ss;
    const float qnan = __int_as_float(0x7fc00000);
    for (uint32_t blk = blockIdx.x * THREADS; blk < n_alive; blk += gridDim.x * THREADS) {
        const uint32_t i = blk + threadIdx.x;
        uint32_t tot = 0, nnet = 0, n_it = 0, cnt_last = 0, rbits = 0;
        f3 o = splat(0.0f), d = splat(1.0f);
        if (i < n_alive) {
            const float4 ot = a.in.o_t[i], di = a.in.d_idx[i];
            o = mk(ot.x, ot.y, ot.z);
            d = mk(di.x, di.y, di.z);
            const f3 idir = inv(d);
            const float dfw = dot(a.cam.c2, d);
            const float rdfw = recip_rn(dfw);
            float t = ot.w;
            float prev = a.in.lt[i].x;   // the previous iteration's last sample (the boundary-sample cache)
            OccCache oc;
            float* tb = a.tbuf + i;
            uint32_t cnt = 0, it = 0, S = sh_S[0];   // S: the current iteration's steps
            float first = qnan, tl = 0.0f;
            const f3 hs = half_sign(d);
            bool going = true;
#pragma unroll 1
            while (going) {
                bool sample = false, stop = false;
                if constexpr (LIN) {
                    const f3 pos = o + d * t;
                    if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) {
                        stop = true;
                    } else {
                        if (occupied_linear_c(pos, vol.occ_linear, oc)) sample = true;
                        else t = dda_step_linear(t, pos, idir, hs);
                    }
                } else {
                    if (occ_step(t, cone, o, d, idir, 0, vol.max_mip, vol)) {
                        if (t >= MAX_DEPTH) stop = true;
                        else sample = true;
                    }
                }
                if (sample) {
                    *tb = t;
                    tb += n_alive;
                    if (cnt == 0) first = t;
                    tl = t;
                    t += LIN ? calc_dt(t, 0.0f) : calc_dt(t, cone);
                    ++cnt;
                }
                if (stop || cnt == S) {   // the iteration's samples are complete
                    const uint32_t ru = (cnt > 0 && first == prev) ? 1u : 0u;
                    rbits |= ru << it;
                    tot += cnt;
                    nnet += cnt - ru;
                    ++n_it;
                    cnt_last = cnt;
                    if (cnt < S || it + 1 == K) {
                        going = false;   // the ray ends in this iteration, or the round's look-ahead does
                    } else {
                        prev = tl;       // the compositor's t reset (574) on the iteration's last sample
                        const f3 q = (o + d * tl) - vol.train_aabb.lo;
                        const f3 wp = mk(div_by(q.x, wdiag.x, rwdiag.x), div_by(q.y, wdiag.y, rwdiag.y), div_by(q.z, wdiag.z, rwdiag.z));
                        const f3 pos = vol.train_aabb.lo + wp * wdiag;
                        t = div_by(dot(a.cam.c2, pos - a.cam.c3), dfw, rdfw);
                        ++it;
                        S = sh_S[it];
                        cnt = 0;
                        first = qnan;
                    }
                }
            }
        }
        const uint32_t base = block_append<THREADS / 64>(&ctrl->n_samples[p], nnet, nullptr, false, nullptr, false, sh_app, lane);
        if (i < n_alive) {
            a.samp[i] = make_uint2(base, n_it | (cnt_last << 5) | (rbits << 9));
            const f3 wd = (d + 1.0f) * 0.5f;
            uint32_t q = base, jx = 0, itx = 0, S = sh_S[0];
#pragma unroll 1
            for (uint32_t x = 0; x < tot; ++x) {
                if (!(jx == 0 && ((rbits >> itx) & 1u))) {   // a cached boundary sample needs no evaluation
                    const float ts = a.tbuf[(size_t)x * n_alive + i];
                    const f3 wp = ((o + d * ts) - vol.train_aabb.lo) / wdiag;
                    float* c = a.coords + (size_t)q * 7;
                    c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(LIN ? calc_dt(ts, 0.0f) : calc_dt(ts, cone)); c[4] = wd.x; c[5] = wd.y; c[6] = wd.z;
                    ++q;
                }
                if (++jx == S) { jx = 0; ++itx; S = sh_S[itx < MSR_KMAX ? itx : 0]; }
            }
        }
    }
}

// spec_composite_sample for trace_alt with the sample's alpha given (msr_count formed it with the same expressions)
__device__ __forceinline__ bool msr_composite_sample(const Volume& vol, const CamDev& cam, f3 o, f3 d, f3 diag, float ts, uint2 raw, float alpha,
                                                     float4& rgba, float& depth) {
    const f3 wp = ((o + d * ts) - vol.train_aabb.lo) / diag;   // generate_kernel's coordinate
    const f3 pos = vol.train_aabb.lo + wp * diag;
    const float T = 1.f - rgba.w;
    const float r = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x & 0xffffu));
    const float g = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.x >> 16));
    const float b = (float)__builtin_bit_cast(_Float16, (uint16_t)(raw.y & 0xffffu));
    const float weight = alpha * T;
    rgba.x += logistic(r) * weight;
    rgba.y += logistic(g) * weight;
    rgba.z += logistic(b) * weight;
    rgba.w += weight;
    depth = dot(cam.c2, pos - cam.c3);
    if (rgba.w > (1.0f - vol.min_transmittance)) {
        const float aa = rgba.w;
        rgba.x /= aa; rgba.y /= aa; rgba.z /= aa; rgba.w /= aa;
        return true;
    }
    return false;
}

// the iteration each ray ends in (opacity, the march's end, or MARCH_ITER's drop), from the opacity chain alone
template <int THREADS = 256>
__global__ __launch_bounds__(THREADS) void msr_count_kernel(MsrArgs a) {
    __shared__ uint32_t h[4 * MSR_KMAX];
    MarchCtrl* ctrl = a.ctrl;
    const int p = a.p;
    __shared__ uint8_t sh_S[MSR_KMAX];
    const uint32_t K = ctrl->msr_K[p];
    if (K == 0) return;
    const uint32_t istep0 = ctrl->i_step[p], n_alive = ctrl->n_alive[p];
    if (threadIdx.x < 4 * MSR_KMAX) h[threadIdx.x] = 0u;
    if (threadIdx.x < MSR_KMAX) sh_S[threadIdx.x] = ctrl->msr_Sv[p][threadIdx.x];
    __syncthreads();
    const Volume& vol = a.vol;
    const float opaque = 1.0f - vol.min_transmittance;
    for (uint32_t i = blockIdx.x * THREADS + threadIdx.x; i < n_alive; i += gridDim.x * THREADS) {
        float w = a.in.rgba[i].w;
        uint2 lraw = a.in.lo[i];
        const uint32_t idx = __float_as_uint(a.in.d_idx[i].w);
        const bool own = !a.sched.global || (idx >= a.sched.own_lo && idx < a.sched.own_hi);
        const uint2 sc = a.samp[i];
        const uint32_t n_it = sc.y & 31u, cnt_last = (sc.y >> 5) & 15u, rbits = sc.y >> 9;
        uint32_t ob = sc.x, s = 0, e = K, istep = istep0;
        for (uint32_t it = 0; it < n_it; ++it) {
            const uint32_t S = sh_S[it];
            const uint32_t cnt = it + 1 == n_it ? cnt_last : S;
            const uint32_t ru = (rbits >> it) & 1u;
            atomicAdd(&h[2 * MSR_KMAX + it], cnt);
            if (ru) atomicAdd(&h[3 * MSR_KMAX + it], 1u);
            istep += S;
            const bool last = istep >= MARCH_ITER;
            // the iteration's t's and outputs loaded together, ahead of the opacity chain
            float tv[MAX_STEPS_BETWEEN_COMPACTION];
            uint2 rv[MAX_STEPS_BETWEEN_COMPACTION];
            uint2 rlast = lraw;   // rv[cnt - 1], selected with static indices (a dynamic one puts the arrays in scratch)
#pragma unroll
            for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) {
                if (q < cnt) {
                    tv[q] = a.tbuf[(size_t)(s + q) * n_alive + i];
                    rv[q] = (ru && q == 0) ? lraw : a.net_out[ob + q - ru];
                    if (q + 1 == cnt) rlast = rv[q];
                }
            }
            uint32_t j = cnt;
#pragma unroll
            for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) {
                if (q >= cnt) break;
                const float T = 1.f - w;
                const float al = msr_alpha(vol, tv[q], rv[q]);
                a.abuf[(size_t)(s + q) * n_alive + i] = al;   // msr_commit composites every sample this loop reaches
                w += al * T;
                if (w > opaque) { j = q; break; }
            }
            if (j < S || last) { e = it; break; }
            lraw = rlast;   // the next iteration's boundary sample (S >= 2: never the reused one)
            ob += cnt - ru;
            s += cnt;
        }
        if (e < K) {
            atomicAdd(&h[e], 1u);
            if (own) atomicAdd(&h[MSR_KMAX + e], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < 4 * MSR_KMAX && h[threadIdx.x]) atomicAdd(&a.hist[threadIdx.x], h[threadIdx.x]);
}

// J = the first relative iteration whose frame-wide alive count is 0 or does not take S steps (or whose i
// reaches MARCH_ITER); the per-iteration statistics of the committed ones as generate / composite record them
__global__ void msr_schedule_kernel(MsrArgs a) {
    MarchCtrl* c = a.ctrl;
    const int p = a.p;
    const uint32_t K = c->msr_K[p];
    if (K == 0 || threadIdx.x != 0) return;
    const uint32_t istep0 = c->i_step[p], k = c->n_iter;
    uint32_t istep = istep0;
    const uint32_t* deaths_l = a.hist;
    const uint32_t* deaths_s = a.sched.global ? a.hist + MSR_KMAX : a.hist;
    uint32_t alive_s = a.sched.global ? c->sched_alive[p] : c->n_alive[p], alive_l = c->n_alive[p];
    uint32_t J = K;
    unsigned long long slots = 0, samp = 0, reused = 0;
    for (uint32_t m = 0; m < K; ++m) {
        const uint32_t S = c->msr_Sv[p][m];
        if (alive_s == 0 || steps_for(alive_s, a.target) != S || istep >= MARCH_ITER) { J = m; break; }
        istep += S;
        const uint32_t sm = a.hist[2 * MSR_KMAX + m], rm = a.hist[3 * MSR_KMAX + m];
        slots += ((unsigned long long)alive_l * S + 255ull) / 256ull * 256ull;
        samp += sm;
        reused += rm;
        if (k + m < 64) { c->alive_hist[k + m] = alive_l; c->steps_hist[k + m] = S; c->samples_hist[k + m] = sm; }
        if (c->log && k + m < MARCH_LOG_CAP) { c->log[3 * (k + m)] = alive_l; c->log[3 * (k + m) + 1] = S; c->log[3 * (k + m) + 2] = sm; }
        if (k + m < TAIL_LIVE_CAP) c->sched_hint[k + m] = (uint8_t)S;
        alive_s -= deaths_s[m];
        alive_l -= deaths_l[m];
    }
    if (J < K && k + J < TAIL_LIVE_CAP && alive_s > 0) c->sched_hint[k + J] = (uint8_t)steps_for(alive_s, a.target);
    c->msr_J = J;
    c->ref_slots += slots;
    c->total_samples += samp;
    c->reused_samples += reused;
    c->net_samples += c->n_samples[p];
    c->msr_evals += c->n_samples[p];
    c->msr_exec += samp - reused;
    c->n_iter = k + J;
    c->i_step[p ^ 1] = istep;   // istep0 + the committed iterations' steps
    c->n_alive[p ^ 1] = 0;
    c->n_owned[p ^ 1] = 0;
    c->n_samples[p ^ 1] = 0;
    c->n_reused[p ^ 1] = 0;
}

// the first J iterations replayed with composite_kernel's arithmetic: rays ending before k + J are extracted
// (extract_from_payload), the others appended to buffer p ^ 1 with their state and boundary-sample cache at k + J
template <int THREADS = 256>
__global__ __launch_bounds__(THREADS) void msr_commit_kernel(MsrArgs a) {
    __shared__ uint32_t sh_app[3 * (THREADS / 64) + 1];
    MarchCtrl* ctrl = a.ctrl;
    const int p = a.p;
    __shared__ uint8_t sh_S[MSR_KMAX];
    const uint32_t K = ctrl->msr_K[p];
    if (K == 0) return;
    const uint32_t J = ctrl->msr_J, istep0 = ctrl->i_step[p], n_alive = ctrl->n_alive[p];
    if (threadIdx.x < MSR_KMAX) sh_S[threadIdx.x] = ctrl->msr_Sv[p][threadIdx.x];
    __syncthreads();
    const Volume& vol = a.vol;
    const CamDev& cam = a.cam;
    const TraceMode mode{0, 1, 1.0f, 0, 0.0f};   // trace_alt
    const int lane = threadIdx.x & 63;
    const f3 diag = vol.train_aabb.hi - vol.train_aabb.lo;
    uint32_t my_hits = 0;
    for (uint32_t blk = blockIdx.x * THREADS; blk < n_alive; blk += gridDim.x * THREADS) {
        const uint32_t i = blk + threadIdx.x;
        bool survive = false, hit = false;
        float4 rgba = make_float4(0, 0, 0, 0), ot = rgba, di = rgba;
        float depth = 0.0f, mw = 0.0f, lt = 0.0f;
        uint2 lraw = make_uint2(0u, 0u);
        if (i < n_alive) {
            rgba = a.in.rgba[i];
            depth = a.in.depth[i];
            ot = a.in.o_t[i];
            di = a.in.d_idx[i];
            lt = a.in.lt[i].x;
            lraw = a.in.lo[i];
            const f3 o = mk(ot.x, ot.y, ot.z), d = mk(di.x, di.y, di.z);
            const uint2 sc = a.samp[i];
            const uint32_t n_it = sc.y & 31u, cnt_last = (sc.y >> 5) & 15u, rbits = sc.y >> 9;
            uint32_t ob = sc.x, s = 0, istep = istep0;
            bool ended = false;
            const uint32_t n_run = n_it < J ? n_it : J;
            for (uint32_t it = 0; it < n_run && !ended; ++it) {
                const uint32_t S = sh_S[it];
                const uint32_t cnt = it + 1 == n_it ? cnt_last : S;
                const uint32_t ru = (rbits >> it) & 1u;
                istep += S;
                const bool last = istep >= MARCH_ITER;
                float tv[MAX_STEPS_BETWEEN_COMPACTION], av[MAX_STEPS_BETWEEN_COMPACTION];
                uint2 rv[MAX_STEPS_BETWEEN_COMPACTION];
#pragma unroll
                for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) {
                    if (q < cnt) {
                        tv[q] = a.tbuf[(size_t)(s + q) * n_alive + i];
                        av[q] = a.abuf[(size_t)(s + q) * n_alive + i];
                        rv[q] = (ru && q == 0) ? lraw : a.net_out[ob + q - ru];
                    }
                }
                uint32_t j = cnt;
                float tq = 0.0f;
                uint2 rq = lraw;
#pragma unroll
                for (uint32_t q = 0; q < MAX_STEPS_BETWEEN_COMPACTION; ++q) {
                    if (q >= cnt) break;
                    tq = tv[q];
                    rq = rv[q];
                    if (msr_composite_sample(vol, cam, o, d, diag, tq, rq, av[q], rgba, depth)) { j = q; break; }
                }
                ot.w = depth / dot(cam.c2, d);   // payload.t reset (574)
                if (j < S) {
                    hit = !last && rgba.w > 0.001f;
                    ended = true;
                } else if (last) {
                    ended = true;
                } else {
                    lt = tq;     // the boundary-sample cache of the next iteration: this one's last sample
                    lraw = rq;
                    ob += cnt - ru;
                    s += cnt;
                }
            }
            survive = !ended;
        }
        const uint32_t own_idx = __float_as_uint(di.w);
        const uint32_t slot = block_append<THREADS / 64>(&ctrl->n_alive[p ^ 1], survive ? 1u : 0u, a.sched.global ? &ctrl->n_owned[p ^ 1] : nullptr,
                                                         survive && own_idx >= a.sched.own_lo && own_idx < a.sched.own_hi, nullptr, false, sh_app, lane);
        if (survive) {
            a.out.o_t[slot] = ot;
            a.out.d_idx[slot] = di;
            a.out.rgba[slot] = rgba;
            a.out.depth[slot] = depth;
            a.out.lt[slot] = make_float2(lt, 0.0f);
            a.out.lo[slot] = lraw;
        }
        if (hit) {   // extract_from_payload (1578-1612)
            ++my_hits;
            const uint32_t idx = own_idx;
            const f3 dir = mk(di.x, di.y, di.z);
            const f3 orig = cam.c3 + dir * ot.w;
            float4 fb = a.frame_rgba[idx];
            const float ta = rgba.w;
            const float r = srgb_to_linear(rgba.x), g = srgb_to_linear(rgba.y), b = srgb_to_linear(rgba.z);
            fb = make_float4(r + fb.x * (1.0f - ta), g + fb.y * (1.0f - ta), b + fb.z * (1.0f - ta), ta + fb.w * (1.0f - ta));
            a.frame_rgba[idx] = fb;
            a.positions[3 * idx + 0] = orig.x; a.positions[3 * idx + 1] = orig.y; a.positions[3 * idx + 2] = orig.z;
            if (ta > 0.2f) a.frame_depth[idx] = depth;
        }
    }
    if (my_hits) atomicAdd(&ctrl->n_hit, my_hits);
}

// write_normals_to_buffer (1523-1576) for rows [row0,row1)
__global__ __launch_bounds__(256) void normals_kernel(int W, int H, int row0, int row1, const float* __restrict__ positions,
                                                      float* __restrict__ normals) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = (uint32_t)(row1 - row0) * (uint32_t)W;
    if (t >= n) return;
    const int x = (int)(t % (uint32_t)W), y = row0 + (int)(t / (uint32_t)W);
    const size_t idx = (size_t)x + (size_t)W * y;
    const f3 pos = mk(positions[3 * idx], positions[3 * idx + 1], positions[3 * idx + 2]);
    const int OX[9] = {1, 0, -1, 0, 2, 0, -2, 0, 1};
    const int OY[9] = {0, 1, 0, -1, 0, 2, 0, -2, 0};
    float factor = 0.0f;
    f3 N = splat(0.0f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int tx = x + OX[k + 1], ty = y + OY[k + 1], bx = x + OX[k], by = y + OY[k];
        if (tx >= W || tx < 0 || ty >= H || ty < 0 || bx >= W || bx < 0 || by >= H || by < 0) continue;
        const float* pt = positions + 3 * ((size_t)ty * W + tx);
        const float* pb = positions + 3 * ((size_t)by * W + bx);
        const f3 T = mk(pt[0], pt[1], pt[2]) - pos;
        const f3 B = mk(pb[0], pb[1], pb[2]) - pos;
        N = N + normalize(cross(normalize(T), B));
        factor += 1.0f;
    }
    N = factor == 0.0f ? N : N / factor;
    const f3 nn = normalize(N);
    normals[3 * idx] = nn.x; normals[3 * idx + 1] = nn.y; normals[3 * idx + 2] = nn.z;
}

// ---------------------------------------------------------------------------
// density grid -> bitfield (update_density_grid_mean_and_bitfield, 3212-3229)
// ---------------------------------------------------------------------------
__global__ void half_to_float_kernel(const uint16_t* __restrict__ in, float* __restrict__ out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (float)__builtin_bit_cast(_Float16, in[i]);
}
// deterministic mean: per-block double partial sums of fmaxf(v,0)/N, then one block sums them
__global__ __launch_bounds__(256) void mean_partial_kernel(const float* __restrict__ grid, uint32_t n, double* __restrict__ partial) {
    __shared__ double sm[256];
    double acc = 0.0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) acc += (double)(fmaxf(grid[i], 0.f) / (float)n);
    sm[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) sm[threadIdx.x] += sm[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = sm[0];
}
// the partials staged in LDS by coalesced loads, then one lane sums them in index order (the same double sequence;
// one lane reading global memory in turn took ~70 us)
__global__ __launch_bounds__(256) void mean_final_kernel(const double* __restrict__ partial, int n_part, float* __restrict__ mean) {
    __shared__ double sm[1024];
    for (int i = threadIdx.x; i < n_part && i < 1024; i += blockDim.x) sm[i] = partial[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
#pragma unroll 16
        for (int i = 0; i < n_part; ++i) s += sm[i];
        *mean = (float)s;
    }
}
__global__ void grid_to_bitfield_kernel(uint32_t n_elements, uint32_t n_nonzero, const float* __restrict__ grid, uint8_t* __restrict__ bf,
                                        const float* __restrict__ mean) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_elements) return;
    if (i >= n_nonzero) { bf[i] = 0; return; }
    const float thresh = fminf(MIN_OPTICAL_THICKNESS, *mean);
    uint8_t bits = 0;
#pragma unroll
    for (uint8_t j = 0; j < 8; ++j) bits |= grid[i * 8 + j] > thresh ? ((uint8_t)1 << j) : 0;
    bf[i] = bits;
}
__global__ void bitfield_max_pool_kernel(uint32_t n_elements, const uint8_t* __restrict__ prev, uint8_t* __restrict__ next) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_elements) return;
    uint8_t bits = 0;
#pragma unroll
    for (uint8_t j = 0; j < 8; ++j) bits |= prev[i * 8 + j] > 0 ? ((uint8_t)1 << j) : 0;
    const uint32_t x = morton3D_invert(i >> 0) + GRID_SIZE / 8;
    const uint32_t y = morton3D_invert(i >> 1) + GRID_SIZE / 8;
    const uint32_t z = morton3D_invert(i >> 2) + GRID_SIZE / 8;
    // each (x,y,z) is written by exactly one thread of this launch
    next[morton3D(x, y, z)] |= bits;
}

// every cascade's occupancy as x-fastest bit rows: word ((mip*128 + z)*128 + y)*4 + x/32, bit x%32 == Morton bit
// (x,y,z) of that mip.  Same bits, cheaper address math for the marchers (mip 0 alone: the linear marcher).
__global__ void bitfield_linear_kernel(const uint8_t* __restrict__ bf, uint32_t* __restrict__ occ) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= GRID_CELLS / 32 * N_CASCADES) return;
    const uint32_t mip = g / (GRID_CELLS / 32), w = g % (GRID_CELLS / 32);
    const uint32_t z = w / (GRID_SIZE * GRID_SIZE / 32), y = (w / (GRID_SIZE / 32)) % GRID_SIZE, x0 = (w % (GRID_SIZE / 32)) * 32;
    const uint8_t* b8 = bf + (size_t)mip * (GRID_CELLS / 8);
    uint32_t bits = 0;
    for (uint32_t b = 0; b < 32; ++b) {
        const uint32_t m = morton3D(x0 + b, y, z);
        bits |= (uint32_t)((b8[m >> 3] >> (m & 7)) & 1u) << b;
    }
    occ[g] = bits;
}

// OccBrick blob (sng_math.h) from the linear mip-0 occupancy: flags, one-block scan, fill
__global__ void occ_brick_flag_kernel(const uint32_t* __restrict__ occ, uint32_t* __restrict__ flags) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= 4096) return;
    const uint32_t bz = b >> 8, by = (b >> 4) & 15u, bx = b & 15u;
    uint32_t any = 0;
    for (uint32_t z = 0; z < 8; ++z)
        for (uint32_t y = 0; y < 8; ++y) any |= (occ[((bz * 8 + z) * GRID_SIZE + by * 8 + y) * (GRID_SIZE / 32) + (bx >> 2)] >> ((bx & 3u) * 8u)) & 0xffu;
    flags[b] = any ? 1u : 0u;
}
__global__ __launch_bounds__(1024) void occ_brick_scan_kernel(const uint32_t* __restrict__ flags, uint32_t* __restrict__ blob, uint32_t* __restrict__ n_out) {
    __shared__ uint32_t ps[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t f0 = flags[4 * t], f1 = flags[4 * t + 1], f2 = flags[4 * t + 2], f3v = flags[4 * t + 3];
    const uint32_t sum = f0 + f1 + f2 + f3v;
    ps[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? ps[t - off] : 0u;
        __syncthreads();
        ps[t] += v;
        __syncthreads();
    }
    uint32_t slot = ps[t] - sum;
    uint16_t* tab = reinterpret_cast<uint16_t*>(blob + OCC_BRICK_TAB);
    const uint32_t fl[4] = {f0, f1, f2, f3v};
    for (int k = 0; k < 4; ++k) {
        tab[4 * t + k] = fl[k] ? (uint16_t)slot : (uint16_t)0xffffu;
        slot += fl[k];
    }
    if (t == 1023) *n_out = ps[t];
}
__global__ void occ_brick_fill_kernel(const uint32_t* __restrict__ occ, uint32_t* __restrict__ blob) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= 4096 * 16) return;
    const uint32_t b = g >> 4, k = g & 15u;
    const uint32_t slot = reinterpret_cast<const uint16_t*>(blob + OCC_BRICK_TAB)[b];
    if (slot == 0xffffu) return;
    const uint32_t bz = b >> 8, by = (b >> 4) & 15u, bx = b & 15u;
    const uint32_t z = bz * 8 + (k >> 1), y0 = by * 8 + (k & 1u) * 4;
    uint32_t w = 0;
    for (uint32_t yy = 0; yy < 4; ++yy) w |= ((occ[(z * GRID_SIZE + y0 + yy) * (GRID_SIZE / 32) + (bx >> 2)] >> ((bx & 3u) * 8u)) & 0xffu) << (yy * 8u);
    blob[OCC_BRICK_HDR_WORDS + slot * 16u + k] = w;
}

__global__ void ctrl_init_kernel(MarchCtrl* c, int32_t* tail_live, uint8_t* sched_hint, uint32_t* log) {
    if (threadIdx.x < 64) {   // the fused tail kernel accumulates into the histograms
        c->alive_hist[threadIdx.x] = 0; c->steps_hist[threadIdx.x] = 0; c->samples_hist[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        c->n_alive[0] = 0; c->n_alive[1] = 0;
        c->n_owned[0] = 0; c->n_owned[1] = 0;
        c->sched_alive[0] = 0; c->sched_alive[1] = 0;
        c->n_samples[0] = 0; c->n_samples[1] = 0;
        c->n_reused[0] = 0; c->n_reused[1] = 0;
        c->i_step[0] = 1; c->i_step[1] = 1;   // trace_alt: uint32_t i = 1 (2163)
        c->n_hit = 0; c->n_iter = 0;
        c->total_samples = 0; c->net_samples = 0; c->ref_slots = 0; c->reused_samples = 0;
        c->spec_K[0] = 0; c->spec_K[1] = 0; c->spec_k0[0] = 0; c->spec_k0[1] = 0;
        c->spec_evals = 0; c->spec_exec = 0;
        c->spec_base_k = 0; c->spec_base_istep = 1; c->spec_kk_valid[0] = 0; c->spec_kk_valid[1] = 0; c->spec_ok = 1;
        c->msr_S[0] = 0; c->msr_S[1] = 0; c->msr_K[0] = 0; c->msr_K[1] = 0; c->msr_J = 0; c->msr_evals = 0; c->msr_exec = 0;
        c->log = log;
        c->tail_live = tail_live;
        c->sched_hint = sched_hint;
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
void launch_ctrl_init(MarchCtrl* ctrl, int32_t* tail_live, uint8_t* sched_hint, hipStream_t s, uint32_t* log) {
    if (log) (void)hipMemsetAsync(log, 0, MARCH_LOG_CAP * 12, s);
    (void)hipMemsetAsync(tail_live, 0, TAIL_LIVE_CAP * 4, s);
    hipLaunchKernelGGL(ctrl_init_kernel, dim3(1), dim3(64), 0, s, ctrl, tail_live, sched_hint, log);
}
// alive(k) = prefix sum of tail_live; the reference's slots of a tail iteration: n_alive(k) * 8 padded to 256
__global__ __launch_bounds__(1024) void tail_slots_kernel(MarchCtrl* ctrl) {
    constexpr uint32_t CH = TAIL_LIVE_CAP / 1024;
    __shared__ int32_t ps[1024];
    __shared__ unsigned long long total;
    if (!ctrl->spec_ok) return;   // the tail did not run (tail_prepare)
    const uint32_t tid = threadIdx.x;
    const int32_t* live = ctrl->tail_live;
    int32_t sum = 0;
    for (uint32_t x = 0; x < CH; ++x) sum += live[tid * CH + x];
    ps[tid] = sum;
    if (tid == 0) total = 0;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const int32_t v = tid >= off ? ps[tid - off] : 0;
        __syncthreads();
        ps[tid] += v;
        __syncthreads();
    }
    int32_t alive = ps[tid] - sum;
    unsigned long long slots = 0;
    for (uint32_t x = 0; x < CH; ++x) {
        alive += live[tid * CH + x];
        slots += ((unsigned long long)(uint32_t)alive * MAX_STEPS_BETWEEN_COMPACTION + 255ull) / 256ull * 256ull;
    }
    if (slots) atomicAdd(&total, slots);
    __syncthreads();
    if (tid == 0) ctrl->ref_slots += total;
}
void launch_tail_slots(MarchCtrl* ctrl, hipStream_t s) { hipLaunchKernelGGL(tail_slots_kernel, dim3(1), dim3(1024), 0, s, ctrl); }
// ---------------------------------------------------------------------------
void launch_init_rays(const NerfFrameArgs& a, const RayBuf& out, MarchCtrl* ctrl, float4* fb, float* depth, float* pos, float* nrm,
                      uint32_t n_cus, hipStream_t s) {
    uint32_t n = (uint32_t)(a.row1 - a.row0) * (uint32_t)a.W;
    if (!n) return;
    const uint32_t blocks = (n + 255) / 256;
    if (a.vol.linear && a.vol.occ_brick_words && a.vol.to_local_identity && a.vol.bitfield)   // persistent: 3 LDS copies per CU
        hipLaunchKernelGGL(init_rays_kernel<true>, dim3(std::min(blocks, n_cus * 3u)), dim3(256), a.vol.occ_brick_words * 4, s, a, out, ctrl, fb, depth,
                           pos, nrm, n);
    else
        hipLaunchKernelGGL(init_rays_kernel<false>, dim3(blocks), dim3(256), 0, s, a, out, ctrl, fb, depth, pos, nrm, n);
}
void launch_generate(const Volume& v, const RayBuf& rays, MarchCtrl* ctrl, int p, uint32_t target, uint32_t iter, float* coords, uint2* samp,
                     uint32_t blocks, int store_t, int global_sched, hipStream_t s) {
    if (v.linear && v.occ_brick_words && v.to_local_identity)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(generate_kernel<true, 256, true>), dim3(blocks), dim3(256), v.occ_brick_words * 4, s, v, rays, ctrl, p, target, iter, coords,
                           samp, store_t, global_sched);
    else if (v.linear) hipLaunchKernelGGL(generate_kernel<true>, dim3(blocks), dim3(256), 0, s, v, rays, ctrl, p, target, iter, coords, samp, store_t, global_sched);
    else hipLaunchKernelGGL(generate_kernel<false>, dim3(blocks), dim3(256), 0, s, v, rays, ctrl, p, target, iter, coords, samp, store_t, global_sched);
}
void launch_composite(const Volume& v, const CamDev& cam, const TraceMode& mode, const Sched& sched, const RayBuf& in, const RayBuf& out, MarchCtrl* ctrl, int p,
                      uint32_t target, uint32_t iter, const float* coords, const uint2* samp, const uint2* net_out, float4* fb, float* depth, float* pos,
                      uint32_t blocks, hipStream_t s, bool wide) {
    // long one-step marches (no fused tail): 1024-thread workgroups, 4x fewer append atomics;
    // the short head of the hybrid schedule keeps 256 (more, smaller blocks beside the raytracer)
    if (wide) hipLaunchKernelGGL(composite_kernel<1024>, dim3(std::max(1u, blocks / 4u)), dim3(1024), 0, s, v, cam, mode, sched, in, out, ctrl, p, target, iter, coords, samp, net_out, fb, depth, pos);
    else hipLaunchKernelGGL(composite_kernel<256>, dim3(blocks), dim3(256), 0, s, v, cam, mode, sched, in, out, ctrl, p, target, iter, coords, samp, net_out, fb, depth, pos);
}
void launch_spec_generate(const SpecArgs& a, uint32_t blocks, hipStream_t s) {
    if (a.vol.linear && a.vol.occ_brick_words && a.vol.to_local_identity)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(spec_generate_kernel<true, true>), dim3(blocks), dim3(256), a.vol.occ_brick_words * 4, s, a);
    else if (a.vol.linear) hipLaunchKernelGGL(HIP_KERNEL_NAME(spec_generate_kernel<true, false>), dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(spec_generate_kernel<false, false>), dim3(blocks), dim3(256), 0, s, a);
}
void launch_spec_composite(const SpecArgs& a, uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(spec_composite_kernel<256>, dim3(blocks), dim3(256), 0, s, a);
}
void launch_msr_generate(const MsrArgs& a, uint32_t blocks, hipStream_t s) {
    if (a.vol.linear) hipLaunchKernelGGL(HIP_KERNEL_NAME(msr_generate_kernel<true>), dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(msr_generate_kernel<false>), dim3(blocks), dim3(256), 0, s, a);
}
void launch_msr_count(const MsrArgs& a, uint32_t blocks, hipStream_t s) { hipLaunchKernelGGL(msr_count_kernel<256>, dim3(blocks), dim3(256), 0, s, a); }
void launch_msr_schedule(const MsrArgs& a, hipStream_t s) { hipLaunchKernelGGL(msr_schedule_kernel, dim3(1), dim3(64), 0, s, a); }
void launch_msr_commit(const MsrArgs& a, uint32_t blocks, hipStream_t s) { hipLaunchKernelGGL(msr_commit_kernel<256>, dim3(blocks), dim3(256), 0, s, a); }
void launch_spec_prepare(const SpecArgs& a, uint32_t blocks, hipStream_t s) {
    hipLaunchKernelGGL(spec_prepare_kernel, dim3(blocks), dim3(256), 0, s, a);
}
void launch_tail_prepare(MarchCtrl* ctrl, uint32_t* work, int p, uint32_t target, int global_sched, hipStream_t s) {
    hipLaunchKernelGGL(tail_prepare_kernel, dim3(1), dim3(64), 0, s, ctrl, work, p, target, global_sched);
}
void launch_normals(int W, int H, int row0, int row1, const float* pos, float* nrm, hipStream_t s) {
    const uint32_t n = (uint32_t)(row1 - row0) * (uint32_t)W;
    if (!n) return;
    hipLaunchKernelGGL(normals_kernel, dim3((n + 255) / 256), dim3(256), 0, s, W, H, row0, row1, pos, nrm);
}
void launch_bitfield(const uint16_t* grid_f16, uint32_t max_cascade, float* grid_f32, double* partial, float* mean, uint8_t* bf, uint32_t* occ_linear,
                     hipStream_t s) {
    const uint32_t N = GRID_CELLS;
    const uint32_t n_cells = N * (max_cascade + 1);
    if (grid_f16) hipLaunchKernelGGL(half_to_float_kernel, dim3((n_cells + 255) / 256), dim3(256), 0, s, grid_f16, grid_f32, n_cells);   // else grid_f32 is given
    hipLaunchKernelGGL(mean_partial_kernel, dim3(1024), dim3(256), 0, s, grid_f32, N, partial);
    hipLaunchKernelGGL(mean_final_kernel, dim3(1), dim3(256), 0, s, partial, 1024, mean);
    const uint32_t n_el = N / 8 * N_CASCADES;
    hipLaunchKernelGGL(grid_to_bitfield_kernel, dim3((n_el + 255) / 256), dim3(256), 0, s, n_el, N / 8 * (max_cascade + 1), grid_f32, bf, mean);
    for (uint32_t level = 1; level < N_CASCADES; ++level)
        hipLaunchKernelGGL(bitfield_max_pool_kernel, dim3((N / 64 + 255) / 256), dim3(256), 0, s, N / 64, bf + (size_t)N / 8 * (level - 1),
                           bf + (size_t)N / 8 * level);
    hipLaunchKernelGGL(bitfield_linear_kernel, dim3(N / 32 * N_CASCADES / 256), dim3(256), 0, s, bf, occ_linear);
}
// dilated brick mask: bit b set when an occupied cell lies in brick b grown by one cell per side.  One
// thread per (brick, z row of the grown brick); the rows' flags OR into the mask word with an atomic.
__global__ void occ_brick_dilate_kernel(const uint32_t* __restrict__ occ, uint32_t* __restrict__ blob) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= 4096 * 10) return;
    const uint32_t b = g / 10, zr = g % 10;
    const int bz = (int)(b >> 8), by = (int)((b >> 4) & 15u), bx = (int)(b & 15u);
    const int z = bz * 8 - 1 + (int)zr;
    if (z < 0 || z > 127) return;
    const int x0 = max(0, bx * 8 - 1), x1 = min(127, bx * 8 + 8);
    bool any = false;
    for (int y = max(0, by * 8 - 1); y <= min(127, by * 8 + 8) && !any; ++y)
        for (int x = x0; x <= x1 && !any; ++x) any = (occ[((uint32_t)z * GRID_SIZE + (uint32_t)y) * (GRID_SIZE / 32) + ((uint32_t)x >> 5)] >> (x & 31)) & 1u;
    if (any) atomicOr(&blob[b >> 5], 1u << (b & 31u));
}
void launch_occ_brick(const uint32_t* occ_linear, uint32_t* flags, uint32_t* blob, uint32_t* n_bricks, hipStream_t s) {
    (void)hipMemsetAsync(blob, 0, 128 * 4, s);
    hipLaunchKernelGGL(occ_brick_dilate_kernel, dim3(4096 * 10 / 256), dim3(256), 0, s, occ_linear, blob);
    hipLaunchKernelGGL(occ_brick_flag_kernel, dim3(16), dim3(256), 0, s, occ_linear, flags);
    hipLaunchKernelGGL(occ_brick_scan_kernel, dim3(1), dim3(1024), 0, s, flags, blob, n_bricks);
    hipLaunchKernelGGL(occ_brick_fill_kernel, dim3(4096 * 16 / 256), dim3(256), 0, s, occ_linear, blob);
}

}  // namespace sng
