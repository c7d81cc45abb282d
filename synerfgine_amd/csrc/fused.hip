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
    const uint32_t i_step0 = a.ctrl->i_step[a.p];
    const uint32_t k0 = a.ctrl->n_iter;
    const f3 wdiag = vol.train_aabb.hi - vol.train_aabb.lo;
    const float cone = LIN ? 0.0f : vol.cone;
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
                        k = k0;
                        istep = i_step0;
                        has = true;
                    }
                }
            }
        }
        if (!__ballot(has)) break;

        // ---- generate: up to 8 samples (generate_next_nerf_network_inputs, testbed_nerf.cu:790-837)
        uint32_t cnt = 0;
        bool reuse = false;
        const uint32_t n_steps = MAX_STEPS_BETWEEN_COMPACTION;
        if (has) {
            const f3 idir = inv(d);
            if constexpr (LIN) {
                const f3 hs = half_sign(d);
                while (cnt < n_steps) {
                    const f3 pos = o + d * t;
                    if (t >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos))) break;
                    if (occupied_linear(pos, vol.occ_linear)) {
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
                for (; cnt < n_steps; ++cnt) {
                    t = advance_to_occupied(t, cone, o, d, idir, 0, vol.max_mip, vol);
                    if (t >= MAX_DEPTH) break;
                    ts_lds[wv][cnt][lane] = t;
                    t += calc_dt(t, cone);
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
            field_tile<F>(W, a.levels, grid, g, wp.x, wp.y, wp.z, wd.x, wd.y, wd.z, out, dens);
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

__global__ void fused_prepare_kernel(MarchCtrl* ctrl, uint32_t* work) {
    // iterations from n_iter on take 8 steps each (the fused kernel's precondition)
    if (threadIdx.x < 64 && threadIdx.x >= ctrl->n_iter) ctrl->steps_hist[threadIdx.x] = MAX_STEPS_BETWEEN_COMPACTION;
    if (threadIdx.x == 0) *work = 0;
}

void launch_nerf_fused(const FusedArgs& a, const NetworkDev& net, uint32_t n_rays_hint, uint32_t max_blocks, hipStream_t s) {
    hipLaunchKernelGGL(fused_prepare_kernel, dim3(1), dim3(64), 0, s, a.ctrl, a.work);
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
