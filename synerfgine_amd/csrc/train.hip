// train.hip -- online NeRF training (BASELINE config 5): one training step
// of Testbed::train_nerf (testbed_nerf.cu:3298-3530, train_nerf_step 3532-3780) on gfx950.
//
//   train_generate_kernel  generate_training_samples_nerf (838-998): random pixels, occupancy march
//   (network)              inference forward of every sample (nerf_network_kernel, layout [n][4])
//   train_loss_kernel      compute_loss_kernel_train_nerf (1000-1313): composite, Huber loss,
//                          dL/d(rgb, sigma) per sample, compaction of the samples that contribute
//   train_rollover_kernel  tcnn fill_rollover(_and_rescale): pad the compacted batch to its target size
//   train_field_kernel     NerfNetwork forward + backward (nerf_network.h:144-268) per 16-sample
//                          tile on MFMA: activations and pre-activation gradients go to a tiled HBM
//                          buffer, hash-grid gradients are scattered with f32 atomics
//   train_dw_kernel        the five weight gradients dW = delta x activation^T, K = samples, MFMA
//   train_adam_kernel      tcnn Ema(ExponentialDecay(Adam)) (base.json:5-22), fp32 master weights
//   density grid           update_density_grid_nerf (3121-3210): mark_untrained_density_grid,
//                          generate_grid_samples_nerf_nonuniform, splat max, ema_grid_samples_nerf
//
// tiny-cuda-nn (GridEncoding / FullyFusedMLP backward, Adam, EMA, pcg32) is unvendored; its
// published algorithms are restated.  MFMA operand layout of v_mfma_f32_16x16x16f16:
// A lane l = (row l%16, k 4(l/16)..+3), B lane l = (k 4(l/16)..+3, col l%16), D lane l = (rows
// 4(l/16)..+3, col l%16) -- so a layer's D fragment IS the next backward layer's B fragment.
#include <algorithm>

#include "nerf_field.h"
#include "train.h"

namespace sng {

typedef _Float16 h4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4v mfma16k16(h4v a, h4v b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0); }

// ---------------------------------------------------------------------------------------------
// generate_training_samples_nerf (testbed_nerf.cu:838-998), no error-map CDFs, no distortion map,
// no envmap, max_level_rand_training off; the dataset lens per image (train_ray)
// ---------------------------------------------------------------------------------------------
// One march per ray (the reference marches twice: once to count, once to write).  The sample distances of the first
// march go to tscr (sample-major [j][ray], so a wave's stores of one step are contiguous); once the ray's range of the
// batch is reserved, its NerfCoordinates are formed from them with the same expressions (pos = o + t dn, dt =
// calc_dt(t)), so the samples are the reference's bit for bit.  BRICK (unit-cube scenes): the occupancy lookups read
// the mip-0 bricks staged in LDS (occupied_brick_nb, the render marchers' exact form) instead of global memory.
// One 64-lane workgroup per 64 rays: a batch has only ~4K rays, so small workgroups spread them over the CUs.
// BRICK 0: bitfield / linear occupancy; 1: the bricks staged in LDS; 2: the bricks read from global memory (their count
// is not known on the host while training rebuilds them every few steps)
// LIN (compile time): the unit-cube linear specialisation (cone 0, one cascade); otherwise the cascaded march with the
// volume's StepSpace constants (the same float expressions as the cone forms, so the same bits, without their logs)
template <int BRICK, bool LIN>
__global__ __launch_bounds__(64) void train_generate_kernel(TrainStepArgs a, TrainImages im, TrainBatch b, Pcg32 rng0, float* __restrict__ tscr) {
    extern __shared__ uint32_t occ_lds[];
    if constexpr (BRICK == 1) stage_occ_brick(occ_lds, a.vol.occ_brick, a.vol.occ_brick_words);
    const uint32_t* const bricks = BRICK == 1 ? occ_lds : a.vol.occ_brick_g;
    // grid-stride over the device's ray count (the grid is sized by the host's estimate of it)
    const uint32_t n_rays = a.sched->n_rays, max_samples = a.sched->max_samples;
    for (uint32_t vb = blockIdx.x; vb * blockDim.x < n_rays; vb += gridDim.x) {
        Pcg32 rng = rng0;   // each grid-stride trip starts from the step's stream (the ray's offset is added below)
        const uint32_t i = vb * blockDim.x + threadIdx.x;
        const int lane = threadIdx.x & 63;
        // every lane stays to the wave's reservations below (wave_reserve); a lane without a ray marches nothing
        const bool in = i < n_rays;
        const uint32_t ii = in ? i : 0u;
        const uint32_t img = ((ii * im.n) / n_rays) % im.n;   // image_idx (nerf_device.cuh:578-597)
        rng.advance((uint64_t)ii * N_MAX_RANDOM_SAMPLES_PER_RAY);
        const f2 uv = train_image_pos(rng, im);
        const bool live = in && !(read_rgba(im, img, uv).x < 0.0f);   // masked pixel: no samples
        (void)rng.next_float();                                    // motionblur_time
        const TrainRay ray = train_ray(im, img, uv);
        const f3 dn = normalize(ray.d);
        const aabb box = a.vol.train_aabb;
        float tmin = fmaxf(aabb_entry(box, ray.o, dn), 0.0f);      // aabb.ray_intersect(...).x, clamped at 0
        const StepSpace& ss = a.vol.ss;
        const float startt = LIN ? advance_n_steps(tmin, 0.0f, rng.next_float()) : advance_n_steps(tmin, ss, rng.next_float());
        const f3 idir = inv(dn);
        uint32_t j = 0;
        float t = startt;
        f3 pos;
        // unit-cube scenes (cone 0, one cascade): the exact linear specialisation of the occupancy test and
        // of advance_to_next_voxel that the render marcher uses (sng_math.h, tests/test_host_fastpaths.py)
        static_assert(BRICK == 0 || LIN, "the brick forms are unit-cube only");
        const f3 hs = half_sign(dn);
        float* const ts = tscr + ii;
        OccCache oc;
        while (live && aabb_contains(box, pos = ray.o + t * dn) && j < NERF_STEPS) {
            const float dt = LIN ? calc_dt(t, 0.0f) : calc_dt(t, ss);
            bool occ;
            // the cached forms reload a word only when the position leaves the last one (~4.6 samples per cell): each trip
            // is a dependent load otherwise, and a batch has too few rays to hide that latency
            if constexpr (BRICK != 0) occ = occupied_brick_c(pos, bricks, oc);
            else if constexpr (LIN) occ = occupied_linear_c(pos, a.vol.occ_linear, oc);
            else occ = occupied_at(pos, a.vol.bitfield, mip_from_dt(dt, pos, a.vol.max_mip));
            // one trip is one sample or one DDA step, as a select: with an if / else the compiler nests a loop of DDA steps
            // inside the sample loop, and a wave then waits at every sample for its lanes' longest run of empty cells
            // (measured 3.4x slower)
            float t_skip;
            if constexpr (LIN) t_skip = dda_step_linear(t, pos, idir, hs);
            else t_skip = advance_to_next_voxel(t, ss, pos, dn, idir, mip_from_dt(dt, pos, a.vol.max_mip));
            if (occ) ts[(size_t)j * n_rays] = t;
            j += occ ? 1u : 0u;
            t = occ ? t + dt : t_skip;
        }
        if (a.debug && live) { b.loss[i] = (float)j; b.coords_c[2 * i] = tmin; b.coords_c[2 * i + 1] = startt; }
        const uint32_t numsteps = j;
        const uint32_t base = wave_reserve(&b.ctrl->numsteps_counter, numsteps, lane);
        const bool keep = numsteps > 0 && base + numsteps <= max_samples;
        const uint32_t ray_idx = wave_reserve(&b.ctrl->ray_counter, keep ? 1u : 0u, lane);
        if (!keep) continue;
        b.ray_indices[ray_idx] = i;
        b.rays[2 * ray_idx] = make_float4(ray.o.x, ray.o.y, ray.o.z, 0.0f);
        b.rays[2 * ray_idx + 1] = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.0f);
        b.numsteps[ray_idx] = make_uint2(numsteps, base);
        const f3 wd = (dn + 1.0f) * 0.5f;   // warp_direction
        const f3 diag = box.hi - box.lo;
        float* co = b.coords + (size_t)base * 7;
        for (uint32_t k = 0; k < numsteps; ++k) {
            const float tk = ts[(size_t)k * n_rays];
            const f3 p = ray.o + tk * dn;
            const f3 wp = (p - box.lo) / diag;   // warp_position = aabb.relative_pos
            float* c = co + (size_t)k * 7;
            c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(LIN ? calc_dt(tk, 0.0f) : calc_dt(tk, ss)); c[4] = wd.x; c[5] = wd.y; c[6] = wd.z;
        }
    }
}

// The same march with G lanes per ray (train_gen_lanes): each trip of the group speculates G steps of the current kind
// and tests their cells together.  In sample mode lane k takes k further samples from t (t += calc_dt(t), the serial
// chain's own float sequence, k times) and tests the cell at its position; the group keeps the samples before the
// first lane whose cell is empty (or that left the box / reached NERF_STEPS), and that lane's position takes the DDA
// step.  In DDA mode lane k takes k further DDA steps and the group continues from the first lane whose cell is
// occupied.  Every t is the one the serial march reaches, so the samples are the same; only the number of dependent
// trips drops (one trip per ~G samples in occupied stretches, where the longest rays spend most of their march).
template <bool LIN, int G>
__global__ __launch_bounds__(64) void train_generate_spec_kernel(TrainStepArgs a, TrainImages im, TrainBatch b, Pcg32 rng0, float* __restrict__ tscr) {
    const int lane = threadIdx.x & 63;
    const uint32_t gl = (uint32_t)lane % G, g0 = (uint32_t)lane - gl;
    const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << g0;
    const uint32_t n_rays = a.sched->n_rays, max_samples = a.sched->max_samples;
    for (uint32_t vb = blockIdx.x; vb * blockDim.x < n_rays * (uint32_t)G; vb += gridDim.x) {
        Pcg32 rng = rng0;   // each grid-stride trip starts from the step's stream (the ray's offset is added below)
        const uint32_t i = (vb * blockDim.x + threadIdx.x) / G;
        const bool in = i < n_rays;
        const uint32_t ii = in ? i : 0u;
        const uint32_t img = ((ii * im.n) / n_rays) % im.n;   // image_idx (nerf_device.cuh:578-597)
        rng.advance((uint64_t)ii * N_MAX_RANDOM_SAMPLES_PER_RAY);
        const f2 uv = train_image_pos(rng, im);
        const bool live = in && !(read_rgba(im, img, uv).x < 0.0f);   // masked pixel: no samples
        (void)rng.next_float();                                    // motionblur_time
        const TrainRay ray = train_ray(im, img, uv);
        const f3 dn = normalize(ray.d);
        const aabb box = a.vol.train_aabb;
        const float tmin = fmaxf(aabb_entry(box, ray.o, dn), 0.0f);
        const StepSpace& ss = a.vol.ss;
        const float startt = LIN ? advance_n_steps(tmin, 0.0f, rng.next_float()) : advance_n_steps(tmin, ss, rng.next_float());
        const f3 idir = inv(dn);
        const f3 hs = half_sign(dn);
        auto step_dt = [&](float t) { return LIN ? calc_dt(t, 0.0f) : calc_dt(t, ss); };
        auto skip = [&](float t, f3 p) {
            if constexpr (LIN) return dda_step_linear(t, p, idir, hs);
            else return advance_to_next_voxel(t, ss, p, dn, idir, mip_from_dt(step_dt(t), p, a.vol.max_mip));
        };
        auto occupied = [&](float t, f3 p) {
            if constexpr (LIN) return occupied_linear(p, a.vol.occ_linear);
            else return occupied_at(p, a.vol.bitfield, mip_from_dt(step_dt(t), p, a.vol.max_mip));
        };
        float* const ts = tscr + ii;
        uint32_t j = 0;
        float t = startt;
        bool dda = false, done = !live;   // uniform over the group
        while (!done) {
            float tk = t;
            if (!dda) {
                for (uint32_t u = 0; u < gl; ++u) tk = tk + step_dt(tk);
            } else {
                for (uint32_t u = 0; u < gl; ++u) tk = skip(tk, ray.o + tk * dn);
            }
            const f3 pk = ray.o + tk * dn;
            const bool ink = aabb_contains(box, pk) && (dda ? j : j + gl) < NERF_STEPS;
            const bool occk = ink && occupied(tk, pk);
            const bool stopk = dda ? (!ink || occk) : !occk;
            const uint64_t sb = __ballot(stopk) & gmask;
            const uint32_t m = sb ? (uint32_t)(__ffsll((long long)sb) - 1) - g0 : (uint32_t)G;
            if (!dda) {
                if (gl < m) ts[(size_t)(j + gl) * n_rays] = tk;
                j += m;
            }
            if (m == (uint32_t)G) {   // every lane continued the kind: the next trip starts after lane G - 1
                const float tl = __shfl(tk, (int)(g0 + G - 1), 64);
                t = dda ? skip(tl, ray.o + tl * dn) : tl + step_dt(tl);
                continue;
            }
            const float tm = __shfl(tk, (int)(g0 + m), 64);
            const bool inm = __shfl((int)ink, (int)(g0 + m), 64) != 0;
            if (!inm) { done = true; continue; }
            if (!dda) { t = skip(tm, ray.o + tm * dn); dda = true; }   // an empty cell inside: its DDA step
            else { t = tm; dda = false; }                              // an occupied cell: samples from here
        }
        if (a.debug && live && gl == 0) { b.loss[i] = (float)j; b.coords_c[2 * i] = tmin; b.coords_c[2 * i + 1] = startt; }
        const uint32_t numsteps = j;
        uint32_t base = wave_reserve(&b.ctrl->numsteps_counter, gl == 0 ? numsteps : 0u, lane);
        base = __shfl(base, (int)g0, 64);
        const bool keep = numsteps > 0 && base + numsteps <= max_samples;
        uint32_t ray_idx = wave_reserve(&b.ctrl->ray_counter, gl == 0 && keep ? 1u : 0u, lane);
        ray_idx = __shfl(ray_idx, (int)g0, 64);
        if (!keep) continue;
        if (gl == 0) {
            b.ray_indices[ray_idx] = i;
            b.rays[2 * ray_idx] = make_float4(ray.o.x, ray.o.y, ray.o.z, 0.0f);
            b.rays[2 * ray_idx + 1] = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.0f);
            b.numsteps[ray_idx] = make_uint2(numsteps, base);
        }
        const f3 wd = (dn + 1.0f) * 0.5f;   // warp_direction
        const f3 diag = box.hi - box.lo;
        float* co = b.coords + (size_t)base * 7;
        for (uint32_t k = gl; k < numsteps; k += G) {
            const float tk = ts[(size_t)k * n_rays];
            const f3 p = ray.o + tk * dn;
            const f3 wp = (p - box.lo) / diag;   // warp_position = aabb.relative_pos
            float* c = co + (size_t)k * 7;
            c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(step_dt(tk)); c[4] = wd.x; c[5] = wd.y; c[6] = wd.z;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// compute_loss_kernel_train_nerf (testbed_nerf.cu:1000-1313): Logistic rgb / Exponential density,
// SRGB colour space (train_in_linear_colors = false), random background colour, no envmap,
// error map, sharpness, exposure or depth supervision
// ---------------------------------------------------------------------------------------------
// 16 lanes per ray (LOSS_G): the lanes form 16 samples' colours and opacities at once (logistic, exp -- the bulk of the
// work), and the group then runs the serial transmittance chain over them, one sample per trip, from shuffled values:
// the chain is the reference's float sequence (weight = alpha T, rgb_ray += weight rgb, T *= 1 - alpha, the EPSILON
// stop before each sample), and the lane that owns a sample writes its partial.  (One lane per ray left the chain's
// per-sample math on the critical path of the longest ray: 0.20 ms per batch.)
constexpr uint32_t LOSS_G = 16;
__global__ __launch_bounds__(256) void train_loss_kernel(TrainStepArgs a, TrainImages im, TrainBatch b, Pcg32 rng0, const float* __restrict__ mean_density) {
    const uint32_t n_rays = a.sched->n_rays, n_in = b.ctrl->ray_counter;
    for (uint32_t vb = blockIdx.x; vb * blockDim.x < n_in * LOSS_G; vb += gridDim.x) {
        Pcg32 rng = rng0;   // each grid-stride trip starts from the step's stream (the ray's offset is added below)
        const uint32_t gi = (vb * blockDim.x + threadIdx.x) / LOSS_G;
        const int lane = threadIdx.x & 63;
        const uint32_t gl = (uint32_t)lane % LOSS_G, g0 = (uint32_t)lane - gl;   // lane within the ray's group, the group's first lane
        const bool in = gi < n_in;   // the groups past the last ray stay for the wave's reservation (cn = 0)
        const uint32_t i = in ? gi : 0u;
        const uint2 ns = in ? b.numsteps[i] : make_uint2(0u, 0u);
        const uint32_t numsteps = ns.x, base = ns.y;
        const float* __restrict__ cin = b.coords + (size_t)base * 7;
        const uint16_t* __restrict__ nout = b.mlp_out + (size_t)base * 4;
        // the ray's target colour first (independent of the chain below, so its image read overlaps it): the same RNG draws
        // as train_generate_kernel for this ray -- uv, (max_level off), motionblur, then bg
        const uint32_t ray_idx = b.ray_indices[i];
        rng.advance((uint64_t)ray_idx * N_MAX_RANDOM_SAMPLES_PER_RAY);
        const uint32_t img = ((ray_idx * im.n) / n_rays) % im.n;
        const f2 uv = train_image_pos(rng, im);
        rng.advance(1);   // motionblur_time
        f3 bg = a.background;
        if (a.random_bg) { const float x = rng.next_float(), y = rng.next_float(), z = rng.next_float(); bg = mk(x, y, z); }
        bg = mk(srgb_to_linear(bg.x), srgb_to_linear(bg.y), srgb_to_linear(bg.z));
        const float4 tex = read_rgba(im, img, uv);
        bg = mk(linear_to_srgb(bg.x), linear_to_srgb(bg.y), linear_to_srgb(bg.z));
        f3 target;
        if (tex.w > 0.0f) {
            const f3 lin = mk(tex.x / tex.w, tex.y / tex.w, tex.z / tex.w);   // exposure_scale = exp(0) = 1
            target = mk(linear_to_srgb(lin.x), linear_to_srgb(lin.y), linear_to_srgb(lin.z)) * tex.w + (1.0f - tex.w) * bg;
        } else {
            target = bg;
        }
        float T = 1.0f;
        const float EPSILON = 1e-4f;
        f3 rgb_ray = splat(0.0f);
        uint32_t cn = 0;
        bool stop = false;
        // the next chunk's output and dt are loaded while this chunk's transmittance chain runs (clamped index: the last
        // sample again past the ray's end, unused)
        uint2 ow_n = make_uint2(0u, 0u);
        float wdt_n = 0.0f;
        if (numsteps) {
            const uint32_t j0 = min(gl, numsteps - 1);
            ow_n = *reinterpret_cast<const uint2*>(nout + (size_t)j0 * 4);
            wdt_n = cin[(size_t)j0 * 7 + 3];
        }
        for (uint32_t c0 = 0; c0 < numsteps && !stop; c0 += LOSS_G) {
            const uint2 ow = ow_n;
            const float wdt = wdt_n;
            {
                const uint32_t jn = min(c0 + LOSS_G + gl, numsteps - 1);
                ow_n = *reinterpret_cast<const uint2*>(nout + (size_t)jn * 4);
                wdt_n = cin[(size_t)jn * 7 + 3];
            }
            const float o0 = h2f((uint16_t)(ow.x & 0xffffu)), o1 = h2f((uint16_t)(ow.x >> 16));
            const float o2 = h2f((uint16_t)(ow.y & 0xffffu)), o3 = h2f((uint16_t)(ow.y >> 16));
            const f3 rgb = mk(logistic(o0), logistic(o1), logistic(o2));
            const float dt = unwarp_dt(wdt);
            const float density = sng_expf(o3);
            const float alpha = 1.0f - sng_expf(-density * dt);
            for (uint32_t u = 0; u < LOSS_G; ++u) {
                if (c0 + u >= numsteps) break;
                if (T < EPSILON) { stop = true; break; }
                const int src = (int)(g0 + u);
                const float au = __shfl(alpha, src, 64);
                const f3 ru = mk(__shfl(rgb.x, src, 64), __shfl(rgb.y, src, 64), __shfl(rgb.z, src, 64));
                const float weight = au * T;
                rgb_ray = rgb_ray + weight * ru;
                if (gl == u) b.partial[base + cn] = make_float4(T, rgb_ray.x, rgb_ray.y, rgb_ray.z);   // train_dloss_kernel replays from here
                T *= (1.0f - au);
                ++cn;
            }
        }
        if (cn == numsteps) rgb_ray = rgb_ray + T * bg;
        if (!in || gl != 0) continue;
        // the compaction slot comes from train_compact_kernel (a prefix of the composited counts in the rays' image order)
        b.cnt_i[ray_idx] = cn;
        // Huber loss (alpha = 0.1) / 5, loss_and_gradient (nerf_device.cuh:100-117, 601-616)
        f3 grad;
        float loss_sum = 0.0f;
        {
            const float alpha_h = 0.1f;
            const float dv[3] = {rgb_ray.x - target.x, rgb_ray.y - target.y, rgb_ray.z - target.z};
            float gv[3];
            for (int k = 0; k < 3; ++k) {
                const float ad = fabsf(dv[k]);
                const float sq = 0.5f / alpha_h * dv[k] * dv[k];
                const float l = ad > alpha_h ? (ad - 0.5f * alpha_h) : sq;
                gv[k] = (ad > alpha_h ? (dv[k] > 0 ? 1.0f : -1.0f) : (dv[k] / alpha_h)) / 5.0f;
                loss_sum += l / 5.0f;
            }
            grad = mk(gv[0], gv[1], gv[2]);
        }
        b.loss[i] = (loss_sum / 3.0f) / (float)n_rays;
        const float loss_scale = a.loss_scale / (float)n_rays;
        const float l1_reg_density = *mean_density < NERF_MIN_OPTICAL_THICKNESS ? 1e-4f : 0.0f;
        // the per-sample gradients need only this ray's constants and the forward partials: they are
        // written by train_dloss_kernel with one wave per ray instead of this lane's serial loop
        b.rayrec[3 * i] = make_float4(0.0f, 0.0f, __uint_as_float(base), 0.0f);
        b.rayrec[3 * i + 1] = make_float4(grad.x, grad.y, grad.z, loss_scale);
        b.rayrec[3 * i + 2] = make_float4(rgb_ray.x, rgb_ray.y, rgb_ray.z, l1_reg_density);
    }
}

// The compaction of the composited samples into the batch (testbed_nerf.cu:1150: an atomicAdd per ray, so the reference
// fills the batch in the order its threads finish): here an exclusive prefix over the rays in their image order (the
// random pixel index i of generate_training_samples_nerf), so which rays make the batch does not depend on how fast each
// ray's march or composite ran.  (A completion order favours the short rays whenever the batch overflows its target: with
// 4 rays per wave in the loss kernel that bias was strong enough to collapse the density field within 200 steps.)  One
// workgroup: ~10^4 rays.
__global__ __launch_bounds__(1024) void train_compact_kernel(const TrainSched* __restrict__ sched, const uint32_t* __restrict__ cnt, uint32_t* __restrict__ cbase, TrainCtrl* ctrl) {
    __shared__ uint32_t part[1024];
    const uint32_t n = sched->n_rays;
    const uint32_t per = (n + 1023u) / 1024u, t0 = threadIdx.x * per, t1 = min(n, t0 + per);
    uint32_t sum = 0;
    for (uint32_t k = t0; k < t1; ++k) sum += cnt[k];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024u; d <<= 1) {   // Hillis-Steele inclusive scan of the thread sums
        const uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - sum;
    for (uint32_t k = t0; k < t1; ++k) { cbase[k] = run; run += cnt[k]; }
    if (threadIdx.x == 1023) ctrl->numsteps_compacted = part[1023];
}

// compute_loss_kernel_train_nerf's gradient loop (testbed_nerf.cu:1209-1275) for the ray's first
// ccount samples, one wave per ray, lanes over the samples: T and the running rgb come from the
// forward pass's partials (the same float sequence), so every value is the serial loop's.
__global__ __launch_bounds__(256) void train_dloss_kernel(TrainStepArgs a, TrainBatch b) {
    const uint32_t n_in = b.ctrl->ray_counter;
    for (uint32_t vb = blockIdx.x; vb * (blockDim.x >> 6) < n_in; vb += gridDim.x) {
        const uint32_t i = (vb * blockDim.x + threadIdx.x) >> 6;
        const uint32_t lane = threadIdx.x & 63;
        if (i >= n_in) continue;
        // the ray's compaction slot and count (a prefix over the rays' image order, train_compact_kernel)
        const uint32_t ri = b.ray_indices[i], cn = b.cnt_i[ri], cbase = b.cbase_i[ri];
        const uint32_t ccount = min(a.target_batch - min(a.target_batch, cbase), cn);
        if (ccount == 0) {   // past the batch target: no loss and no gradient for this ray (testbed_nerf.cu: compacted_numsteps == 0)
            if (lane == 0) b.loss[i] = 0.0f;
            continue;
        }
        const float4 r0 = b.rayrec[3 * i], r1 = b.rayrec[3 * i + 1], r2 = b.rayrec[3 * i + 2];
        const uint32_t base = __float_as_uint(r0.z);
        const f3 grad = mk(r1.x, r1.y, r1.z), rgb_ray = mk(r2.x, r2.y, r2.z);
        const float loss_scale = r1.w, l1_reg_density = r2.w;
        const aabb box = a.vol.train_aabb;
        const f3 diag = box.hi - box.lo;
        const float4 ro4 = b.rays[2 * i];
        const f3 ray_o = mk(ro4.x, ro4.y, ro4.z);
        const float* __restrict__ cin = b.coords + (size_t)base * 7;
        const uint16_t* __restrict__ nout = b.mlp_out + (size_t)base * 4;
        float* __restrict__ cout = b.coords_c + (size_t)cbase * 7;
        uint16_t* __restrict__ dout = b.dloss + (size_t)cbase * 4;
        for (uint32_t j = lane; j < ccount; j += 64) {
            const float* c = cin + (size_t)j * 7;
            for (int k = 0; k < 7; ++k) cout[(size_t)j * 7 + k] = c[k];
            const f3 pos = box.lo + mk(c[0], c[1], c[2]) * diag;   // unwarp_position
            const float depth = length(pos - ray_o);
            const float dt = unwarp_dt(c[3]);
            const uint16_t* o = nout + (size_t)j * 4;
            const float o0 = h2f(o[0]), o1 = h2f(o[1]), o2 = h2f(o[2]), o3 = h2f(o[3]);
            const f3 rgb = mk(logistic(o0), logistic(o1), logistic(o2));
            const float density = sng_expf(o3);
            const float alpha = 1.0f - sng_expf(-density * dt);
            const float4 pt = b.partial[base + j];
            const float weight = alpha * pt.x;
            const f3 rgb_ray2 = mk(pt.y, pt.z, pt.w);
            const float T = pt.x * (1.0f - alpha);
            const f3 suffix = rgb_ray - rgb_ray2;
            const f3 dl_drgb = weight * grad;
            const float d0 = loss_scale * (dl_drgb.x * (rgb.x * (1.0f - rgb.x)));
            const float d1 = loss_scale * (dl_drgb.y * (rgb.y * (1.0f - rgb.y)));
            const float d2 = loss_scale * (dl_drgb.z * (rgb.z * (1.0f - rgb.z)));
            const float dens_deriv = sng_expf(fminf(fmaxf(o3, -15.0f), 15.0f));
            const float dl_dmlp = dens_deriv * (dt * dot(grad, T * rgb - suffix));
            const float d3 = loss_scale * dl_dmlp + (o3 < 0.0f ? -l1_reg_density : 0.0f) + (o3 > -10.0f && depth < a.near_distance ? 1e-4f : 0.0f);
            dout[(size_t)j * 4 + 0] = f2h(d0);
            dout[(size_t)j * 4 + 1] = f2h(d1);
            dout[(size_t)j * 4 + 2] = f2h(d2);
            dout[(size_t)j * 4 + 3] = f2h(d3);
        }
    }
}

// NerfCounters::update_after_training (testbed_nerf.cu:3272-3296) on the device: the next step's rays_per_batch from this
// step's compacted count, with the host expressions' float operations (correctly rounded multiply and divide), and the
// next max_inference from the count before compaction (train_args' rounding)
__device__ void sched_update(TrainSched* __restrict__ sched, const TrainCtrl* __restrict__ ctrl, uint32_t target) {
    TrainSched n = *sched;
    const uint32_t before = ctrl->numsteps_counter, after = ctrl->numsteps_compacted;
    if (before == 0 || after == 0) {
        n.measured = n.measured_before = 0;
    } else {
        n.measured_before = before;
        n.measured = after;
        const uint32_t r = (uint32_t)__fdiv_rn(__fmul_rn((float)n.n_rays, (float)target), (float)after);
        n.n_rays = min((r + BATCH_SIZE_GRANULARITY - 1) / BATCH_SIZE_GRANULARITY * BATCH_SIZE_GRANULARITY, 1u << 18);
    }
    const uint32_t cap = target * 16;
    n.max_samples = n.measured_before == 0 ? cap : (min(n.measured_before, cap) + BATCH_SIZE_GRANULARITY - 1) / BATCH_SIZE_GRANULARITY * BATCH_SIZE_GRANULARITY;
    *sched = n;
}

// tcnn fill_rollover / fill_rollover_and_rescale: entries [n_in, target) repeat entry (i mod n_in);
// rolled-over gradients are scaled by n_in / target
// sched_next (training steps, not the parity hooks): one thread also forms the next step's batch sizes (sched_update)
__global__ void train_rollover_kernel(TrainStepArgs a, TrainBatch b, TrainSched* __restrict__ sched_next) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (sched_next && i == 0) sched_update(sched_next, b.ctrl, a.target_batch);
    if (i >= a.target_batch) return;
    const uint32_t n_in = min(b.ctrl->numsteps_compacted, a.target_batch);
    if (n_in == 0 || i < n_in) return;
    const uint32_t src = i % n_in;
    for (int k = 0; k < 7; ++k) b.coords_c[(size_t)i * 7 + k] = b.coords_c[(size_t)src * 7 + k];
    const float s = (float)n_in / (float)a.target_batch;
    for (int k = 0; k < 4; ++k) b.dloss[(size_t)i * 4 + k] = f2h(h2f(b.dloss[(size_t)src * 4 + k]) * s);
}

// ---------------------------------------------------------------------------------------------
// MLP weight fragments from an fp16 parameter blob (tcnn order, nerf_network.h:356-371):
// forward A fragments (20 x 64 lanes x 8, the same image host_render.cpp set_model packs on the host)
// and backward A fragments of W^T (36 x 64 lanes x 4) for v_mfma_f32_16x16x16f16
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint16_t fwd_frag_elem(const uint16_t* W, int n_in, int mb, int kb, bool permuted, int lane, int j) {
    const int row = 16 * mb + (lane & 15), g = lane >> 4;
    const int k = permuted ? 32 * kb + 16 * (j >= 4) + 4 * g + (j & 3) : 32 * kb + 8 * g + j;
    return W[row * n_in + k];
}
// clamp_in (the training step's pack): one thread also writes the network's sample count, min(numsteps_counter,
// max_samples) -- the generator drops rays beyond max_samples
__global__ void train_pack_kernel(const uint16_t* __restrict__ p, uint16_t* __restrict__ wfrag, uint16_t* __restrict__ wfrag_t, const uint32_t* __restrict__ clamp_in,
                                  const TrainSched* __restrict__ sched, uint32_t* __restrict__ clamp_out) {
    if (clamp_in && blockIdx.x == 0 && threadIdx.x == 0) *clamp_out = min(*clamp_in, sched->max_samples);
    const int lane = threadIdx.x & 63, f = blockIdx.x;   // grid: 20 forward + 36 backward fragments
    const uint16_t *dW0 = p, *dW1 = p + 64 * 32, *rW0 = p + 3072, *rW1 = rW0 + 64 * 32, *rW2 = rW1 + 64 * 64;
    if (f < 20) {
        for (int j = 0; j < 8; ++j) {
            uint16_t v;
            if (f < 4) v = fwd_frag_elem(dW0, 32, f, 0, false, lane, j);
            else if (f < 6) v = fwd_frag_elem(dW1, 64, 0, f - 4, true, lane, j);
            else if (f < 10) v = fwd_frag_elem(rW0, 32, f - 6, 0, true, lane, j);
            else if (f < 18) v = fwd_frag_elem(rW1, 64, (f - 10) / 2, (f - 10) % 2, true, lane, j);
            else v = fwd_frag_elem(rW2, 64, 0, f - 18, true, lane, j);
            wfrag[(f * 64 + lane) * 8 + j] = v;
        }
        return;
    }
    // W^T fragment (i, q): lane l, j -> W[16q + 4(l/16) + j][16i + l%16]
    const int b = f - 20;
    const uint16_t* W;
    int n_in, i, q;
    if (b < 4) { W = rW2; n_in = 64; i = b; q = 0; }                       // dh2 <- do      (T_RGB2)
    else if (b < 20) { W = rW1; n_in = 64; i = (b - 4) / 4; q = (b - 4) % 4; }   // dh1 <- dh2 (T_RGB1)
    else if (b < 24) { W = rW0; n_in = 32; i = 0; q = b - 20; }            // drin[0:16] <- dh1 (T_RGB0)
    else if (b < 28) { W = dW1; n_in = 64; i = b - 24; q = 0; }            // dh0 <- ddens   (T_DEN1)
    else { W = dW0; n_in = 32; i = (b - 28) / 4; q = (b - 28) % 4; }       // denc <- dh0    (T_DEN0)
    for (int j = 0; j < 4; ++j) wfrag_t[(b * 64 + lane) * 4 + j] = W[(16 * q + 4 * (lane >> 4) + j) * n_in + 16 * i + (lane & 15)];
}
constexpr int T_RGB2 = 0, T_RGB1 = 4, T_RGB0 = 20, T_DEN1 = 24, T_DEN0 = 28;

struct U16x8 { uint16_t v[8]; };
__device__ __forceinline__ h4v to_h4(f4v v) { return {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]}; }
__device__ __forceinline__ f4v relu_mask(f4v d, f4v pre) {
    // ReLU backward on the post-activation value (tcnn: grad *= (y > 0)); y = relu(pre) > 0 <=> pre > 0
    // with y rounded to fp16 exactly as the forward stores it
    f4v r;
    for (int k = 0; k < 4; ++k) r[k] = ((_Float16)fmaxf(pre[k], 0.0f) > (_Float16)0.0f) ? d[k] : 0.0f;
    return r;
}
// tiled activation/gradient store: [tile][feature][16 samples] fp16
__device__ __forceinline__ void store_rows(uint16_t* tile_base, int feat0, int g, int col, f4v v) {
    for (int k = 0; k < 4; ++k) tile_base[(feat0 + 4 * g + k) * 16 + col] = __builtin_bit_cast(uint16_t, (_Float16)v[k]);
}
__device__ __forceinline__ void store_rows_relu(uint16_t* tile_base, int feat0, int g, int col, f4v v) {
    for (int k = 0; k < 4; ++k) tile_base[(feat0 + 4 * g + k) * 16 + col] = __builtin_bit_cast(uint16_t, (_Float16)fmaxf(v[k], 0.0f));
}

// hash-grid backward for one level and F features of one sample: d(param) += w_corner * d(feature)
// (tcnn kernel_grid_backward: float weights, atomic adds)
template <int F>
__device__ __forceinline__ void grid_backward_level(const LevelInfo& L, float* __restrict__ ggrad, float x0, float x1, float x2, const float* dfeat) {
    const float p0 = fmaf(L.scale, x0, 0.5f), p1 = fmaf(L.scale, x1, 0.5f), p2 = fmaf(L.scale, x2, 0.5f);
    const float q0 = floorf(p0), q1 = floorf(p1), q2 = floorf(p2);
    const uint32_t g0 = (uint32_t)(int)q0, g1 = (uint32_t)(int)q1, g2 = (uint32_t)(int)q2;
    const float f0 = p0 - q0, f1 = p1 - q1, f2 = p2 - q2;
    float* tbl = ggrad + (size_t)L.offset * F;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float w = 1.0f;
        w *= (c & 1) ? f0 : 1.0f - f0;
        w *= (c & 2) ? f1 : 1.0f - f1;
        w *= (c & 4) ? f2 : 1.0f - f2;
        const uint32_t idx = grid_index(L, g0 + (c & 1), g1 + ((c >> 1) & 1), g2 + ((c >> 2) & 1)) * F;
#pragma unroll
        for (int f = 0; f < F; ++f)
            if (dfeat[f] != 0.0f) atomicAdd(tbl + idx + f, w * dfeat[f]);
    }
}

// The same scatter with the atomics shaped for the memory-side atomic unit (F = 4): one atomic
// wave-instruction covers 16 corner entries x 4 features = 16 aligned 16-B segments (lane 4q + f adds
// feature f of the corner of source lane 16i + q) instead of 64 scattered dwords, so each instruction
// leaves L2 as 16 requests rather than 64 (MI355X_MICROARCH.md "Global float atomics": scattered
// lanes run ~17x below the contiguous rate).  Same products w * dfeat[f], same atomics, regrouped.
// Source lanes 16i..16i+15 share lane group g = i, hence one level per instruction.
__device__ __forceinline__ void grid_backward_level_coop4(const LevelInfo& L, float* __restrict__ ggrad, float x0, float x1, float x2,
                                                          const float* dfeat, int lane) {
    const float p0 = fmaf(L.scale, x0, 0.5f), p1 = fmaf(L.scale, x1, 0.5f), p2 = fmaf(L.scale, x2, 0.5f);
    const float q0 = floorf(p0), q1 = floorf(p1), q2 = floorf(p2);
    const uint32_t g0 = (uint32_t)(int)q0, g1 = (uint32_t)(int)q1, g2 = (uint32_t)(int)q2;
    const float f0 = p0 - q0, f1 = p1 - q1, f2 = p2 - q2;
    const int f = lane & 3, qd = lane >> 2;
    float ds[4];   // dfeat[f] of source lane 16i + qd
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int src = 16 * i + qd;
        const float v0 = __shfl(dfeat[0], src, 64), v1 = __shfl(dfeat[1], src, 64), v2 = __shfl(dfeat[2], src, 64), v3 = __shfl(dfeat[3], src, 64);
        ds[i] = f == 0 ? v0 : (f == 1 ? v1 : (f == 2 ? v2 : v3));
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float w = 1.0f;
        w *= (c & 1) ? f0 : 1.0f - f0;
        w *= (c & 2) ? f1 : 1.0f - f1;
        w *= (c & 4) ? f2 : 1.0f - f2;
        const uint32_t at = L.offset * 4u + grid_index(L, g0 + (c & 1), g1 + ((c >> 1) & 1), g2 + ((c >> 2) & 1)) * 4u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int src = 16 * i + qd;
            const float ws = __shfl(w, src, 64);
            const uint32_t as = __shfl(at, src, 64);
            // consecutive samples of a ray that share this corner entry (the coarse levels: a 16^3 cell
            // holds ~37 samples of a ray) form runs over qd; a segmented scan sums each run and only
            // its last lane adds to memory, instead of up to 16 adds to one address in one instruction
            float v = ws * ds[i];
            const uint32_t a_prev = __shfl_up(as, 4u, 64), a_next = __shfl_down(as, 4u, 64);
            bool head = qd == 0 || a_prev != as;
#pragma unroll
            for (int d = 1; d < 16; d <<= 1) {
                const float u = __shfl_up(v, 4u * (unsigned)d, 64);
                const bool hu = __shfl_up(head, 4u * (unsigned)d, 64);
                if (qd >= d && !head) { v += u; head = hu; }
            }
            const bool tail = qd == 15 || a_next != as;
            if (tail && v != 0.0f) atomicAdd(ggrad + as + f, v);
        }
    }
}

// The same scatter into an fp16 gradient with packed atomics (train_grid_grad_f16): tcnn accumulates the hash-grid
// gradient in the network's precision, __half2 atomicAdd per feature pair (GridEncoding backward, grad_t = T when a
// thread holds 2 features).  One global_atomic_pk_add_f16 wave-instruction covers 32 corner entries x 2 feature pairs
// (lane 2q' + h adds features 2h, 2h+1 of source lane 32i + q'), half the bytes of the f32 scatter, which the
// memory-side atomic unit moves at the same byte rate (MI355X_MICROARCH.md, Global float atomics).  Runs of equal
// entries are summed in f32 (the segmented scan of the f32 form) and rounded to fp16 once per run.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void grid_backward_level_coop4_h(const LevelInfo& L, uint16_t* __restrict__ ggrad, float x0, float x1, float x2,
                                                            const float* dfeat, int lane) {
    const float p0 = fmaf(L.scale, x0, 0.5f), p1 = fmaf(L.scale, x1, 0.5f), p2 = fmaf(L.scale, x2, 0.5f);
    const float q0 = floorf(p0), q1 = floorf(p1), q2 = floorf(p2);
    const uint32_t g0 = (uint32_t)(int)q0, g1 = (uint32_t)(int)q1, g2 = (uint32_t)(int)q2;
    const float f0 = p0 - q0, f1 = p1 - q1, f2 = p2 - q2;
    const int h = lane & 1, qd = (lane >> 1) & 15, sq = lane >> 1;
    float dlo[2], dhi[2];   // features 2h, 2h+1 of source lane 32i + sq
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int src = 32 * i + sq;
        const float v0 = __shfl(dfeat[0], src, 64), v1 = __shfl(dfeat[1], src, 64), v2 = __shfl(dfeat[2], src, 64), v3 = __shfl(dfeat[3], src, 64);
        dlo[i] = h ? v2 : v0;
        dhi[i] = h ? v3 : v1;
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float w = 1.0f;
        w *= (c & 1) ? f0 : 1.0f - f0;
        w *= (c & 2) ? f1 : 1.0f - f1;
        w *= (c & 4) ? f2 : 1.0f - f2;
        const uint32_t at = L.offset * 4u + grid_index(L, g0 + (c & 1), g1 + ((c >> 1) & 1), g2 + ((c >> 2) & 1)) * 4u;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int src = 32 * i + sq;
            const float ws = __shfl(w, src, 64);
            const uint32_t as = __shfl(at, src, 64);
            float va = ws * dlo[i], vb = ws * dhi[i];
            const uint32_t a_prev = __shfl_up(as, 2u, 64), a_next = __shfl_down(as, 2u, 64);
            bool head = qd == 0 || a_prev != as;
#pragma unroll
            for (int d = 1; d < 16; d <<= 1) {
                const float ua = __shfl_up(va, 2u * (unsigned)d, 64), ub = __shfl_up(vb, 2u * (unsigned)d, 64);
                const bool hu = __shfl_up(head, 2u * (unsigned)d, 64);
                if (qd >= d && !head) { va += ua; vb += ub; head = hu; }
            }
            const bool tail = qd == 15 || a_next != as;
            if (tail && (va != 0.0f || vb != 0.0f)) {
                const h2v v = {(_Float16)va, (_Float16)vb};
                __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2v*)(ggrad + as + 2 * h), v);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// NerfNetwork forward + backward per 16-sample tile (nerf_network.h:144-268).  Activations
// (post-ReLU, fp16) and pre-activation gradients (fp16) go to acts[tile][TRAIN_FEATS][16] for
// train_dw_kernel; the encoding gradient is scattered into the f32 grid gradient.
// ---------------------------------------------------------------------------------------------
template <int F, bool H16 = false>
__global__ __launch_bounds__(256) void train_field_kernel(TrainStepArgs a, TrainBatch b, const h8* __restrict__ wfrag, const h4v* __restrict__ wfrag_t,
                                                          const _Float16* __restrict__ grid, const LevelInfo* __restrict__ levels,
                                                          float* __restrict__ ggrad, uint16_t* __restrict__ ggrad_h) {
    const uint32_t n = a.target_batch;
    const uint32_t n_tiles = (n + 15) >> 4;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
    const int g = lane >> 4, col = lane & 15;
    const f4v zero = {0.0f, 0.0f, 0.0f, 0.0f};
    h8 W[20];
#pragma unroll
    for (int f = 0; f < 20; ++f) W[f] = wfrag[f * 64 + lane];
    for (uint32_t tile = wave; tile < n_tiles; tile += n_waves) {
        const uint32_t s = tile * 16 + col;
        const bool valid = s < n;
        const float* c = b.coords_c + (size_t)(valid ? s : n - 1) * 7;
        const float x0 = c[0], x1 = c[1], x2 = c[2], d0 = c[4], d1 = c[5], d2 = c[6];
        uint16_t* tb = b.acts + (size_t)tile * TRAIN_FEATS * 16;
        // ---- forward (field_tile, keeping the activations)
        const h8 enc = encode_lane<F>(levels, grid, g, x0, x1, x2);
        f4v a0 = mfma16(W[0], enc, zero), a1 = mfma16(W[1], enc, zero), a2 = mfma16(W[2], enc, zero), a3 = mfma16(W[3], enc, zero);
        f4v dens = mfma16(W[4], pack_relu(a0, a1), zero);
        dens = mfma16(W[5], pack_relu(a2, a3), dens);
        float sh[4];
        sh_lane(g, d0, d1, d2, sh);
        h8 rin;
        rin[0] = (_Float16)dens[0]; rin[1] = (_Float16)dens[1]; rin[2] = (_Float16)dens[2]; rin[3] = (_Float16)dens[3];
        rin[4] = (_Float16)sh[0]; rin[5] = (_Float16)sh[1]; rin[6] = (_Float16)sh[2]; rin[7] = (_Float16)sh[3];
        f4v b0 = mfma16(W[6], rin, zero), b1 = mfma16(W[7], rin, zero), b2 = mfma16(W[8], rin, zero), b3 = mfma16(W[9], rin, zero);
        const h8 k0 = pack_relu(b0, b1), k1 = pack_relu(b2, b3);
        f4v c0 = mfma16(W[10], k0, zero); c0 = mfma16(W[11], k1, c0);
        f4v c1 = mfma16(W[12], k0, zero); c1 = mfma16(W[13], k1, c1);
        f4v c2 = mfma16(W[14], k0, zero); c2 = mfma16(W[15], k1, c2);
        f4v c3 = mfma16(W[16], k0, zero); c3 = mfma16(W[17], k1, c3);
        // activations for the weight gradients
        // whole-vector bit casts: element-wise __builtin_bit_cast(uint16_t, v[k]) of an ext_vector
        // element stored v[0] for every k with this compiler (caught by tests/test_gpu_train.py)
        const U16x8 eu = __builtin_bit_cast(U16x8, enc), ru = __builtin_bit_cast(U16x8, rin);
        for (int k = 0; k < 8; ++k) tb[(A_ENC + 8 * g + k) * 16 + col] = eu.v[k];
        store_rows_relu(tb, A_H0 + 0, g, col, a0); store_rows_relu(tb, A_H0 + 16, g, col, a1);
        store_rows_relu(tb, A_H0 + 32, g, col, a2); store_rows_relu(tb, A_H0 + 48, g, col, a3);
        for (int k = 0; k < 4; ++k) {
            tb[(A_RIN + 4 * g + k) * 16 + col] = ru.v[k];
            tb[(A_RIN + 16 + 4 * g + k) * 16 + col] = ru.v[4 + k];
        }
        store_rows_relu(tb, A_H1 + 0, g, col, b0); store_rows_relu(tb, A_H1 + 16, g, col, b1);
        store_rows_relu(tb, A_H1 + 32, g, col, b2); store_rows_relu(tb, A_H1 + 48, g, col, b3);
        store_rows_relu(tb, A_H2 + 0, g, col, c0); store_rows_relu(tb, A_H2 + 16, g, col, c1);
        store_rows_relu(tb, A_H2 + 32, g, col, c2); store_rows_relu(tb, A_H2 + 48, g, col, c3);

        // ---- backward.  dL/d(rgb output rows 0..2) and dL/dsigma from the loss (extract_rgb, add_density_gradient)
        f4v d_o = zero;
        float d_sigma = 0.0f;
        if (valid && g == 0) {
            const uint16_t* dl = b.dloss + (size_t)s * 4;
            d_o[0] = h2f(dl[0]); d_o[1] = h2f(dl[1]); d_o[2] = h2f(dl[2]);
            d_sigma = h2f(dl[3]);
        }
        store_rows(tb, D_O, g, col, d_o);
        const h4v bo = to_h4(d_o);
        // rgb W2: dh2 = W2^T d_o, masked by relu(c)
        f4v e0 = relu_mask(mfma16k16(wfrag_t[(T_RGB2 + 0) * 64 + lane], bo, zero), c0);
        f4v e1 = relu_mask(mfma16k16(wfrag_t[(T_RGB2 + 1) * 64 + lane], bo, zero), c1);
        f4v e2 = relu_mask(mfma16k16(wfrag_t[(T_RGB2 + 2) * 64 + lane], bo, zero), c2);
        f4v e3 = relu_mask(mfma16k16(wfrag_t[(T_RGB2 + 3) * 64 + lane], bo, zero), c3);
        store_rows(tb, D_H2 + 0, g, col, e0); store_rows(tb, D_H2 + 16, g, col, e1);
        store_rows(tb, D_H2 + 32, g, col, e2); store_rows(tb, D_H2 + 48, g, col, e3);
        const h4v he[4] = {to_h4(e0), to_h4(e1), to_h4(e2), to_h4(e3)};
        // rgb W1: dh1 = W1^T dh2, masked by relu(b)
        f4v f[4];
        const f4v bpre[4] = {b0, b1, b2, b3};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f4v acc = zero;
#pragma unroll
            for (int q = 0; q < 4; ++q) acc = mfma16k16(wfrag_t[(T_RGB1 + 4 * i + q) * 64 + lane], he[q], acc);
            f[i] = relu_mask(acc, bpre[i]);
            store_rows(tb, D_H1 + 16 * i, g, col, f[i]);
        }
        const h4v hf[4] = {to_h4(f[0]), to_h4(f[1]), to_h4(f[2]), to_h4(f[3])};
        // rgb W0: d(rgb input rows 0..15) = density-network output gradient; + dL/dsigma on row 0
        f4v ddens = zero;
#pragma unroll
        for (int q = 0; q < 4; ++q) ddens = mfma16k16(wfrag_t[(T_RGB0 + q) * 64 + lane], hf[q], ddens);
        {
            // tcnn keeps dL/d(rgb network input) in fp16 before add_density_gradient
            for (int k = 0; k < 4; ++k) ddens[k] = (float)(_Float16)ddens[k];
            if (g == 0) ddens[0] = (float)(_Float16)(ddens[0] + d_sigma);
        }
        store_rows(tb, D_DENS, g, col, ddens);
        const h4v hd = to_h4(ddens);
        // density W1: dh0 = W1^T ddens, masked by relu(a)
        f4v h[4];
        const f4v apre[4] = {a0, a1, a2, a3};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            h[i] = relu_mask(mfma16k16(wfrag_t[(T_DEN1 + i) * 64 + lane], hd, zero), apre[i]);
            store_rows(tb, D_H0 + 16 * i, g, col, h[i]);
        }
        const h4v hh[4] = {to_h4(h[0]), to_h4(h[1]), to_h4(h[2]), to_h4(h[3])};
        // density W0: denc = W0^T dh0 (32 features = 2 blocks)
        f4v de0 = zero, de1 = zero;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            de0 = mfma16k16(wfrag_t[(T_DEN0 + q) * 64 + lane], hh[q], de0);
            de1 = mfma16k16(wfrag_t[(T_DEN0 + 4 + q) * 64 + lane], hh[q], de1);
        }
        // encoding gradient (fp16, as tcnn's dL_ddensity_network_input) -> grid; the lane holds
        // features 4g..4g+3 and 16+4g..16+4g+3 (tail lanes of the last tile contribute nothing)
        float df0[4], df1[4];
        for (int k = 0; k < 4; ++k) { df0[k] = valid ? (float)(_Float16)de0[k] : 0.0f; df1[k] = valid ? (float)(_Float16)de1[k] : 0.0f; }
        if constexpr (F == 4 && H16) {
            grid_backward_level_coop4_h(levels[g], ggrad_h, x0, x1, x2, df0, lane);
            grid_backward_level_coop4_h(levels[4 + g], ggrad_h, x0, x1, x2, df1, lane);
        } else if constexpr (F == 4) {
            grid_backward_level_coop4(levels[g], ggrad, x0, x1, x2, df0, lane);
            grid_backward_level_coop4(levels[4 + g], ggrad, x0, x1, x2, df1, lane);
        } else {
            if (!valid) continue;
            grid_backward_level<2>(levels[2 * g], ggrad, x0, x1, x2, df0);
            grid_backward_level<2>(levels[2 * g + 1], ggrad, x0, x1, x2, df0 + 2);
            grid_backward_level<2>(levels[8 + 2 * g], ggrad, x0, x1, x2, df1);
            grid_backward_level<2>(levels[8 + 2 * g + 1], ggrad, x0, x1, x2, df1 + 2);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Weight gradients: dW[out][in] = sum_s delta[out][s] * act[in][s] over the batch (K = samples),
// v_mfma_f32_16x16x16f16 with both operands read straight from the tiled buffer (4 consecutive
// samples of one feature = 8 B per lane).  Five waves per workgroup split the 40 16x16 blocks;
// each workgroup covers a slab of tiles and adds its partial sums to the f32 gradient.
// ---------------------------------------------------------------------------------------------
struct DwJob { int dfeat, afeat, mb, nb, n_in, param_off; };
__device__ __forceinline__ DwJob dw_job(int blk) {
    // blocks: rgb W1 (16) | rgb W0 (8) | dens W0 (8) | rgb W2 (4) | dens W1 (4)
    if (blk < 16) return {D_H2, A_H1, blk / 4, blk % 4, 64, 3072 + 64 * 32};
    if (blk < 24) { const int b = blk - 16; return {D_H1, A_RIN, b / 2, b % 2, 32, 3072}; }
    if (blk < 32) { const int b = blk - 24; return {D_H0, A_ENC, b / 2, b % 2, 32, 0}; }
    if (blk < 36) { const int b = blk - 32; return {D_O, A_H2, 0, b, 64, 3072 + 64 * 32 + 64 * 64}; }
    const int b = blk - 36;
    return {D_DENS, A_H0, 0, b, 64, 64 * 32};
}
template <bool PIPE>
__global__ __launch_bounds__(320) void train_dw_kernel(TrainStepArgs a, const uint16_t* __restrict__ acts, uint32_t tiles_per_block, float* __restrict__ wgrad) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;   // 5 waves x 8 blocks
    const uint32_t n_tiles = (a.target_batch + 15) >> 4;
    const uint32_t t0 = blockIdx.x * tiles_per_block, t1 = min(n_tiles, t0 + tiles_per_block);
    const int r = lane & 15, kq = lane >> 4;
    f4v acc[8];
    uint32_t oa[8], ob[8];   // the job's A / B operand offsets inside a tile
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        acc[j] = f4v{0.0f, 0.0f, 0.0f, 0.0f};
        const DwJob jb = dw_job(wv * 8 + j);
        oa[j] = (uint32_t)((jb.dfeat + 16 * jb.mb + r) * 16 + 4 * kq);
        ob[j] = (uint32_t)((jb.afeat + 16 * jb.nb + r) * 16 + 4 * kq);
    }
    if constexpr (PIPE) {
        // two register sets used in turn: the loads of the next tile are issued before the current tile's 8 MFMAs,
        // and no copy between the sets waits on them (the last trips reload the last tile and multiply nothing twice)
        if (t0 < t1) {
            h4v A0[8], B0[8], A1[8], B1[8];
            auto load = [&](uint32_t t, h4v* A, h4v* B) {
                const uint16_t* tb = acts + (size_t)min(t, t1 - 1) * TRAIN_FEATS * 16;
#pragma unroll
                for (int j = 0; j < 8; ++j) { A[j] = *reinterpret_cast<const h4v*>(tb + oa[j]); B[j] = *reinterpret_cast<const h4v*>(tb + ob[j]); }
            };
            load(t0, A0, B0);
            // one basic block per trip (a branch between the halves lets the compiler sink the loads to their use);
            // an odd slab's last half multiplies the reloaded last tile and keeps the old sums (select)
            for (uint32_t t = t0; t < t1; t += 2) {
                load(t + 1, A1, B1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] = mfma16k16(A0[j], B0[j], acc[j]);
                __builtin_amdgcn_sched_barrier(0);
                load(t + 2, A0, B0);
                __builtin_amdgcn_sched_barrier(0);
                const bool second = t + 1 < t1;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const f4v r = mfma16k16(A1[j], B1[j], acc[j]);
                    acc[j] = second ? r : acc[j];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else {
        for (uint32_t t = t0; t < t1; ++t) {
            const uint16_t* tb = acts + (size_t)t * TRAIN_FEATS * 16;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const h4v A = *reinterpret_cast<const h4v*>(tb + oa[j]);
                const h4v B = *reinterpret_cast<const h4v*>(tb + ob[j]);
                acc[j] = mfma16k16(A, B, acc[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const DwJob jb = dw_job(wv * 8 + j);
        for (int k = 0; k < 4; ++k) {
            const int row = 16 * jb.mb + 4 * kq + k, cin = 16 * jb.nb + r;
            atomicAdd(&wgrad[jb.param_off + row * jb.n_in + cin], acc[j][k]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// tcnn Ema(ExponentialDecay(Adam)) step (base.json:5-22).  Matrix params (the 10240 MLP weights)
// get l2_reg; grid params with a zero gradient are skipped (sparse update, per-parameter step
// counts for the bias correction).  Writes the fp32 master, the fp16 training copy and the EMA
// (debiased) fp16 inference copy.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float adam_corr(float beta1, float beta2, uint32_t step) {
    return sqrtf(1.0f - powf(beta2, (float)step)) / (1.0f - powf(beta1, (float)step));
}
__global__ void train_adam_corr_kernel(float* __restrict__ corr, uint32_t from, uint32_t to, float beta1, float beta2) {
    const uint32_t s = from + blockIdx.x * blockDim.x + threadIdx.x;
    if (s <= to) corr[s] = adam_corr(beta1, beta2, s);
}
// One parameter's update; `deb_old` / `deb_new` are the EMA debias terms 1 - decay^t, 1 - decay^(t+1) (uniform over the
// params: formed once per step on the host with the same powf the oracle uses)
__device__ __forceinline__ void adam_one(const AdamArgs& o, bool matrix, float gsum, float& w, float& m1, float& m2, uint32_t& step, float& e, bool& touched) {
    float gradient = gsum / o.loss_scale;
    touched = matrix || gradient != 0.0f;
    if (touched) {   // an untouched grid entry keeps its weight; the EMA still advances (tcnn EmaOptimizer steps every param)
        step += 1;
        if (matrix) gradient += o.l2_reg * w;
        const float gsq = gradient * gradient;
        m1 = o.beta1 * m1 + (1.0f - o.beta1) * gradient;
        m2 = o.beta2 * m2 + (1.0f - o.beta2) * gsq;
        // tcnn adam_step: learning_rate *= sqrtf(1 - beta2^t) / (1 - beta1^t) (the quotient first); the quotient from the
        // step-indexed table (train_adam_corr_kernel, the same expression), so no powf per parameter
        const float lr = o.lr * (step <= o.corr_n ? o.corr[step] : adam_corr(o.beta1, o.beta2, step));
        const float eff = lr / (sqrtf(m2) + o.epsilon);
        w = w - eff * m1;
    }
    e = (e * o.ema_decay * o.deb_old + w * (1.0f - o.ema_decay)) / o.deb_new;   // EMA with debiasing (tcnn EmaOptimizer)
}
// Four consecutive params per thread with 16-B loads / stores (8-B for the fp16 copies); the first-moment / second-moment /
// step arrays are read and written only for the groups that hold a touched param.  A group is all-matrix or all-grid
// (n_matrix % 4 == 0); n % 4 != 0 leaves a scalar tail.
__global__ __launch_bounds__(256) void train_adam_kernel(AdamArgs o, uint64_t n, uint32_t n_matrix, float* __restrict__ master,
                                                         const float* __restrict__ grads, float* __restrict__ m1, float* __restrict__ m2,
                                                         uint32_t* __restrict__ steps, float* __restrict__ ema, uint16_t* __restrict__ p_train,
                                                         uint16_t* __restrict__ p_infer) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = q * 4;
    if (i0 >= n) return;
    if (i0 + 4 > n) {   // scalar tail
        for (uint64_t i = i0; i < n; ++i) {
            float w = master[i], a = m1[i], b = m2[i], e = ema[i];
            uint32_t st = steps[i];
            bool touched;
            const float gi = (o.grads_h && i >= n_matrix) ? h2f(o.grads_h[i - n_matrix]) : grads[i];
            adam_one(o, i < n_matrix, gi, w, a, b, st, e, touched);
            if (touched) { master[i] = w; m1[i] = a; m2[i] = b; steps[i] = st; }
            ema[i] = e;
            p_train[i] = f2h(w);
            p_infer[i] = f2h(e);
        }
        return;
    }
    const bool matrix = i0 < n_matrix;
    float4 g;
    if (o.grads_h && !matrix) {   // four fp16 grid gradients (n_matrix % 4 == 0: 8-B aligned)
        const uint2 hg = *reinterpret_cast<const uint2*>(o.grads_h + (i0 - n_matrix));
        g = make_float4(h2f((uint16_t)(hg.x & 0xffffu)), h2f((uint16_t)(hg.x >> 16)), h2f((uint16_t)(hg.y & 0xffffu)), h2f((uint16_t)(hg.y >> 16)));
    } else {
        g = *reinterpret_cast<const float4*>(grads + i0);
    }
    float4 w = *reinterpret_cast<const float4*>(master + i0);
    float4 e = *reinterpret_cast<const float4*>(ema + i0);
    const bool any = matrix || g.x != 0.0f || g.y != 0.0f || g.z != 0.0f || g.w != 0.0f;
    float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = a;
    uint4 st = make_uint4(0u, 0u, 0u, 0u);
    if (any) {
        a = *reinterpret_cast<const float4*>(m1 + i0);
        b = *reinterpret_cast<const float4*>(m2 + i0);
        st = *reinterpret_cast<const uint4*>(steps + i0);
    }
    bool t0, t1, t2, t3;
    adam_one(o, matrix, g.x, w.x, a.x, b.x, st.x, e.x, t0);
    adam_one(o, matrix, g.y, w.y, a.y, b.y, st.y, e.y, t1);
    adam_one(o, matrix, g.z, w.z, a.z, b.z, st.z, e.z, t2);
    adam_one(o, matrix, g.w, w.w, a.w, b.w, st.w, e.w, t3);
    if (any) {   // untouched params of the group carry their loaded values back unchanged
        *reinterpret_cast<float4*>(master + i0) = w;
        *reinterpret_cast<float4*>(m1 + i0) = a;
        *reinterpret_cast<float4*>(m2 + i0) = b;
        *reinterpret_cast<uint4*>(steps + i0) = st;
    }
    *reinterpret_cast<float4*>(ema + i0) = e;
    const uint2 pt = make_uint2((uint32_t)f2h(w.x) | ((uint32_t)f2h(w.y) << 16), (uint32_t)f2h(w.z) | ((uint32_t)f2h(w.w) << 16));
    const uint2 pi = make_uint2((uint32_t)f2h(e.x) | ((uint32_t)f2h(e.y) << 16), (uint32_t)f2h(e.z) | ((uint32_t)f2h(e.w) << 16));
    *reinterpret_cast<uint2*>(p_train + i0) = pt;
    *reinterpret_cast<uint2*>(p_infer + i0) = pi;
}

// ---------------------------------------------------------------------------------------------
// density grid (update_density_grid_nerf, testbed_nerf.cu:3121-3210)
// ---------------------------------------------------------------------------------------------
// mark_untrained_density_grid (75-141): cells no training camera sees are -1
__global__ void train_mark_untrained_kernel(uint32_t n_elements, float* __restrict__ grid, TrainImages im, int clear_visible) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_elements) return;
    const uint32_t level = i / GRID_CELLS, pos_idx = i % GRID_CELLS;
    const uint32_t x = morton3D_invert(pos_idx >> 0), y = morton3D_invert(pos_idx >> 1), z = morton3D_invert(pos_idx >> 2);
    const float voxel_size = scalbnf(1.0f / (float)GRID_SIZE, (int)level);
    const f3 pos = (mk((float)x, (float)y, (float)z) / (float)GRID_SIZE - 0.5f) * scalbnf(1.0f, (int)level) + 0.5f;
    uint32_t count = 0;
    for (uint32_t j = 0; j < (uint32_t)im.n && count < 1; ++j) {
        const float* xf = im.xforms + 12 * j;
        const f3 c0 = mk(xf[0], xf[1], xf[2]), c1 = mk(xf[3], xf[4], xf[5]), c2 = mk(xf[6], xf[7], xf[8]), c3 = mk(xf[9], xf[10], xf[11]);
        const f2 focal = {im.focal[2 * j], im.focal[2 * j + 1]}, pp = {im.pp[2 * j], im.pp[2 * j + 1]};
        const int32_t lm = im.lens ? im.lens[j].mode : LENS_PERSPECTIVE;
        // F-Theta has no forward mapping and LatLong / Equirectangular see everything: counted as seeing the cell (116-121)
        if (lm == LENS_FTHETA || lm == LENS_LATLONG || lm == LENS_EQUIRECTANGULAR) { ++count; continue; }
        for (uint32_t k = 0; k < 8; ++k) {
            const f3 corner = pos + mk((k & 1) ? voxel_size : 0.0f, (k & 2) ? voxel_size : 0.0f, (k & 4) ? voxel_size : 0.0f);
            const f3 dir = normalize(corner - c3);
            if (dot(dir, c2) < 1e-4f) continue;
            // pos_to_uv (common_device.cuh:507-541): camera-space direction, the lens's forward distortion, project; then the
            // uv_to_ray round trip (through the Newton undistortion for OpenCV lenses)
            const f3 v = corner - c3;
            const f3 lc = mk(dot(v, c0), dot(v, c1), dot(v, c2));
            float px = lc.x / lc.z, py = lc.y / lc.z;
            if (lm != LENS_PERSPECTIVE) {
                float du, dv;
                lens_delta(lm, im.lens[j].params, px, py, du, dv);
                px += du;
                py += dv;
            }
            const f2 uv = {px * focal.x / (float)im.w + pp.x, py * focal.y / (float)im.h + pp.y};
            f3 dl = mk((uv.x - pp.x) * (float)im.w / focal.x, (uv.y - pp.y) * (float)im.h / focal.y, 1.0f);
            if (lm != LENS_PERSPECTIVE) lens_undistort(lm, im.lens[j].params, dl.x, dl.y);
            const f3 rd = normalize(c0 * dl.x + c1 * dl.y + c2 * dl.z);
            if (length(rd - dir) < 1e-3f && uv.x > 0.0f && uv.y > 0.0f && uv.x < 1.0f && uv.y < 1.0f) { ++count; break; }
        }
    }
    if (clear_visible || (grid[i] < 0) != (count < 1)) grid[i] = count >= 1 ? 0.0f : -1.0f;
}

// generate_grid_samples_nerf_nonuniform (186-215): NerfPosition written as a 7-float coordinate
// (direction unused by the density output)
// morton (n_elements a multiple of GRID_CELLS, as in the uniform updates of the first 256 steps): slot t holds the sample
// i whose first candidate cell is the t-th cell in Morton order (its hashed index is an affine bijection of i mod
// GRID_CELLS: i = (f - 96925573) * 56924617^-1 - step n mod 2^21), so the network reads neighbouring cells' hash
// entries together instead of one random cell per lane; the samples, and the splat's max per cell, are the same
__global__ void train_grid_samples_kernel(uint32_t n_elements, Pcg32 rng, uint32_t step, aabb box, const float* __restrict__ grid_in, float* __restrict__ coords,
                                          uint32_t* __restrict__ indices, uint32_t n_cascades, float thresh, int morton) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_elements) return;
    static_assert(GRID_CELLS == (1u << 21), "the affine inverse below is mod 2^21");
    const uint32_t i = morton ? (t & ~(GRID_CELLS - 1u)) | ((((t & (GRID_CELLS - 1u)) - 96925573u) * 53369u - step * n_elements) & (GRID_CELLS - 1u)) : t;
    rng.advance((uint64_t)i * 4);
    const uint32_t level = (uint32_t)(rng.next_float() * (float)n_cascades) % n_cascades;
    uint32_t idx = 0;
    for (uint32_t j = 0; j < 10; ++j) {
        idx = ((i + step * n_elements) * 56924617u + j * 19349663u + 96925573u) % GRID_CELLS;
        idx += level * GRID_CELLS;
        if (grid_in[idx] > thresh) break;
    }
    const uint32_t pos_idx = idx % GRID_CELLS;
    const uint32_t x = morton3D_invert(pos_idx >> 0), y = morton3D_invert(pos_idx >> 1), z = morton3D_invert(pos_idx >> 2);
    const float rx = rng.next_float(), ry = rng.next_float(), rz = rng.next_float();
    const f3 pos = ((mk((float)x, (float)y, (float)z) + mk(rx, ry, rz)) / (float)GRID_SIZE - 0.5f) * scalbnf(1.0f, (int)level) + 0.5f;
    const f3 wp = (pos - box.lo) / (box.hi - box.lo);
    float* c = coords + (size_t)t * 7;
    c[0] = wp.x; c[1] = wp.y; c[2] = wp.z; c[3] = warp_dt(MIN_STEP); c[4] = 0.5f; c[5] = 0.5f; c[6] = 0.5f;
    indices[t] = idx;
}

// splat_grid_samples_nerf_max_nearest_neighbor (217-233): optical thickness, atomic max on the bits
__global__ void train_grid_splat_kernel(uint32_t n, const uint32_t* __restrict__ indices, const uint16_t* __restrict__ out4, float* __restrict__ tmp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float mlp = sng_expf(h2f(out4[(size_t)i * 4 + 3]));
    const float ot = mlp * MIN_STEP;
    atomicMax(reinterpret_cast<uint32_t*>(&tmp[indices[i]]), __float_as_uint(ot));
}

// ema_grid_samples_nerf (254-275): max(prev * decay, new), negative (untrained) cells stay
__global__ void train_grid_ema_kernel(uint32_t n, float decay, float* __restrict__ grid, const float* __restrict__ tmp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float prev = grid[i];
    grid[i] = prev < 0.0f ? prev : fmaxf(prev * decay, tmp[i]);
}



// the per-ray buffers the step fills by ray index, cleared up to the device's ray count
__global__ __launch_bounds__(256) void train_clear_kernel(const TrainSched* __restrict__ sched, float* __restrict__ loss, float4* __restrict__ rayrec,
                                                          uint32_t* __restrict__ cnt, TrainCtrl* __restrict__ ctrl) {
    const uint32_t n = sched->n_rays;
    if (blockIdx.x == 0 && threadIdx.x == 0) *ctrl = TrainCtrl{0u, 0u, 0u, 0u};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < 3 * n; i += gridDim.x * blockDim.x) {
        rayrec[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (i < n) { loss[i] = 0.0f; cnt[i] = 0u; }
    }
}

// ---------------------------------------------------------------------------------------------
void launch_train_clear(const TrainStepArgs& a, const TrainBatch& b, hipStream_t s) {
    hipLaunchKernelGGL(train_clear_kernel, dim3(std::max(1u, (3 * a.n_rays_grid + 255) / 256)), dim3(256), 0, s, a.sched, b.loss, b.rayrec, b.cnt_i, b.ctrl);
}
void launch_train_generate(const TrainStepArgs& a, const TrainImages& im, const TrainBatch& b, Pcg32 rng, float* tscr, hipStream_t s) {
    const dim3 grid(std::max(1u, (a.n_rays_grid + 63) / 64));
    const bool lin = a.vol.linear && a.vol.max_mip == 0 && a.vol.cone <= 1e-5f;
    if (a.gen_bricks && lin && a.vol.occ_brick_words && a.vol.occ_brick_words * 4u <= 64u * 1024u)
        hipLaunchKernelGGL((train_generate_kernel<1, true>), grid, dim3(64), a.vol.occ_brick_words * 4, s, a, im, b, rng, tscr);
    else if (a.gen_bricks && lin && a.vol.occ_brick_g)
        hipLaunchKernelGGL((train_generate_kernel<2, true>), grid, dim3(64), 0, s, a, im, b, rng, tscr);
    else if (a.gen_lanes == 8 || a.gen_lanes == 16) {
        const dim3 g2(std::max(1u, (a.n_rays_grid * (uint32_t)a.gen_lanes + 63) / 64));
        if (lin && a.vol.occ_linear) {
            if (a.gen_lanes == 8) hipLaunchKernelGGL((train_generate_spec_kernel<true, 8>), g2, dim3(64), 0, s, a, im, b, rng, tscr);
            else hipLaunchKernelGGL((train_generate_spec_kernel<true, 16>), g2, dim3(64), 0, s, a, im, b, rng, tscr);
        } else {
            if (a.gen_lanes == 8) hipLaunchKernelGGL((train_generate_spec_kernel<false, 8>), g2, dim3(64), 0, s, a, im, b, rng, tscr);
            else hipLaunchKernelGGL((train_generate_spec_kernel<false, 16>), g2, dim3(64), 0, s, a, im, b, rng, tscr);
        }
    } else if (lin && a.vol.occ_linear)
        hipLaunchKernelGGL((train_generate_kernel<0, true>), grid, dim3(64), 0, s, a, im, b, rng, tscr);
    else
        hipLaunchKernelGGL((train_generate_kernel<0, false>), grid, dim3(64), 0, s, a, im, b, rng, tscr);
}
void launch_train_loss(const TrainStepArgs& a, const TrainImages& im, const TrainBatch& b, Pcg32 rng, const float* mean_density, TrainSched* sched_next,
                       hipStream_t s) {
    // rayrec, cnt_i and loss were cleared at the start of the step (launch_train_clear)
    const uint32_t n = std::max(1u, a.n_rays_grid);
    hipLaunchKernelGGL(train_loss_kernel, dim3((n * LOSS_G + 255) / 256), dim3(256), 0, s, a, im, b, rng, mean_density);
    hipLaunchKernelGGL(train_compact_kernel, dim3(1), dim3(1024), 0, s, a.sched, b.cnt_i, b.cbase_i, b.ctrl);
    hipLaunchKernelGGL(train_dloss_kernel, dim3((n + 3) / 4), dim3(256), 0, s, a, b);
    hipLaunchKernelGGL(train_rollover_kernel, dim3((a.target_batch + 255) / 256), dim3(256), 0, s, a, b, sched_next);
}
void launch_train_pack(const uint16_t* params, uint16_t* wfrag, uint16_t* wfrag_t, hipStream_t s, const uint32_t* clamp_in, const TrainSched* sched,
                       uint32_t* clamp_out) {
    hipLaunchKernelGGL(train_pack_kernel, dim3(56), dim3(64), 0, s, params, wfrag, wfrag_t, clamp_in, sched, clamp_out);
}
void launch_train_field(const TrainStepArgs& a, const TrainBatch& b, const NetworkDev& net, const uint16_t* wfrag, const uint16_t* wfrag_t,
                        const uint16_t* grid, float* ggrad, uint16_t* ggrad_h, hipStream_t s) {
    const uint32_t tiles = (a.target_batch + 15) / 16;
    const uint32_t waves = std::min<uint32_t>(tiles, (uint32_t)net.n_cus * 8u);
    const uint32_t blocks = (waves + 3) / 4;
    const h8* w = reinterpret_cast<const h8*>(wfrag);
    const h4v* wt = reinterpret_cast<const h4v*>(wfrag_t);
    const _Float16* gr = reinterpret_cast<const _Float16*>(grid);
    if (net.F == 4 && ggrad_h) hipLaunchKernelGGL((train_field_kernel<4, true>), dim3(blocks), dim3(256), 0, s, a, b, w, wt, gr, net.levels, ggrad, ggrad_h);
    else if (net.F == 4) hipLaunchKernelGGL((train_field_kernel<4>), dim3(blocks), dim3(256), 0, s, a, b, w, wt, gr, net.levels, ggrad, ggrad_h);
    else hipLaunchKernelGGL((train_field_kernel<2>), dim3(blocks), dim3(256), 0, s, a, b, w, wt, gr, net.levels, ggrad, ggrad_h);
}
void launch_train_dw(const TrainStepArgs& a, const uint16_t* acts, float* wgrad, uint32_t n_cus, hipStream_t s) {
    const uint32_t tiles = (a.target_batch + 15) / 16;
    const uint32_t blocks_target = n_cus * (uint32_t)std::max(1, a.dw_blocks_per_cu);
    const uint32_t per = std::max<uint32_t>(8, (tiles + blocks_target - 1) / blocks_target);
    if (a.dw_pipe) hipLaunchKernelGGL(train_dw_kernel<true>, dim3((tiles + per - 1) / per), dim3(320), 0, s, a, acts, per, wgrad);
    else hipLaunchKernelGGL(train_dw_kernel<false>, dim3((tiles + per - 1) / per), dim3(320), 0, s, a, acts, per, wgrad);
}
void launch_train_adam(const AdamArgs& o, uint64_t n, uint32_t n_matrix, float* master, const float* grads, float* m1, float* m2, uint32_t* steps, float* ema,
                       uint16_t* p_train, uint16_t* p_infer, hipStream_t s) {
    const uint64_t groups = (n + 3) / 4;   // every buffer is a hipMalloc allocation (16-B aligned); n_matrix % 4 == 0
    hipLaunchKernelGGL(train_adam_kernel, dim3((uint32_t)((groups + 255) / 256)), dim3(256), 0, s, o, n, n_matrix, master, grads, m1, m2, steps, ema,
                       p_train, p_infer);
}
void launch_train_adam_corr(float* corr, uint32_t from, uint32_t to, float beta1, float beta2, hipStream_t s) {
    if (to < from) return;
    const uint32_t n = to - from + 1;
    hipLaunchKernelGGL(train_adam_corr_kernel, dim3((n + 255) / 256), dim3(256), 0, s, corr, from, to, beta1, beta2);
}
void launch_train_mark_untrained(uint32_t n, float* grid, const TrainImages& im, int clear_visible, hipStream_t s) {
    hipLaunchKernelGGL(train_mark_untrained_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, grid, im, clear_visible);
}
void launch_train_grid_samples(uint32_t n, Pcg32 rng, uint32_t step, const aabb& box, const float* grid, float* coords, uint32_t* indices, uint32_t n_cascades,
                               float thresh, int morton, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(train_grid_samples_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, rng, step, box, grid, coords, indices, n_cascades, thresh,
                       morton && n % GRID_CELLS == 0 ? 1 : 0);
}
void launch_train_grid_splat_ema(uint32_t n_samples, const uint32_t* indices, const uint16_t* out4, float* tmp, uint32_t n_cells, float decay, float* grid,
                                 hipStream_t s) {
    hipLaunchKernelGGL(train_grid_splat_kernel, dim3((n_samples + 255) / 256), dim3(256), 0, s, n_samples, indices, out4, tmp);
    hipLaunchKernelGGL(train_grid_ema_kernel, dim3((n_cells + 255) / 256), dim3(256), 0, s, n_cells, decay, grid, tmp);
}

}  // namespace sng
