// train.h -- device structs and helpers of the online training step (train.hip, host_train.cpp)
#pragma once
#include "sng_internal.h"
#include "sng_math.h"

namespace sng {

constexpr uint32_t N_MAX_RANDOM_SAMPLES_PER_RAY = 16;   // nerf_device.cuh:40
constexpr float NERF_MIN_OPTICAL_THICKNESS = 0.01f;      // nerf_device.cuh:43
constexpr uint32_t BATCH_SIZE_GRANULARITY = 256;         // tcnn

// tcnn pcg32 (random.h; M. O'Neill's PCG32 XSH-RR, Wenzel Jakob's pcg32.h) -- restated
struct Pcg32 {
    uint64_t state, inc;
    static constexpr uint64_t MULT = 0x5851f42d4c957f2dULL;
    SNG_HD static Pcg32 seeded(uint64_t initstate, uint64_t initseq = 1u) {
        Pcg32 r{0u, (initseq << 1u) | 1u};
        r.next_uint();
        r.state += initstate;
        r.next_uint();
        return r;
    }
    SNG_HD uint32_t next_uint() {
        const uint64_t old = state;
        state = old * MULT + inc;
        const uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    SNG_HD float next_float() {
        const uint32_t u = (next_uint() >> 9) | 0x3f800000u;
        float f;
        __builtin_memcpy(&f, &u, 4);
        return f - 1.0f;
    }
    // multi-step advance in O(log n) (Brown, "Random number generation with arbitrary stride")
    SNG_HD void advance(uint64_t delta = (1ull << 32)) {
        uint64_t cur_mult = MULT, cur_plus = inc, acc_mult = 1u, acc_plus = 0u;
        while (delta > 0) {
            if (delta & 1) {
                acc_mult *= cur_mult;
                acc_plus = acc_plus * cur_mult + cur_plus;
            }
            cur_plus = (cur_mult + 1) * cur_plus;
            cur_mult *= cur_mult;
            delta /= 2;
        }
        state = acc_mult * state + acc_plus;
    }
};

SNG_HD float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
SNG_HD uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// training images (NerfDataset after load: RGBA8 sRGB, cameras in NGP space)
struct TrainImages {
    const uint32_t* pixels;   // [n][h][w] RGBA8 (0x00FF00FF = masked)
    const float* xforms;      // [n][12]: camera columns c0 c1 c2 c3 (mat4x3)
    const float* xforms_ray;  // the same after get_xform_given_rolling_shutter's quat round trip (ray generation)
    const float* focal;       // [n][2] pixels
    const float* pp;          // [n][2] principal point (uv)
    const Lens* lens;         // [n] dataset lens per image (read_lens, nerf_loader.cu:175-239); nullptr: every image Perspective
    int w, h, n;
};

// read_rgba (common_device.cuh:803-835), Byte images: premultiplied linear
SNG_HD float4 read_rgba(const TrainImages& im, uint32_t img, f2 uv) {
    int px = (int)(uv.x * (float)im.w), py = (int)(uv.y * (float)im.h);
    px = px < 0 ? 0 : (px > im.w - 1 ? im.w - 1 : px);
    py = py < 0 ? 0 : (py > im.h - 1 ? im.h - 1 : py);
    const uint32_t v = im.pixels[(size_t)img * im.w * im.h + (size_t)py * im.w + px];
    if (v == 0x00FF00FFu) return make_float4(-1.0f, -1.0f, -1.0f, -1.0f);
    const float alpha = (float)(v >> 24) * (1.0f / 255.0f);
    return make_float4(srgb_to_linear((float)(v & 0xFF) * (1.0f / 255.0f)) * alpha, srgb_to_linear((float)((v >> 8) & 0xFF) * (1.0f / 255.0f)) * alpha,
                       srgb_to_linear((float)((v >> 16) & 0xFF) * (1.0f / 255.0f)) * alpha, alpha);
}

// nerf_random_image_pos_training (nerf_device.cuh:553-576), snap_to_pixel_centers, no CDF
SNG_HD f2 train_image_pos(Pcg32& rng, const TrainImages& im) {
    const float u = rng.next_float(), v = rng.next_float();
    int px = (int)(u * (float)im.w), py = (int)(v * (float)im.h);
    px = px < 0 ? 0 : (px > im.w - 1 ? im.w - 1 : px);
    py = py < 0 ? 0 : (py > im.h - 1 ? im.h - 1 : py);
    return {((float)px + 0.5f) / (float)im.w, ((float)py + 0.5f) / (float)im.h};
}

// n items per lane reserved from one counter with ONE atomic per wave (every lane of the wave must be active): the
// lane's exclusive prefix within the wave plus the wave's base.  The reference reserves per thread
// (testbed_nerf.cu:956-963, 1150); the batch order of the atomics is arbitrary in both, and ~20 K single-word atomics per
// batch serialise at ~90 per us (MI355X_MICROARCH.md, dequeue).
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* counter, uint32_t n, int lane) {
    uint32_t incl = n;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    uint32_t base = 0;
    if (lane == 63 && total) base = atomicAdd(counter, total);
    base = __shfl(base, 63, 64);
    return base + incl - n;
}

struct TrainRay { f3 o, d; };
// uv_to_ray (common_device.cuh:403-470) with the image's lens (testbed_nerf.cu:890-905), no parallax / aperture / near
// distance / distortion map; an invalid ray (F-Theta outside its domain) becomes {xform[3], xform[2]} (testbed_nerf.cu:901-903)
SNG_HD TrainRay train_ray(const TrainImages& im, uint32_t img, f2 uv) {
    const float* xf = im.xforms_ray + 12 * img;
    const m3 rot = {mk(xf[0], xf[1], xf[2]), mk(xf[3], xf[4], xf[5]), mk(xf[6], xf[7], xf[8])};
    const f2 pp = {im.pp[2 * img], im.pp[2 * img + 1]}, focal = {im.focal[2 * img], im.focal[2 * img + 1]};
    f3 dir;
    if (!im.lens || im.lens[img].mode == LENS_PERSPECTIVE)
        dir = mk((uv.x - pp.x) * (float)im.w / focal.x, (uv.y - pp.y) * (float)im.h / focal.y, 1.0f);
    else if (!lens_dir(im.lens[img], uv, pp, im.w, im.h, focal, dir))
        return {mk(xf[9], xf[10], xf[11]), rot.c2};
    return {mk(xf[9], xf[10], xf[11]), mul(rot, dir)};
}

// mip_from_dt (nerf_device.cuh:450-460)
SNG_HD uint32_t mip_from_dt(float dt, f3 pos, uint32_t max_cascade) {
    const uint32_t mip = mip_from_pos(pos, max_cascade);
    dt *= 2.0f * (float)GRID_SIZE;
    if (dt < 1.0f) return mip;
    int exponent;
    frexpf(dt, &exponent);
    int r = (int)mip < exponent ? exponent : (int)mip;
    return (uint32_t)(r > (int)max_cascade ? (int)max_cascade : r);
}

struct TrainCtrl {
    uint32_t ray_counter;
    uint32_t numsteps_counter;
    uint32_t numsteps_compacted;
    uint32_t pad;
};

// NerfCounters' batch sizes (testbed_nerf.cu:3272-3296), kept on the device: the step's kernels read them, and
// train_rollover_kernel forms the next step's from the step's counters, so the host never waits for a step
struct TrainSched {
    uint32_t n_rays;            // rays_per_batch
    uint32_t max_samples;       // max_inference (from measured_before)
    uint32_t measured;          // measured_batch_size (after compaction)
    uint32_t measured_before;   // measured_batch_size_before_compaction
};

struct TrainStepArgs {
    Volume vol;              // train_aabb, bitfield, max_mip, cone
    const TrainSched* sched; // this step's n_rays / max_samples (device)
    uint32_t n_rays_grid;    // the host's estimate of n_rays: grid sizes only (the kernels loop over the device count)
    uint32_t target_batch;   // m_training_batch_size
    int random_bg;
    f3 background;
    float loss_scale;        // LOSS_SCALE() = 128 for fp16
    float near_distance;     // 0.1
    int debug;               // generate: per-ray step count / entry distances into loss / coords_c
    int gen_bricks;          // generate's unit-cube occupancy source: 1 bricks (LDS when staged, else global), 0 linear words
    int gen_lanes;           // lanes per ray of the generator's speculative march (8, 16; else one lane per ray)
    int dw_pipe;             // dW kernel: 1 = the next tile's operands loaded while the current tile's MFMAs run
    int dw_blocks_per_cu;    // dW kernel: workgroups per CU (each adds its partial sums to the gradient once)
    int grid_grad_f16;       // hash-grid gradients accumulated in fp16 with packed atomics (tcnn's grad_t = __half), else f32
};

// per-batch buffers
struct TrainBatch {
    TrainCtrl* ctrl;
    uint32_t* ray_indices;   // [n_rays]
    float4* rays;            // [n_rays][2] origin, unnormalized direction
    uint2* numsteps;         // [n_rays] {numsteps, base}
    float* coords;           // [max_samples][7]
    uint16_t* mlp_out;       // [max_samples][4] fp16
    float* coords_c;         // [target][7] compacted
    uint16_t* dloss;         // [target][4] fp16
    float* loss;             // [n_rays]
    uint16_t* acts;          // [target/16][TRAIN_FEATS][16] fp16
    float4* partial;         // [max_samples] {T before the sample, running rgb after it} (train_loss_kernel)
    float4* rayrec;          // [n_rays][3] {cbase, ccount, base, -} {grad, loss_scale} {rgb_ray, l1_reg} (train_dloss_kernel)
    uint32_t* cnt_i;         // [n_rays] composited samples per ray, by the ray's image index (train_compact_kernel)
    uint32_t* cbase_i;       // [n_rays] its compaction slot (exclusive prefix of cnt_i)
};

// feature rows of the tiled activation / gradient buffer
constexpr int A_ENC = 0, A_H0 = 32, A_RIN = 96, A_H1 = 128, A_H2 = 192, D_O = 256, D_H2 = 272, D_H1 = 336, D_DENS = 400, D_H0 = 416;
constexpr int TRAIN_FEATS = 480;

struct AdamArgs {
    float lr, beta1, beta2, epsilon, l2_reg, loss_scale, ema_decay;
    uint32_t ema_step;
    float deb_old, deb_new;   // 1 - ema_decay^ema_step, 1 - ema_decay^(ema_step + 1) (host powf, as the oracle)
    const float* corr;        // [corr_n + 1] Adam's bias correction sqrtf(1 - beta2^s) / (1 - beta1^s) for s = 1..corr_n
    uint32_t corr_n;
    const uint16_t* grads_h;  // fp16 grid gradients (param index - n_matrix), nullptr: every gradient in `grads`
};

// zero loss / rayrec / cnt_i for the step's rays (device count)
void launch_train_clear(const TrainStepArgs& a, const TrainBatch& b, hipStream_t s);
// tscr: [NERF_STEPS][n_rays] floats of scratch (the first march's sample distances)
void launch_train_generate(const TrainStepArgs& a, const TrainImages& im, const TrainBatch& b, Pcg32 rng, float* tscr, hipStream_t s);
// sched_next: the next step's batch sizes formed at the end of the stage (NerfCounters::update_after_training); null in the parity hooks
void launch_train_loss(const TrainStepArgs& a, const TrainImages& im, const TrainBatch& b, Pcg32 rng, const float* mean_density, TrainSched* sched_next,
                       hipStream_t s);
// clamp_in / sched / clamp_out: also *clamp_out = min(*clamp_in, sched->max_samples) (the training step's network count)
void launch_train_pack(const uint16_t* params, uint16_t* wfrag, uint16_t* wfrag_t, hipStream_t s, const uint32_t* clamp_in = nullptr,
                       const TrainSched* sched = nullptr, uint32_t* clamp_out = nullptr);
void launch_train_field(const TrainStepArgs& a, const TrainBatch& b, const NetworkDev& net, const uint16_t* wfrag, const uint16_t* wfrag_t,
                        const uint16_t* grid, float* ggrad, uint16_t* ggrad_h, hipStream_t s);
void launch_train_dw(const TrainStepArgs& a, const uint16_t* acts, float* wgrad, uint32_t n_cus, hipStream_t s);
void launch_train_adam(const AdamArgs& o, uint64_t n, uint32_t n_matrix, float* master, const float* grads, float* m1, float* m2, uint32_t* steps, float* ema,
                       uint16_t* p_train, uint16_t* p_infer, hipStream_t s);
// Adam's bias-correction factor for the per-parameter step counts s = from..to (the expression adam_one would form)
void launch_train_adam_corr(float* corr, uint32_t from, uint32_t to, float beta1, float beta2, hipStream_t s);
void launch_train_mark_untrained(uint32_t n, float* grid, const TrainImages& im, int clear_visible, hipStream_t s);
// morton: slots in the Morton order of the samples' first candidate cells when n is a multiple of GRID_CELLS
void launch_train_grid_samples(uint32_t n, Pcg32 rng, uint32_t step, const aabb& box, const float* grid, float* coords, uint32_t* indices, uint32_t n_cascades,
                               float thresh, int morton, hipStream_t s);
void launch_train_grid_splat_ema(uint32_t n_samples, const uint32_t* indices, const uint16_t* out4, float* tmp, uint32_t n_cells, float decay, float* grid,
                                 hipStream_t s);

}  // namespace sng
