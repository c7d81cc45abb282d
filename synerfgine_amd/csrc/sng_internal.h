// sng_internal.h -- device-side data layout shared by the host runtime and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

#include "../../include/sng.h"

#include "sng_math.h"

namespace sng {

// Per-level hash-grid metadata (tcnn GridOffsetTable + grid_scale/grid_resolution).
struct LevelInfo {
    uint32_t offset;     // first entry of the level
    uint32_t size;       // hashmap_size (entries)
    uint32_t pow2_mask;  // size-1 if size is a power of two, else 0
    uint32_t dense;      // 1 if the tcnn stride loop keeps the dense index
    uint32_t res;        // grid_resolution(scale)
    uint32_t res2;       // res*res (dense index)
    float scale;         // grid_scale(level)
    uint32_t pad;
};

struct NetworkDev {
    int F = 4, L = 8;
    int n_cus = 256;
    void* wfrag = nullptr;      // 20 fragments x 64 lanes x 8 halves (MFMA A operands, permuted k)
    void* grid = nullptr;       // fp16 grid params (entries x F)
    LevelInfo* levels = nullptr;
};

// Wavefront control block (device), ping-pong by iteration parity.
struct MarchCtrl {
    uint32_t n_alive[2];
    uint32_t n_owned[2];      // alive rays of the band's own rows (Sched::own_lo/hi), counted when Sched::global
    uint32_t sched_alive[2];  // frame-wide alive count (sum of n_owned over ranks) the step schedule uses
    uint32_t n_samples[2];    // network samples of the iteration (appended by generate)
    uint32_t n_reused[2];     // boundary samples of the iteration that reuse the previous iteration's output
    uint32_t i_step[2];
    uint32_t n_hit;
    uint32_t n_iter;
    unsigned long long total_samples;
    unsigned long long net_samples;   // samples of the whole-GPU network launches (the rest ran in the fused tail)
    unsigned long long ref_slots;
    unsigned long long reused_samples;   // march samples taken from the ray's cached output (no network evaluation)
    uint32_t alive_hist[64];
    uint32_t steps_hist[64];
    uint32_t samples_hist[64];
    // speculative tail rounds (nerf.hip spec_generate / spec_composite), per ping-pong buffer
    uint32_t spec_K[2];       // iterations the round marched ahead
    uint32_t spec_k0[2];      // iteration index of the round's first iteration
    unsigned long long spec_evals;   // samples the rounds' network launches evaluated (incl. those past a ray's end)
    unsigned long long spec_exec;    // ... of which composited
    uint32_t spec_base_k;            // iteration index and trace_alt step counter i at the tail's start: a ray at
    uint32_t spec_base_istep;        //   iteration k has i = base_istep + 8 (k - base_k)
    uint32_t spec_kk_valid[2];       // RayBuf::kk of buffer p holds per-ray iteration indices
    uint32_t spec_ok;                // tail_prepare: every later iteration takes 8 steps (else the tail kernels queued
                                     // ahead of that check leave every buffer untouched and the wavefront continues)
    uint32_t spec_round_samples[4];  // network samples of the frame's speculative rounds 0..3 (spec_composite; sizes the next
                                     //   frame's round count, nerf_spec_adapt)
    uint32_t fused_rays_in;          // rays the fused tail kernel took over (after the rounds)
    // multi-step speculative rounds (nerf.hip msr_*), per ping-pong buffer of the round's rays
    uint32_t msr_S[2];               // steps the round's first iteration takes (0: the round is a no-op)
    uint32_t msr_K[2];               // iterations the round marched ahead
    uint32_t msr_J;                  // iterations the last round commits (msr_schedule)
    uint8_t msr_Sv[2][16];           // steps of each of the round's K iterations (MSR_KMAX; from the last frame's schedule)
    unsigned long long msr_evals;    // samples the rounds' network launches evaluated
    unsigned long long msr_exec;     // ... of which the wavefront would have evaluated (the committed iterations')
    int32_t* tail_live;              // [TAIL_LIVE_CAP] the tail's alive rays per iteration as a difference array (+1 where a
                                     //   ray enters the tail's bookkeeping, -1 after its last iteration): reference slots
    uint8_t* sched_hint;             // [TAIL_LIVE_CAP] steps of every iteration of the last frame (0: unknown), written by the
                                     //   wavefront, one-step and msr schedules; sizes the msr rounds (exact for any value)
    uint32_t* log;                   // diagnostics (param march_log): [MARCH_LOG_CAP][3] {alive, steps, samples} per iteration
    uint32_t net_launch_samples[16]; // sample count each whole-GPU network launch of the frame read (collect_kernel_times;
                                     //   indexed like the host's launch events: the per-launch roofline)
};
constexpr uint32_t MARCH_LOG_CAP = 2048;
constexpr uint32_t TAIL_LIVE_CAP = 10240;   // > MARCH_ITER: iterations a frame can have

// Alive-ray SoA buffer (NerfPayload + rgba + depth, nerf_device.cuh:145-153; nerf.h:22-42)
struct RayBuf {
    float4* o_t;       // origin.xyz, t
    float4* d_idx;     // dir.xyz, pixel index (bits)
    float4* rgba;
    float* depth;
    float* mw;         // payload.max_weight (instant-NGP trace path only)
    // trace_alt boundary-sample cache: the t reset (composite_kernel_nerf_alt:574) makes the next
    // iteration's first sample the previous iteration's last one, bit for bit in the common case.
    float2* lt;        // x: t of the previous iteration's last sample (NaN: none); y: this iteration's (generate)
    uint2* lo;         // raw fp16 (r, g, b, density) network output of that sample
    uint32_t* kk;      // speculative tail: the ray's next iteration index (rays of one buffer may differ once the
                       // rounds look ahead per ray; MarchCtrl::spec_kk_valid says whether this buffer's are set)
};

// atomicAdd(&arr[key], v) from every lane with on == true, as one atomic per distinct key of the wave (same-address
// atomics from many lanes serialise).  v is the same on every lane; call with the whole wave converged.
__device__ __forceinline__ void wave_add_keyed(int32_t* arr, uint32_t key, int32_t v, bool on) {
    const int lane = (int)(threadIdx.x & 63u);
    unsigned long long pend = __ballot(on);
    while (pend) {
        const int leader = __ffsll((long long)pend) - 1;
        const uint32_t lk = __shfl(key, leader, 64);
        const unsigned long long m = pend & __ballot(key == lk);
        if (lane == leader) atomicAdd(&arr[lk], (int32_t)__popcll(m) * v);
        pend &= ~m;
    }
}

// n_steps_between_compaction = clamp(target / n_alive, 1, 8) (testbed_nerf.cu:2189-2190)
SNG_HD uint32_t steps_for(uint32_t n_alive, uint32_t target) {
    const uint32_t s = target / n_alive;
    return s < 1 ? 1 : (s > MAX_STEPS_BETWEEN_COMPACTION ? MAX_STEPS_BETWEEN_COMPACTION : s);
}

// Which NeRF tracer runs: SyNeRFgine's trace_alt (ngp = 0: depth of the last sample,
// payload.t reset to it, extract_from_payload) or instant-NGP's trace (ngp = 1: depth of the
// max-weight sample, no t reset, shade_kernel_nerf with ERenderMode render_mode).
struct TraceMode {
    int ngp;
    int render_mode;     // ERenderMode: 0 AO, 1 Shade, 3 Positions, 4 Depth, 6 Cost, 10 EncodingVis
    float depth_scale;   // 1 / dataset.scale
    int glow_mode;       // Testbed::Nerf::glow_mode / glow_y_cutoff (testbed.h:870-871), instant-NGP path only
    float glow_y_cutoff;
};

struct CamDev {
    f3 c0, c1, c2, c3;   // mat4x3 columns (right, down, fwd, position)
};

// Step schedule of a band: n_steps = clamp(target / n_alive, 1, 8) uses the
// FRAME-wide alive count (testbed_nerf.cu:2189-2190).  global = 1: the kernels read
// MarchCtrl::sched_alive (the sum over ranks of the rays alive in each band's own rows, pixel
// indices [own_lo, own_hi)), so every band marches with the single-GPU schedule.
struct Sched {
    int global;
    uint32_t own_lo, own_hi;
};

struct NerfFrameArgs {
    Volume vol;
    CamDev cam;          // camera0 (composite/extract)
    q4 q0, q1;           // quat_cast of camera0 / camera1 (get_xform_given_rolling_shutter, common_device.cuh:361-368)
    f3 pos1;             // camera1 position (camera0's: cam.c3)
    float rolling_shutter[4];
    Lens lens;           // uv_to_ray's lens (Perspective unless render_with_lens_distortion)
    f2 focal;
    f2 screen_center;
    int W, H;            // full NeRF resolution (pixel indices are global)
    int row0, row1;      // rows traced for this band
    uint32_t spp;
    int snap;
    int reset;           // clear alpha of the frame buffer (camera moved)
    uint32_t target_n_queries;
    TraceMode mode;
    Sched sched;
};

// fused.hip: ray-local NeRF wavefront (generate + field + composite in one persistent kernel)
struct FusedArgs {
    Volume vol;
    CamDev cam;
    TraceMode mode;
    RayBuf rays;                  // initial alive rays (init_rays_kernel output), count = ctrl->n_alive[0]
    MarchCtrl* ctrl;
    const void* wfrag;            // MFMA weight fragments (NetworkDev::wfrag)
    const void* grid_params;      // fp16 hash grid
    const LevelInfo* levels;
    float4* frame_rgba;
    float* frame_depth;
    float* positions;
    uint32_t* work;               // ray-queue cursor (zeroed by the launcher)
    int p;                        // ping-pong buffer holding the alive rays (MarchCtrl::n_alive[p], i_step[p])
    uint32_t lanes;               // rays per wave (64; fewer shorten a wave's per-iteration field chain for thin bands)
    uint8_t* hint;                // SpecArgs::hint, written when a ray ends here (nullptr: off)
};
void launch_nerf_fused(const FusedArgs& a, const NetworkDev& net, uint32_t n_rays_hint, uint32_t max_blocks, hipStream_t s, bool prepare = true);

// fused.hip: trace_alt's one-step regime (n_alive > target / 2, so every iteration takes ONE step).
// A speculative ray-local pass simulates each ray on its own under n_steps = 1 and histograms the
// iteration at which it leaves; the schedule kernel finds the first iteration k + J whose frame-wide
// alive count allows more steps; the final pass re-simulates every ray to k + J and writes the
// survivors to the other ray buffer (dying rays are extracted on the way).
constexpr uint32_t ONESTEP_HIST = 10240;   // >= MARCH_ITER: iterations a regime can span
struct OnestepState {
    uint32_t k;             // first iteration of the regime
    uint32_t istep0;        // trace_alt's i at k
    uint32_t n_local;       // rays of this band alive at k
    uint32_t n_sched;       // frame-wide alive count at k (the schedule's)
    uint32_t H;             // iterations the histograms span (MARCH_ITER - istep0, capped at the horizon)
    uint32_t J;             // iterations the regime lasts (schedule kernel)
    uint32_t work[2];       // ray-queue cursors of the two passes
    unsigned long long evals[2];   // field evaluations of the two passes
};
struct OnestepArgs {
    Volume vol;
    CamDev cam;
    Sched sched;
    RayBuf in, out;               // rays alive at k (buffer p) -> rays alive at k + J (buffer p ^ 1)
    MarchCtrl* ctrl;
    OnestepState* os;
    uint32_t* deaths_local;       // [ONESTEP_HIST] rays alive at k + m but not at k + m + 1
    uint32_t* deaths_sched;       // the same, own rows only (summed over ranks for a banded frame)
    uint32_t* nosample;           // [ONESTEP_HIST] rays that found no occupied sample at k + m
    const void* wfrag;
    const void* grid_params;
    const LevelInfo* levels;
    float4* frame_rgba;
    float* frame_depth;
    float* positions;
    int p;
    uint32_t target;
};
void launch_onestep_begin(const OnestepArgs& a, uint32_t k, uint32_t horizon, int first, hipStream_t s);
void launch_onestep_pass(const OnestepArgs& a, const NetworkDev& net, int final_pass, uint32_t n_rays_hint, hipStream_t s);
void launch_onestep_schedule(const OnestepArgs& a, hipStream_t s);

void launch_sh_encode(const float* coords, uint32_t stride, uint32_t dir_offset, uint32_t n, uint16_t* out, hipStream_t stream);
// ev0 / ev1: optional timing events recorded by the kernel's own dispatch (hipExtLaunchKernelGGL), so
// the measured interval is the kernel's execution, as rocprofv3 reports it
int launch_network(const NetworkDev& net, const float* coords, uint32_t stride, uint32_t n_static, const uint32_t* n_dev,
                   uint16_t* out, int layout, uint32_t max_tiles_hint, hipStream_t stream, hipEvent_t ev0 = nullptr,
                   hipEvent_t ev1 = nullptr, uint32_t* n_rec = nullptr);
// Normals (mode 2) input gradient / EncodingVis (mode 10) activation, rewriting the samples' coordinates in place
void launch_field_probe(const NetworkDev& net, const uint16_t* mlp_params, float* coords, const uint32_t* n_dev, int mode, int layer, int dim,
                        hipStream_t stream);
int launch_encode(const NetworkDev& net, const float* coords, uint32_t stride, uint32_t n, uint16_t* out, hipStream_t stream);

struct ShadowArgs {
    Volume vol;
    int W, H, row0, row1;
    int radius;                 // kernel_size / 2
    float intensity;            // nerf_shadow_intensity
    float threshold;            // nerf_on_nerf_shadow_threshold
    const ObjectGpu* objs; int n_objs;
    const LightGpu* lights; int n_lights;
    int n_point;                // lights of type 0 (Light::sample draws)
    // the mesh query's scene (as RaytraceArgs): BVH records + triangles staged in LDS when scene_in_lds
    const float4* scene_blob; uint32_t scene_f4;
    uint32_t stack_depth;       // traversal stack entries per thread
    int bvh_flat;
    int scene_in_lds;
    uint32_t tpb, blocks;       // persistent grid of the term kernel
};

// raytracer work counters (RaytraceArgs::work): [0] path-kernel tiles, [SHADOW_CTR0 + x * SHADOW_CTR_STRIDE]
// the shadow-ray chunk counters, one per memory channel (mesh.hip shadow_rays_kernel)
#ifndef SHADOW_NCTR
#define SHADOW_NCTR 8u
#endif
constexpr uint32_t SHADOW_CTR_STRIDE = 256;   // u32 (1 KiB) between counters
constexpr uint32_t SHADOW_CTR0 = 256;
constexpr uint32_t RT_WORK_WORDS = SHADOW_CTR0 + SHADOW_NCTR * SHADOW_CTR_STRIDE;
constexpr uint32_t RT_REC_COUNT = 128;        // work[128]: the hit-record counter (RtQueue::count; cleared with the work words)

struct RaytraceArgs {
    Volume vol;
    int W, row0, row1;
    f3 up;                      // camera[0]
    const ObjectGpu* objs; int n_objs;
    const LightGpu* lights; int n_lights;
    const MaterialGpu* mats;
    uint32_t samples, bounces, shadow_iters, shadow_steps;
    float lens;
    int show_nerf_shadow;
    float syn_shadow_factor;
    // traversal resources (host_scene.cpp upload_scene, host_render.cpp render_frame)
    const float4* scene_blob;   // all objects' BVH nodes + triangles, 16-B aligned (ObjectGpu::lds_nodes or lds_wide, lds_trit)
    uint32_t scene_f4;          // blob size in float4
    int scene_in_lds;           // copy the blob into LDS per workgroup
    uint32_t lds_tpb;           // threads per traversal workgroup (512, or 1024 when only one blob copy per CU fits)
    uint32_t stack_depth;       // traversal stack entries per thread (max BVH depth + 2, <= 32)
    uint32_t persistent_blocks; // workgroups per launch unit (number of CUs)
    uint32_t* work;             // RT_WORK_WORDS device work counters (pixel tiles, shadow-ray chunks)
    const uint32_t* tile_order; // 8x8 tile visiting order (nullptr: row-major)
    uint32_t* tile_cost;        // per-tile cycles of this frame (nullptr: not recorded)
    int bvh_flat;               // BvhWide traversal with the nearer child in a register (bvh_walk_near)
    int tile;                   // path-kernel tile width in pixels (8 or 4)
    int tile_h;                 // ... and height (tile * tile_h <= 64 lanes per wave: 8x8, 8x4, 4x4)
    unsigned long long* counts; // counting frames (rt_count): path kernel {queries, box, tri}, shadow kernel {queries, box, tri}
    int count_waves;            // rt_count = 2: box / tri entries count wave iterations of those loops (SIMD efficiency)
    int buffer_type;            // ImgBufferType (raytracer.cuh:20): 0 Final, 1 NextOrigin .. 7 NerfShadow (one-kernel path)
    uint32_t prio_tiles;        // the first prio_tiles tiles of tile_order run at wave priority 3 (0: off)
    uint32_t prio2_tiles;       // ... and the tiles before prio2_tiles at priority 2
    int spread;                 // first tile of every wave dealt statically across the CUs (rt_spread), the rest claimed
    int fused_shadow;           // the path kernel's idle waves trace the shadow rays (banded frames, mesh.hip fq_consume)
    uint32_t* started;          // rt_first: every path-kernel workgroup writes started_seq here as it lands (nullptr: off)
    uint32_t started_seq;
    int sample_par;             // rt_rng = 1: per-(pixel, sample) XORWOW streams, a pixel's samples on adjacent lanes (raytrace_sp_kernel)
    uint32_t sp_chunk;          // raytrace_sp_kernel: (64 / samples)-pixel units per work claim
};
constexpr uint32_t RT_SP_MAX_BOUNCES = 4;   // raytrace_sp_kernel keeps a lane's record indices in registers

// fused shadow queue of a banded path kernel (mesh.hip fq_publish / fq_consume): entries per workgroup, LDS words
constexpr uint32_t RT_FQ_CAP = 1024;
constexpr uint32_t RT_FQ_WORDS = 4 + 2 * RT_FQ_CAP;

// Deferred-shadow raytracer queues (mesh.hip, wavefront mode).  One "hit record" per (pixel,
// sample, bounce) that hit an object: header {next, spp, mat, pos.z} {pdf, att, pos.x, pos.y}, and the
// light colour {lc, 0} of every (light, shadow iteration) jl in loop order.  One "shadow ray" per
// point-light sample jp: {L, full_dist} (origin: its record's pos); its mask is written by the shadow
// kernel.  Light colours and shadow rays are stored sample-major ([jl][k], [jp][k]): the lanes of a
// wave shade consecutive records (wave_alloc), so each of their stores is one contiguous 1-KiB run
// instead of 64 scattered 16-B pieces (record-major scatter ran at ~1.7 TB/s).
struct RtQueue {
    float4* rec;          // cap x rec_stride float4: {next, spp, mat, pos.z} {pdf, att, pos.x, pos.y}
    float4* lc;           // nls x cap float4: {lc, 0} of record k, light sample jl at [jl * cap + k]
    float4* srec;         // nps x cap float4: {L, full_dist} of record k, shadow sample jp at [jp * cap + k]
    float* mask;          // cap x nps
    int* head;            // per mesh pixel: first hit record or -1
    uint32_t* count;      // hit records allocated (device counter)
    uint32_t rec_stride;  // float4 per hit record (2)
    uint32_t nls;         // n_lights * shadow_iters
    uint32_t nps;         // n_point_lights * shadow_iters
    uint32_t cap;
    // per-pixel record lists (tile path kernel): plist[t * max_hits + h] = the pixel's h-th hit record, pcount[t]
    // = its hits; rt_record_colour_kernel writes each record's colour term to rval and rt_accumulate_kernel
    // sums them in list order without walking the record chain.  nullptr: chain walk.
    int* plist;
    uint8_t* pcount;
    float4* rval;         // {colour * pdf * att, spp bits}
    uint32_t max_hits;    // samples * bounces (<= 255)
    // The shadow kernel traces in record-major order (a wave: the nps shadow samples of 64 / nps consecutive
    // records; sample-major tracing -- 64 records towards one light sample per wave -- measured 40 % slower:
    // the rays of one hit point share their walk until they part towards the lights); the storage is
    // sample-major (writes coalesce, the shadow kernel's reads are nps runs of 64 / nps records).
    __host__ __device__ float4* shadow_ray(uint32_t k, uint32_t jp) const { return srec + (size_t)jp * cap + k; }
    __host__ __device__ float4* lc_at(uint32_t k, uint32_t jl) const { return lc + (size_t)jl * cap + k; }
    __host__ __device__ size_t mask_at(uint32_t k, uint32_t jp) const { return (size_t)k * nps + jp; }
};

// nerf.hip: speculative tail rounds.  Once every iteration takes 8 steps a surviving ray's next
// samples depend only on the march and the t reset, so a round marches each alive ray K iterations
// ahead, ONE whole-GPU network launch evaluates them, and the compositor replays the iterations in
// order, stopping each ray where the wavefront would (samples past that point are discarded).
struct SpecArgs {
    Volume vol;
    CamDev cam;
    TraceMode mode;
    RayBuf in, out;               // alive rays (buffer p) -> survivors of the round (buffer p ^ 1)
    MarchCtrl* ctrl;
    int p;
    uint32_t budget;              // samples one round may generate: K = clamp(budget / (8 n_alive), 1, kmax)
    uint32_t kmax;                // <= SPEC_KMAX
    int k_policy;                 // 1: a ray looks ahead fewer iterations the more opaque it already is (spec_k_of)
    float* coords;                // NerfCoordinate AoS of the network samples
    uint2* samp;                  // per ray: {first network sample, n_it | cnt_last << 5 | reuse bits << 9}
    float* tbuf;                  // [sample j of the ray][ray] march t of every sample (incl. reused boundary samples)
    const uint2* net_out;         // [n][4] fp16
    float4* frame_rgba;
    float* frame_depth;
    float* positions;
    float4* pre;                  // per network sample: {logistic r, g, b, alpha} (spec_prepare; nullptr: the compositor
    float* pre_depth;             //   activates the raw outputs itself) and dot(fwd, pos - cam)
    uint8_t* hint;                // per NeRF pixel: 1 + the iteration its ray ended at in the last frame, counted from the
                                  // tail's first iteration (0: unknown);
                                  // a ray looks ahead just that far (exact whatever the hint: it only sizes the round)
    int hint_read;                // 0: the hints are another view's (the camera moved): written, not read
    uint32_t round;               // the round's index in the frame's tail (MarchCtrl::spec_round_samples)
};
constexpr uint32_t SPEC_KMAX = 16;

// nerf.hip: multi-step speculative rounds.  While n_steps = clamp(target / n_alive, 1, 8) is in [2, 7]
// (between the one-step regime and the 8-step tail) every alive ray of a round is at the same iteration
// k.  A round guesses that iterations k .. k + K - 1 all take S = steps_for(n_alive(k)) steps and
// marches every ray that far ahead (the positions depend on the march and the t reset only); ONE
// network launch evaluates the samples; msr_count replays the opacity of every ray and histograms the
// iteration it ends in; msr_schedule forms the frame-wide alive count of each iteration from it and
// commits J = the first iteration whose step count is not S (J >= 1); msr_commit replays the first J
// iterations exactly as composite_kernel does.
constexpr uint32_t MSR_KMAX = 16;
struct MsrArgs {
    Volume vol;
    CamDev cam;
    Sched sched;
    RayBuf in, out;               // alive rays at k (buffer p) -> alive at k + J (buffer p ^ 1)
    MarchCtrl* ctrl;
    int p;
    uint32_t target;
    uint32_t budget;              // samples one round may generate: K = clamp(budget / (S n_sched), 1, kmax)
    uint32_t kmax;                // <= MSR_KMAX
    int span;                     // a round may follow the hint across step changes (else: one step count per round)
    float* coords;                // NerfCoordinate AoS of the network samples
    uint2* samp;                  // per ray: {first network sample, n_it | cnt_last << 5 | reuse bits << 9}
    float* tbuf;                  // [sample j of the ray][ray] march t of every sample
    float* abuf;                  // [sample j of the ray][ray] its alpha (msr_count -> msr_commit), tbuf's layout
    const uint2* net_out;         // [n][4] fp16
    uint32_t* hist;               // [4][MSR_KMAX]: deaths (band), deaths (own rows; summed over ranks), samples, reused
    float4* frame_rgba;
    float* frame_depth;
    float* positions;
};
void launch_msr_generate(const MsrArgs& a, uint32_t blocks, hipStream_t s);
void launch_msr_count(const MsrArgs& a, uint32_t blocks, hipStream_t s);
void launch_msr_schedule(const MsrArgs& a, hipStream_t s);
void launch_msr_commit(const MsrArgs& a, uint32_t blocks, hipStream_t s);
void launch_spec_generate(const SpecArgs& a, uint32_t blocks, hipStream_t s);
void launch_spec_composite(const SpecArgs& a, uint32_t blocks, hipStream_t s);
void launch_spec_prepare(const SpecArgs& a, uint32_t blocks, hipStream_t s);
void launch_tail_prepare(MarchCtrl* ctrl, uint32_t* work, int p, uint32_t target, int global_sched, hipStream_t s);

// nerf.hip
void launch_init_rays(const NerfFrameArgs& a, const RayBuf& out, MarchCtrl* ctrl, float4* fb, float* depth, float* pos, float* nrm, uint32_t n_cus,
                      hipStream_t s);
void launch_generate(const Volume& v, const RayBuf& rays, MarchCtrl* ctrl, int p, uint32_t target, uint32_t iter, float* coords, uint2* samp,
                     uint32_t blocks, int store_t, int global_sched, hipStream_t s);
void launch_composite(const Volume& v, const CamDev& cam, const TraceMode& mode, const Sched& sched, const RayBuf& in, const RayBuf& out, MarchCtrl* ctrl, int p,
                      uint32_t target, uint32_t iter, const float* coords, const uint2* samp, const uint2* net_out, float4* fb, float* depth, float* pos, uint32_t blocks,
                      hipStream_t s, bool wide = false);
void launch_normals(int W, int H, int row0, int row1, const float* pos, float* nrm, hipStream_t s);
void launch_bitfield(const uint16_t* grid_f16, uint32_t max_cascade, float* grid_f32, double* partial, float* mean, uint8_t* bf, uint32_t* occ_linear,
                     hipStream_t s);
void launch_ctrl_init(MarchCtrl* ctrl, int32_t* tail_live, uint8_t* sched_hint, hipStream_t s, uint32_t* log = nullptr);
// reference slots of the tail's iterations (sum over k of n_alive(k) * 8 padded to 256) from MarchCtrl::tail_live
void launch_tail_slots(MarchCtrl* ctrl, hipStream_t s);
// OccBrick blob (sng_math.h) of the linear occupancy; flags: 4096 u32 scratch, blob: OCC_BRICK_CAP_WORDS, n_bricks: 1 u32
void launch_occ_brick(const uint32_t* occ_linear, uint32_t* flags, uint32_t* blob, uint32_t* n_bricks, hipStream_t s);
// mesh.hip
// scratch: shadow_scratch_bytes(a) of device memory (light samples and terms per neighbour slot)
size_t shadow_scratch_bytes(const ShadowArgs& a);
void launch_shadows(const ShadowArgs& a, float4* rgba, const float* pos, const float* nrm, uint32_t* rng, uint32_t n_rng, void* scratch, hipStream_t s);
void launch_mesh_rays(int W, int H, int row0, int row1, const CamDev& cam, f2 focal, f2 sc, float4* o, float4* d, float4* acc, float* accd,
                      hipStream_t s);
// rt_first: one wave on the NeRF stream waits until the path kernel's first workgroup has landed (*started == seq) or
// `timeout_us` has passed, so init_rays does not take the CUs first (the slower of the frame's two dispatch orders)
void launch_rt_wait_started(const uint32_t* started, uint32_t seq, uint32_t timeout_us, hipStream_t s);
void launch_raytrace_wavefront(const RaytraceArgs& a, const RtQueue& q, const float4* o, const float4* d, uint32_t* rng, uint32_t n_rng, float4* acc,
                               float* accd, uint32_t shadow_blocks, hipStream_t s);
void launch_tile_sort(const uint32_t* cost, uint32_t n, uint32_t* order, uint32_t* aux, hipStream_t s);

void launch_raytrace(const RaytraceArgs& a, const float4* o, const float4* d, uint32_t* rng, uint32_t n_rng, float4* acc, float* accd,
                     hipStream_t s);
// display.hip
void launch_display(const float4* img, int W, int H, int OW, int OH, f3 clear, uint8_t* out, hipStream_t s);
void launch_rgba8_band(const float4* img, uint32_t n, uint32_t* out, hipStream_t s);
void launch_overlay(int W, int row0, int row1, int scale, int nerf_w, int n_nerf, int show_nerf, float depth_offset, float exposure_mul, int srgb,
                    int tonemap, const float4* syn, const float* synd, const float4* nerf, const float* nerfd, float4* fin, float* find, hipStream_t s);
void launch_xorwow_init(uint32_t n, uint64_t seed, const uint32_t* seq_pow, uint32_t* st, hipStream_t s);

// error carrying an sng_status code (host.h guarded(), around every C ABI entry point, turns it into the return value + sng_last_error)
struct SngError : std::runtime_error {
    int code;
    SngError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// comm.cpp: the frame-wide step schedule exchange (Sched).  Either an RCCL communicator (device
// all-reduce on the NeRF stream) or a host callback (sng_set_sched_reducer) sums the counts.
struct SchedComm {
    void* comm = nullptr;              // ncclComm_t
    int rank = 0, world = 0;
    sng_sched_reduce_fn host_fn = nullptr;
    void* host_user = nullptr;
    // schedule replay (sng_set_sched_replay): records {n, v[0..n)} of one frame's reductions in pinned memory,
    // copied to the device at each reduction point in call order; the cursor restarts every frame
    uint32_t* replay = nullptr;
    size_t replay_words = 0, replay_cursor = 0, replay_calls = 0;
    bool active() const { return comm != nullptr || host_fn != nullptr || replay != nullptr; }
};
void comm_unique_id(uint8_t out[SNG_COMM_ID_BYTES]);
void comm_init(SchedComm& c, const uint8_t* id, int rank, int world);
void comm_destroy(SchedComm& c);
void comm_allreduce_u32(SchedComm& c, const uint32_t* src, uint32_t* dst, size_t n, hipStream_t s);   // src == dst: in place
void comm_gather_to_root(SchedComm& c, const void* d_band, void* d_frame, const size_t* offsets, const size_t* sizes, hipStream_t s);

}  // namespace sng
