/*
 * sng_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * This is a plain scalar C++ restatement of SyNeRFgine's render hot path, used
 * ONLY by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * parity checker.  The product (libsng_hip.so) never links or calls it.
 *
 * Parity status: PARTIALLY PINNED.  The reference (/root/reference) cannot be
 * compiled here (CUDA headers absent, tiny-cuda-nn submodule unvendored) and
 * ships no golden vectors.  Functions that restate reference code are cited
 * (file:line, relative to the reference root); functions that restate
 * tiny-cuda-nn / cuRAND semantics are marked [tcnn, unvendored] /
 * [cuRAND, unvendored] and are pinned only by published constants
 * (SURVEY.md Appendix B/C level tables, SH constants) -- "parity unpinned"
 * for those parts.  See DESIGN.md "Oracle".
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- scene / model descriptors (oracle-private, plain C) ---------------- */
typedef struct {
    uint32_t n_levels;          /* L   (base.json:23-29) */
    uint32_t n_features;        /* F   */
    uint32_t log2_hashmap_size; /* log2 T */
    uint32_t base_resolution;   /* Nmin */
    float per_level_scale;      /* b (read from snapshot, testbed.cu:3737-3741) */
    const uint16_t* params;     /* fp16 blob: density MLP (3072), rgb MLP (7168), grid */
} orc_model;

typedef struct {
    float render_aabb_min[3], render_aabb_max[3];
    float train_aabb_min[3], train_aabb_max[3];
    float render_aabb_to_local[9]; /* column-major mat3 */
    float cone_angle_constant;
    uint32_t max_mip;              /* m_nerf.max_cascade */
    float min_transmittance;       /* render_min_transmittance, testbed.h:867 */
    const uint8_t* bitfield;       /* NERF_CASCADES * 128^3 / 8 bytes, Morton order */
} orc_volume;

typedef struct {
    float camera[12];          /* mat4x3, column-major (right, down, fwd, pos) */
    float focal[2];
    float screen_center[2];
    int32_t res[2];
    uint32_t spp;              /* render_buffer.spp (sample index) */
    int32_t snap_to_pixel_centers;
    uint32_t target_n_queries; /* 2*1024*1024 in the reference (testbed_nerf.cu:2189) */
} orc_camera;

typedef struct {
    const float* nodes;  /* n_nodes x 8 floats: bb.min xyz, bb.max xyz, left_idx (int bits), right_idx (int bits) */
    const float* tris;   /* n_tris x 9 floats: a, b, c */
    float rot[9];        /* column-major mat3 */
    float pos[3];
    float scale;
    int32_t mat_id;
} orc_object;

typedef struct { float pos[3]; float intensity; float size; int32_t type; /* 0 point, 1 directional */ } orc_light;
typedef struct { float ka[3], kd[3], ks[3]; float n, rg, spec_angle; int32_t type; /* 0 lambertian, 1 glossy */ } orc_material;

typedef struct {
    uint32_t n_iterations;    /* wavefront iterations executed */
    uint64_t n_samples;       /* real (non-stale) network samples */
    uint64_t n_slots;         /* reference slots incl. stale + padding */
    uint32_t n_hit;           /* rays in the hit list */
    uint32_t alive_per_iter[64];
    uint32_t steps_per_iter[64];
} orc_nerf_stats;

typedef struct {
    int32_t nerf_res[2];
    int32_t mesh_res[2];
    int32_t syn_px_scale;           /* m_relative_vo_scale */
    int32_t show_nerf;              /* m_show_nerf */
    int32_t show_virtual_obj;       /* RayTracer::m_show_virtual_obj */
    int32_t shadow_on_nerf;         /* m_view_syn_shadow */
    int32_t shadow_on_virtual_obj;  /* RayTracer::m_view_nerf_shadow */
    float nerf_shadow_intensity;    /* engine.cuh:117 */
    float nerf_on_nerf_shadow_threshold; /* engine.cuh:119 */
    int32_t nerf_kernel_size;       /* Testbed::sng_position_kernel_size (testbed.h:686) */
    uint32_t light_samples;         /* RayTracer::m_samples */
    uint32_t path_trace_depth;      /* RayTracer::m_ray_iters */
    uint32_t shadow_iters;          /* RayTracer::m_shadow_iters */
    uint32_t shadow_steps;          /* RayTracer::m_n_steps (8) */
    float lens_angle_constant;      /* RayTracer::m_lens_angle_constant */
    float syn_shadow_factor;        /* RayTracer::m_syn_shadow_factor */
    float rt_depth_offset;          /* RayTracer::m_depth_offset (overlay z-test) */
    float exposure;
    int32_t srgb_output;            /* EColorSpace::SRGB (engine.cu:406) */
    int32_t tonemap_curve;          /* Testbed::m_tonemap_curve (engine.cu:406): ETonemapCurve 0 Identity, 1 ACES, 2 Hable, 3 Reinhard */
    int32_t rt_buffer_type;         /* RayTracer::m_buffer_to_show (raytracer.cuh:20,179): ImgBufferType 0 Final .. 7 NerfShadow */
} orc_frame_params;

/* ---- primitives (KAT-level) --------------------------------------------- */
uint32_t orc_morton3D(uint32_t x, uint32_t y, uint32_t z);
uint32_t orc_morton3D_invert(uint32_t x);
uint32_t orc_sobol(uint32_t index, uint32_t dim);
float    orc_ld_random_val(uint32_t index, uint32_t seed, uint32_t dim);
void     orc_ld_random_pixel_offset(uint32_t spp, float out[2]);
uint16_t orc_float_to_half(float f);
float    orc_half_to_float(uint16_t h);

/* cuRAND XORWOW [cuRAND, unvendored] */
void     orc_xorwow_init(uint64_t seed, uint64_t subsequence, uint64_t offset, uint32_t state[6]);
void     orc_xorwow_init_many(uint64_t seed, uint32_t n, uint32_t* states /* n x 6 */);
uint32_t orc_xorwow_next(uint32_t state[6]);
float    orc_curand_uniform(uint32_t state[6]);
void     orc_xorwow_jump_steps_naive(uint32_t state[6], uint64_t steps); /* stepping (test helper) */
void     orc_xorwow_jump_matrix(uint32_t state[6], uint32_t log2_steps);  /* M^(2^k), k in 0..63 or 67..98 (test helper) */

/* ---- network (A6-A8) ----------------------------------------------------- */
uint32_t orc_grid_level_table(const orc_model* m, uint32_t* offsets /* L+1 */, uint32_t* resolutions /* L */);
uint32_t orc_n_params(const orc_model* m);
/* trace_alt's per-iteration n_steps (testbed_nerf.cu:2188-2190) and padded batch n_elements (:2210) for each
 * n_alive; target 0 = 2^21 */
void orc_wavefront_schedule(const uint32_t* n_alive, uint32_t n, uint32_t target, uint32_t* n_steps, uint64_t* n_elements);
void orc_hashgrid_encode(const orc_model* m, const float* coords, uint32_t stride_floats, uint32_t n, uint16_t* out /* n x L*F */);
void orc_sh_encode(const float* coords, uint32_t stride_floats, uint32_t dir_offset, uint32_t n, uint16_t* out /* n x 16 */);
void orc_nerf_inference(const orc_model* m, const float* coords, uint32_t stride_floats, uint32_t n, uint16_t* out /* n x 16 (tcnn rgbsigma row block) */);

/* ---- occupancy (A17) ------------------------------------------------------ */
void orc_density_grid_to_bitfield(const uint16_t* grid_f16, uint32_t max_cascade, uint8_t* bitfield /* 8*128^3/8 */, float* mean_out);

/* ---- NeRF render (A1-A5, A9-A10c) --------------------------------------- */
void orc_render_nerf(const orc_model* m, const orc_volume* v, const orc_camera* c,
                     float* frame_rgba /* W*H*4, in/out */, float* frame_depth /* W*H, in/out */,
                     float* positions /* W*H*3 out */, float* normals /* W*H*3 out */,
                     orc_nerf_stats* stats);

/* ---- shadows on NeRF (A11) ---------------------------------------------- */
/* instant-NGP render path (A22): NerfTracer::trace + composite_kernel_nerf + shade_kernel_nerf
 * (testbed_nerf.cu:2279-2401, 577-788, 1788-1828).  render_mode: ERenderMode (0 AO, 1 Shade,
 * 3 Positions, 4 Depth, 6 Cost, 10 EncodingVis); depth_scale = 1 / dataset.scale. */
/* View::camera1 / rolling_shutter (testbed.h:1032,1042) for the NeRF camera rays (testbed_nerf.cu:1895);
 * camera1 NULL: camera0, rolling_shutter NULL: (0, 0, 0, 1) */
void orc_set_motion_blur(const float* camera1, const float* rolling_shutter);
/* Lens (common.h:188-205): mode 0 Perspective, 1 OpenCV {k1 k2 p1 p2}, 2 F-Theta {p0..p4, w, h}, 3 LatLong,
 * 4 OpenCV fisheye {k1..k4}, 5 Equirectangular.  orc_set_render_lens: the NeRF camera rays' lens (NULL:
 * Perspective); orc_set_train_lens: one per training image for orc_train_generate (n = 0: all Perspective) */
typedef struct { int32_t mode; float params[7]; } orc_lens;
void orc_set_render_lens(const orc_lens* lens);
void orc_set_train_lens(const orc_lens* lenses, uint32_t n);
/* uv_to_ray's camera-space direction for one uv (common_device.cuh:403-447); returns 0 for Ray::invalid() */
int32_t orc_uv_to_ray_dir(const orc_lens* lens, const float* uv, int32_t W, int32_t H, const float* focal, const float* screen_center, float* dir);
/* the forward distortion pos_to_uv applies (common_device.cuh:526-534): OpenCV or OpenCV fisheye delta */
void orc_lens_distortion_delta(const orc_lens* lens, float u, float v, float* du, float* dv);
/* Testbed::Nerf::glow_mode / glow_y_cutoff (testbed.h:870-871) for orc_render_nerf_ngp (testbed_nerf.cu:638-734) */
void orc_set_glow(int32_t mode, float y_cutoff);
/* shade_nerf_shadows' light-sample RNG for nerf_shadow_samples > 0: 0 = the centre pixel's stream (this
 * library's kernels), 1 = the neighbour's stream as the reference's racy rand_state[idx] (serialised) */
void orc_set_shadow_rng_mode(int32_t neighbour);
/* 1 (default): the reference's text as written -- IEEE division in the BVH box test (bounding_box.cuh:163-211),
 * powf for the Phong term and the shadow masks (material.cuh:96-98, raytracer.cu:6-57, testbed_nerf.cu:1614-1786),
 * overlay_nerf's NeRF pixel index unclamped (raytracer.cu:242-246; an index past the buffer, which the reference
 * reads out of bounds, gives NaN).  0: the product's restatements of the reference's --use_fast_math build
 * (CMakeLists.txt:82): (b - o) * RN(1/d) box tests, integer powers by binary exponentiation, the clamped index --
 * the forms libsng_hip.so evaluates, so GPU and oracle agree bit for bit. */
void orc_set_literal(int32_t on);
void orc_render_nerf_ngp(const orc_model* m, const orc_volume* v, const orc_camera* c, int32_t render_mode, float depth_scale,
                         float* frame_rgba /* W*H*4 */, float* frame_depth /* W*H */, orc_nerf_stats* stats);
void orc_shade_nerf_shadows(const orc_volume* v, const int32_t res[2],
                            float* frame_rgba, const float* positions, const float* normals,
                            const orc_object* objs, uint32_t n_objs, const orc_light* lights, uint32_t n_lights,
                            uint32_t* rng_states /* W*H*6, in/out */,
                            float nerf_shadow_intensity, float nerf_on_nerf_shadow_threshold, int32_t kernel_size);

/* ---- BVH (A12, A13) ------------------------------------------------------ */
int32_t orc_bvh_build(float* tris /* n x 9, reordered in place */, uint32_t n_tris, uint32_t prims_per_leaf, float* nodes_out /* cap x 8 */, uint32_t cap);
void orc_depth_test_world(const orc_object* objs, uint32_t n_objs, const float* origins, const float* dirs, uint32_t n, float* t_out, int32_t* obj_out);

/* ---- virtual objects (A14, A15, A19) ------------------------------------- */
void orc_mesh_init_rays(const orc_camera* c, float* origins, float* dirs, float* acc_rgba, float* acc_depth);
void orc_raytrace(const orc_volume* v, const float* camera /* mat4x3 */, const orc_frame_params* p,
                  const orc_object* objs, uint32_t n_objs, const orc_light* lights, uint32_t n_lights,
                  const orc_material* mats, uint32_t n_mats,
                  const float* origins, const float* dirs, uint32_t n,
                  uint32_t* rng_states, float* acc_rgba, float* acc_depth);
void orc_overlay(const orc_frame_params* p, const float* syn_rgba, const float* syn_depth,
                 const float* nerf_rgba, const float* nerf_depth, float* final_rgba, float* final_depth);

/* ---- whole frame (A18-A20) ------------------------------------------------ */
void orc_render_frame(const orc_model* m, const orc_volume* v, const orc_camera* nerf_cam, const orc_camera* mesh_cam,
                      const orc_frame_params* p,
                      const orc_object* objs, uint32_t n_objs, const orc_light* lights, uint32_t n_lights,
                      const orc_material* mats, uint32_t n_mats,
                      uint32_t* nerf_rng, uint32_t* mesh_rng,
                      float* final_rgba, float* final_depth,
                      float* nerf_rgba, float* nerf_depth, orc_nerf_stats* stats);

/* ---- online training (BASELINE config 5, Testbed::train_nerf) --------------- */
typedef struct {
    const uint8_t* rgba;    /* n x h x w x 4 sRGB 8-bit (0x00FF00FF little-endian word = masked) */
    const float* xforms;    /* n x 12: camera columns c0 c1 c2 c3 (mat4x3, NGP space) */
    const float* focal;     /* n x 2 pixels */
    const float* pp;        /* n x 2 principal point (uv) */
    int32_t w, h, n;
} orc_train_images;
/* generate_training_samples_nerf (testbed_nerf.cu:838-998) for rays [0, n_rays) of a batch drawn from the
 * tcnn pcg32 {rng_state, rng_inc}: per ray, numsteps (0 = masked pixel or no occupied sample), the
 * unnormalised ray (o, d) and the first min(numsteps, max_per_ray) NerfCoordinates (7 floats). */
void orc_train_generate(const orc_volume* v, const orc_train_images* im, uint64_t rng_state, uint64_t rng_inc, uint32_t n_rays,
                        uint32_t max_per_ray, uint32_t* numsteps, float* rays /* n_rays x 6 */, float* coords /* n_rays x max_per_ray x 7 */);
/* one tcnn Adam step (adam_step: l2_reg on the first n_matrix params, zero-gradient non-matrix params
 * skipped, per-param step counts) followed by the EmaOptimizer's debiased EMA (ema_step) */
void orc_train_adam_ema(uint64_t n, uint32_t n_matrix, float lr, float beta1, float beta2, float eps, float l2_reg, float loss_scale,
                        float ema_decay, uint32_t ema_step, float* master, const float* grads, float* m1, float* m2, uint32_t* steps,
                        float* ema);

/* ---- scene animation: CamPath (cam_path.cuh:30-143) driving Testbed::set_view_dir /
 * set_look_at / set_scale (testbed.cu:405-425), Light::next_frame (light.cuh:39-49), VirtualObject::next_frame
 * (virtual_object.cuh:53-64), played in Engine::frame's order (engine.cu:365-372, 80-127). */
typedef struct { float view[3], at[3], zoom; } orc_keyframe;
typedef struct { int32_t on; float start[3], end[3], ratio, step; } orc_light_anim;
typedef struct { float angle, axis[3], centre[3], rot[9] /* object rotation, column-major */, pos[3]; } orc_object_anim;
/* Engine::init's camera from the scene JSON (engine.cu:148-152): set_view_dir(view), set_look_at(at), set_scale(zoom) */
void orc_camera_set_view(float cam[12], float* scale, const float up[3], const float view[3], const float at[3], float zoom);
void orc_animation_play(float cam[12] /* in/out */, float* scale /* in/out */, const float up[3], const orc_keyframe* keys, uint32_t n_keys,
                        int32_t total_frames, int32_t playing, float anim_speed, orc_light_anim* lights, uint32_t n_lights,
                        orc_object_anim* objs, uint32_t n_objs, uint32_t n_frames, float* cams_out /* n x 12 */,
                        float* light_pos_out /* n x n_lights x 3 */, float* obj_pos_out /* n x n_objs x 3 */);

/* headless display stage: main.frag (scripts/virtual_desc/main.frag:24-117) FXAA of the final RGBA32F
 * frame (W x H texture, GL_LINEAR + GL_REPEAT) into an OW x OH window, blended GL_ONE /
 * GL_ONE_MINUS_SRC_ALPHA over the clear colour (display.cu:265-281), unorm8 RGB, top-down rows */
void orc_display(const float* rgba, int32_t W, int32_t H, int32_t OW, int32_t OH, const float clear[3], uint8_t* rgb_out);

int32_t orc_num_threads(void);
void orc_set_num_threads(int32_t n);
/* MLP accumulation model (sng_oracle.cpp dense()): 0 = fp32 over K (default), 1 = tcnn WMMA __half
 * accumulators, rounded to fp16 after every `chunk` (16) products */
void orc_set_mlp_accum(int32_t mode, int32_t chunk);
/* EncodingVis: Testbed::m_visualized_layer / m_visualized_dimension for orc_render_nerf_ngp(render_mode 10) */
void orc_set_visualization(int32_t layer, int32_t dim);
/* orc_render_frame also copies the NeRF G-buffer (positions, normals: 3 floats per NeRF pixel, before the
 * shadow pass) into these host buffers when set (NULL: off) */
void orc_set_gbuffer_out(float* positions, float* normals);   /* OpenMP threads of the later calls (bench CPU baseline) */

#ifdef __cplusplus
}
#endif
