/*
 * sng.h -- C-ABI of libsng_hip.so, the MI355X-native SyNeRFgine render path.
 *
 * Plain pointers and sizes only (no torch / HIP C++ types in signatures).
 * Device pointers are marked d_*; everything else is host memory.  Every call
 * returns an int status (SNG_OK = 0) and records a message for
 * sng_last_error() on failure -- the C equivalent of the reference's
 * CUDA_CHECK_THROW -> std::runtime_error (main.cu:225-227).
 *
 * Each entry point names the reference interface it replaces (file:line,
 * relative to the reference root).  INTEGRATION.md shows the binding a
 * maintainer would add on the reference side.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SNG_ABI_VERSION 4

enum {
    SNG_OK = 0,
    SNG_ERR_INVALID = -1,   /* bad argument / shape mismatch */
    SNG_ERR_HIP = -2,       /* HIP runtime error */
    SNG_ERR_IO = -3,        /* file missing / parse error */
    SNG_ERR_STATE = -4,     /* call order (e.g. render before a model is set) */
    SNG_ERR_NOGPU = -5      /* no HIP device visible */
};

typedef struct sng_ctx sng_ctx;

typedef struct {
    int32_t device_id;       /* HIP device ordinal (one context per GPU / rank) */
    int32_t reserved[7];
} sng_ctx_desc;

/* NerfNetwork configuration (configs/nerf/base.json:23-55; nerf_network.h:79-101).
 * The fused kernel is specialised for the base.json shape: 64-neuron MLPs,
 * density 1 hidden layer, rgb 2 hidden layers, SH degree 4, L*F = 32. */
typedef struct {
    uint32_t n_levels;              /* 8  */
    uint32_t n_features_per_level;  /* 4  */
    uint32_t log2_hashmap_size;     /* 19 */
    uint32_t base_resolution;       /* 16 */
    float per_level_scale;          /* from the snapshot (testbed.cu:3737-3741) */
    uint32_t aabb_scale;            /* power of two; -> m_aabb, max_cascade, cone (testbed_nerf.cu:3069-3085) */
    uint32_t reserved[6];
} sng_nerf_config;

typedef struct {
    int32_t nerf_res[2];   /* NeRF render buffer resolution (Engine::resize, engine.cu:236-255) */
    int32_t mesh_res[2];   /* virtual-object (raytracer) resolution */
    int32_t syn_px_scale;  /* m_relative_vo_scale after resize */
    int32_t reserved[3];
} sng_resolution_info;

typedef struct {
    uint32_t spp;                /* render_buffer.spp: sample index for pixel jitter */
    int32_t reset_accumulation;  /* 1: camera-moved semantics (fresh accumulation buffers) */
    int32_t row_begin;           /* band of final-image rows to produce, [row_begin,row_end); 0,0 = all */
    int32_t row_end;
    int32_t collect_kernel_times;/* 1: hipEvent-time every network launch (bench roofline) */
    uint32_t target_n_queries;   /* 0 = 2*1024*1024 (testbed_nerf.cu:2189) */
    int32_t reserved[2];
} sng_frame_params;

typedef struct {
    /* device buffers owned by the context, valid until the next render/resize */
    float* d_final_rgba;      /* mesh_res, RGBA32F, overlay output (raytracer.cu:256) */
    float* d_final_depth;     /* mesh_res */
    float* d_nerf_rgba;       /* nerf_res, NeRF frame buffer after shadows */
    float* d_nerf_depth;      /* nerf_res */
    float* d_nerf_positions;  /* nerf_res x 3 */
    float* d_nerf_normals;    /* nerf_res x 3 */
    float* d_syn_rgba;        /* mesh_res, raytracer accumulation buffer (m_rays[0].rgba) */
    float* d_syn_depth;       /* mesh_res */
    /* statistics */
    uint32_t n_iterations;    /* wavefront iterations of trace_alt */
    uint32_t n_hit;           /* rays that reached the hit list */
    uint64_t n_samples;       /* march samples composited (real, compacted; equals the reference's real samples) */
    uint64_t n_reference_slots; /* slots the reference would evaluate (incl. stale + padding) */
    float ms_frame;           /* device time of the whole frame (hipEvents) */
    float ms_raytrace, ms_nerf, ms_shadow, ms_overlay;
    float ms_network;         /* sum of fused network kernel durations (collect_kernel_times) */
    uint32_t network_launches;
    uint32_t alive_per_iter[64];
    uint32_t steps_per_iter[64];
    uint32_t samples_per_iter[64];
    uint32_t fused_from_iter;   /* first iteration marched by the ray-local fused tail (n_iterations: none) */
    uint64_t n_samples_network; /* samples of the whole-GPU network launches (device counter); the other
                                   n_samples - n_samples_network were evaluated inside the fused tail */
    float ms_fused_tail;        /* device time of the fused tail launch (collect_kernel_times) */
    uint64_t n_samples_reused;  /* march samples whose network output was reused, not evaluated: trace_alt's t reset
                                   (testbed_nerf.cu:574) makes an iteration's first sample the previous one's last */
    uint32_t onestep_from_iter; /* trace_alt's one-step regime (n_alive > target/2) marched ray-locally from this
                                   iteration (n_iterations: none) ... */
    uint32_t onestep_iterations;/* ... for this many iterations */
    float ms_onestep;           /* device time of the one-step regime's kernels (collect_kernel_times) */
    uint32_t onestep_field_evals; /* field evaluations of the regime's final pass (its samples are otherwise cached) */
    uint32_t spec_rounds;       /* speculative tail rounds enqueued (nerf_spec_rounds; 0: none) */
    uint32_t spec_evals;        /* samples their network launches evaluated, incl. those past a ray's end */
    uint32_t spec_exec;         /* ... of which composited (the rest is the rounds' discarded look-ahead) */
    uint32_t msr_rounds;        /* multi-step speculative rounds that committed iterations (nerf_msr; 0: none) */
    uint32_t msr_evals;         /* samples their network launches evaluated ... */
    uint32_t msr_exec;          /* ... of which the per-iteration wavefront would have evaluated */
    uint32_t sched_reductions;  /* frame-wide schedule reductions (all-reduces per rank) the frame made; 0 without a
                                   communicator, reducer or replay */
    uint32_t n_launch_rec;      /* network launches recorded below (collect_kernel_times; min(network_launches, 16)) */
    float ms_network_launch[16];        /* each launch's duration (its own dispatch's start/stop events) ... */
    uint32_t samples_network_launch[16];/* ... and the sample count it evaluated (read by the kernel itself) */
} sng_frame_result;

typedef struct { float pos[3]; float intensity; float size; int32_t type; /* 0 point, 1 directional */ } sng_light;
typedef struct { float ka[3], kd[3], ks[3]; float n, rg, spec_angle; int32_t type; /* 0 lambertian, 1 glossy */ } sng_material;
typedef struct {
    uint32_t n_nodes, n_tris;
    float rot[9];      /* column-major mat3 */
    float pos[3];
    float scale;
    int32_t mat_id;
} sng_object_info;

/* ---- context ------------------------------------------------------------- */
const char* sng_last_error(void);
int sng_abi_version(void);
int sng_device_count(int* out);
/* replaces Testbed::Testbed + Engine ctor (testbed.cu:3897, engine.cuh:22) */
int sng_ctx_create(const sng_ctx_desc* desc, sng_ctx** out);
int sng_ctx_destroy(sng_ctx* ctx);

/* ---- model: Testbed::load_snapshot (testbed.cu:4878-5015, 4994) ---------- */
int sng_load_snapshot(sng_ctx* ctx, const char* ingp_path);
/* Testbed::save_snapshot(path, include_optimizer_state, compress) (testbed.cu:4812-4876): the network
 * config + tcnn Trainer::serialize (inference params; with the optimizer state: EMA weights, Adam
 * moments / param steps / step) + the Testbed fields (density grid fp16, aabbs, camera, dataset
 * metadata, batch counters).  ".ingp": gzip(msgpack), else msgpack.  sng_load_snapshot restores the
 * optimizer state when present (training continues from it). */
int sng_save_snapshot(sng_ctx* ctx, const char* path, int32_t include_optimizer_state, int32_t compress);
/* host-only parse of the same file (no device): config, sizes, and optionally the fp16 params and
 * density grid copied out (buffers may be NULL) -- the load_snapshot parse step (testbed.cu:4880-4931) */
int sng_snapshot_probe(const char* ingp_path, sng_nerf_config* cfg, uint64_t* n_params, uint64_t* n_grid_cells,
                       uint16_t* params_out, uint64_t params_cap, uint16_t* grid_out, uint64_t grid_cap);
/* NerfNetwork params in tcnn order (nerf_network.h:356-371): density MLP, rgb MLP, grid; fp16 */
int sng_set_nerf_model(sng_ctx* ctx, const sng_nerf_config* cfg, const uint16_t* params_f16, uint64_t n_params);
uint64_t sng_nerf_param_count(const sng_nerf_config* cfg);
/* density_grid_binary (fp16, 128^3 x (max_cascade+1)) -> bitfield
 * (update_density_grid_mean_and_bitfield, testbed_nerf.cu:3212-3229) */
int sng_set_density_grid(sng_ctx* ctx, const uint16_t* grid_f16, uint64_t n_cells);
int sng_get_bitfield(sng_ctx* ctx, uint8_t* out, uint64_t n_bytes);
int sng_get_density_mean(sng_ctx* ctx, float* out);

/* ---- operator boundary: NerfNetwork::inference_mixed_precision (nerf_network.h:105-139)
 * d_coords: NerfCoordinate AoS {pos(3), dt, dir(3)} with stride_floats >= 7;
 * out_layout 0: tcnn GPUMatrix<half,RM> [16][n] (row c at c*n; row 3 = density);
 * out_layout 1: AoS [n][4] = (r,g,b,density) raw network outputs;
 * out_layout 2: AoS [n][4] with the density only, rgb = 0 (NerfNetwork::density, nerf_network.h:270: the density MLP
 *               alone, as the density-grid update evaluates it). */
int sng_nerf_inference(sng_ctx* ctx, const float* d_coords, uint32_t stride_floats, uint32_t n,
                       uint16_t* d_out, int32_t out_layout, void* hip_stream);
/* pos encoding only (tcnn GridEncoding forward), out [n][L*F] fp16 -- parity hook */
int sng_hashgrid_encode(sng_ctx* ctx, const float* d_coords, uint32_t stride_floats, uint32_t n, uint16_t* d_out, void* hip_stream);
/* NerfNetwork::m_dir_encoding->inference_mixed_precision (nerf_network.h:84,122-127): SphericalHarmonics
 * degree 4 of the direction at d_coords[i * stride + dir_offset .. +2] (warped to [0,1]^3), d_out [n][16] fp16 */
int sng_sh_encode(sng_ctx* ctx, const float* d_coords, uint32_t stride_floats, uint32_t dir_offset, uint32_t n, uint16_t* d_out, void* hip_stream);

/* ---- virtual scene: Engine::set_virtual_world + Engine::init keys (engine.cu:21-78, 129-234) */
int sng_load_virtual_scene(sng_ctx* ctx, const char* json_path);
int sng_clear_virtual_scene(sng_ctx* ctx);
/* scalar engine/raytracer parameters by their scene-JSON key ("light_samples", "path_trace_depth",
 * "syn_shadow_samples", "nerf_shadow_samples", "nerf_shadow_intensity", "exposure", "res_factor",
 * "vo_scale", "shadow_on_nerf", "shadow_on_virtual_obj", "show_virtual_obj", "show_nerf", "lens_size",
 * "depth_offset", "syn_shadow_intensity", "nerf_on_nerf_shadow_threshold", ...) and the CLI
 * flags --sshadows/--nshadows (main.cu:93-126, engine.cuh:29-33) as "sshadows"/"nshadows". */
int sng_set_param(sng_ctx* ctx, const char* key, double value);
int sng_get_param(sng_ctx* ctx, const char* key, double* value);
int sng_get_scene_counts(sng_ctx* ctx, uint32_t* n_objects, uint32_t* n_lights, uint32_t* n_materials);
int sng_get_object(sng_ctx* ctx, uint32_t i, sng_object_info* out);
int sng_get_object_bvh(sng_ctx* ctx, uint32_t i, float* nodes_out /* n_nodes x 8 */, float* tris_out /* n_tris x 9 */);
int sng_get_light(sng_ctx* ctx, uint32_t i, sng_light* out);
int sng_get_material(sng_ctx* ctx, uint32_t i, sng_material* out);

/* ---- camera: Testbed::set_view_dir / set_look_at / set_scale (testbed.cu:405-425), set_fov (3562) */
int sng_set_camera_view(sng_ctx* ctx, const float view_dir[3], const float look_at[3], float scale);
int sng_set_camera_matrix(sng_ctx* ctx, const float m[12]);
int sng_get_camera_matrix(sng_ctx* ctx, float m[12]);
/* View::camera1 and View::rolling_shutter (testbed.h:1032,1042; Engine::nerf_render_buffer_view,
 * engine.cuh:50-52): NeRF rays use get_xform_given_rolling_shutter({camera0, camera1}, rolling_shutter,
 * uv, motionblur_time) per pixel (testbed_nerf.cu:1895). camera1 NULL: camera1 = camera0 (the engine's
 * default); rolling_shutter NULL: (0, 0, 0, 1), the View default.  camera1 is dropped (camera1 =
 * camera0 again) by the next change of camera0 -- sng_set_camera_matrix / _view, set_fov keeps it,
 * camera-path playback -- as the reference re-derives camera1 from camera0 every frame
 * (testbed.cu:2850): set the blur after the pose.  Only the NeRF layer is blurred; the virtual
 * objects are path-traced from camera0 (the reference's raytracer takes one camera too). */
int sng_set_motion_blur(sng_ctx* ctx, const float camera1[12], const float rolling_shutter[4]);
int sng_set_fov(sng_ctx* ctx, float degrees);                 /* fov_axis = 1 */
int sng_get_focal_length(sng_ctx* ctx, int which /*0 nerf,1 mesh*/, float out[2]);

/* ---- frame: Engine::resize + Engine::frame (engine.cu:236-255, 352-433) ---- */
int sng_set_window(sng_ctx* ctx, int32_t width, int32_t height);
int sng_get_resolution(sng_ctx* ctx, sng_resolution_info* out);
/* Each call first advances the scene animation exactly as Engine::frame does before rendering
 * (engine.cu:365-372): the camera path when playing (CamPath::update, cam_path.cuh:117-135), then,
 * when "animation_speed" > 0, every object (VirtualObject::next_frame, virtual_object.cuh:53-64)
 * and light (Light::next_frame, light.cuh:39-49).  Animation parameters (sng_set_param):
 * "animation_speed", "camera_path_playing" (Play/Pause), "camera_path_frame" (the frame slider);
 * read-only "camera_path_total_frames". */
int sng_render_frame(sng_ctx* ctx, const sng_frame_params* params, sng_frame_result* out);
/* Traversal counts of the last frame rendered with parameter rt_count = 1 (the deferred path tracer's
 * counting instantiation; the timed kernels carry no counters): out[6] = path kernel {world queries
 * (camera + bounce rays), box tests, triangle tests}, shadow-ray kernel {queries, box tests, triangle
 * tests}.  Zeros when no counting frame ran. */
int sng_rt_counters(sng_ctx* ctx, uint64_t* out);
/* Debug hook: copy a wavefront buffer of the last frame to the host -- "coords" (the last network
 * launch's NerfCoordinates), "net_out" ([n][4] fp16 outputs), "samp" (per-ray {first, count}). */
int sng_frame_buffer(sng_ctx* ctx, const char* name, void* out, uint64_t capacity_bytes, uint64_t* size_bytes);
/* Band composition for tiled multi-GPU frames (the reference has no multi-GPU render): the
 * last frame's final RGBA rows [row_begin, row_end) at mesh resolution as RGBA8 (unorm8 =
 * round(clamp(c, 0, 1) * 255), one uint32 per px, R in the low byte) into the device buffer d_out,
 * enqueued on hip_stream -- the 4 B/px tile each rank contributes to the RCCL gather. */
int sng_final_rgba8(sng_ctx* ctx, int32_t row_begin, int32_t row_end, uint32_t* d_out, void* hip_stream);
/* ---- headless display stage (Display::present / save_image, display.cu:265-322; main.frag:24-117) ----
 * The last frame's final RGBA at mesh resolution, drawn to the window resolution through main.frag's
 * FXAA (GL_LINEAR / GL_REPEAT sampling), blended over rendering.clear_color and read back as RGB8,
 * top-down.  rgb_out: host buffer of width*height*3 bytes (window resolution), may be NULL. */
int sng_display_frame(sng_ctx* ctx, uint8_t* rgb_out, uint64_t capacity);
/* Display::save_image: display_frame, then <folder>/output-NNN.png (NNN = ++image count, 3 digits);
 * *written = 0 once the count exceeds output.img_count (default: the camera path's frames).  folder
 * NULL/"" = the scene JSON's output.folder.  Parameters "record", "img_count", "img_count_max". */
int sng_save_image(sng_ctx* ctx, const char* folder, int32_t* written);
/* host: 8-bit RGB (3) / RGBA (4) PNG writer (stbi_write_png) */
int sng_image_write_png(const char* path, const uint8_t* pixels, int32_t width, int32_t height, int32_t channels);
/* host-only: load a scene JSON and play n_frames of its animation without a device; per frame the
 * camera (mat4x3, column-major), light positions [n_lights][3] and object positions [n_objects][3].
 * playing / animation_speed < 0 keep the JSON's move_on_start / animation_speed. */
int sng_animation_probe(const char* scene_json, uint32_t n_frames, int32_t playing, float animation_speed, float* cameras,
                        float* light_pos, uint32_t light_cap, float* object_pos, uint32_t object_cap, uint32_t* n_lights,
                        uint32_t* n_objects);
/* Testbed::render_nerf (testbed_nerf.cu:2679-2837): the instant-NGP tracer (NerfTracer::trace 2279-2401,
 * composite_kernel_nerf 577-788, shade_kernel_nerf 1788-1828) into d_nerf_rgba / d_nerf_depth at NeRF
 * resolution; parameters "render_mode" (ERenderMode) and "depth_scale".  row_begin/row_end are NeRF rows. */
int sng_render_nerf_ngp(sng_ctx* ctx, const sng_frame_params* params, sng_frame_result* out);
/* ---- online training (BASELINE config 5; Testbed::train_nerf, testbed_nerf.cu:3298-3780) ----------
 * Training images: n RGBA8 sRGB images of w x h (0x00FF00FF = masked pixel), one camera per image
 * as a column-major mat4x3 in NGP space (c0 c1 c2 c3, i.e. nerf_matrix_to_ngp already applied,
 * nerf_loader.h:101-120), focal lengths in pixels, principal points in uv.  The model (config,
 * aabb, cascades) is the one set by sng_set_nerf_model / sng_load_snapshot. */
typedef struct {
    uint32_t step;                              /* training steps done */
    float loss;                                 /* loss of the last step (NerfCounters::update_after_training) */
    uint32_t rays_per_batch;                    /* adapted to reach the target batch */
    uint32_t measured_batch;                    /* compacted samples of the last step */
    uint32_t measured_batch_before_compaction;
    float ms;                                   /* device time of the call */
    /* param train_kernel_times = 1: each stage's device time per step (HIP events), averaged over timed_steps */
    float ms_generate, ms_network, ms_loss, ms_grad_clear, ms_field, ms_dw, ms_optimizer;
    uint32_t timed_steps;
    uint32_t reserved[2];
} sng_train_stats;
/* 8-bit PNG -> RGBA8 (host): the dataset loader's image decode (nerf_loader.cu, stb_image); out may be NULL to query the size */
int sng_image_load_png(const char* path, uint8_t* out_rgba8, uint64_t capacity, int32_t* width, int32_t* height);
int sng_train_set_dataset(sng_ctx* ctx, uint32_t n_images, uint32_t width, uint32_t height, const uint8_t* rgba8, const float* xforms_4x3,
                          const float* focal_px, const float* principal_uv);
/* Lens (common.h:188-205): mode 0 Perspective, 1 OpenCV {k1 k2 p1 p2}, 2 F-Theta {p0..p4, w, h}, 3 LatLong,
 * 4 OpenCV fisheye {k1 k2 k3 k4}, 5 Equirectangular -- what read_lens (nerf_loader.cu:175-239) takes from a
 * transforms.json / frame, and TrainingImageMetadata::lens */
typedef struct { int32_t mode; float params[7]; } sng_lens;
/* the training images' lenses, one per image of sng_train_set_dataset (NULL / 0: all Perspective, also the state
 * after sng_train_set_dataset); generate_training_samples_nerf's uv_to_ray(..., lens) (testbed_nerf.cu:890-905) and
 * mark_untrained_density_grid's pos_to_uv / uv_to_ray round trip (testbed_nerf.cu:112-141) use them */
int sng_train_set_lens(sng_ctx* ctx, const sng_lens* lenses, uint32_t n);
/* Testbed::Nerf::render_lens: the NeRF camera rays go through it when param render_with_lens_distortion is set
 * (render_nerf_with_buffers, testbed_nerf.cu:2504; uv_to_ray 403-447).  sng_load_snapshot sets it to the
 * dataset's first lens (load_nerf_post, testbed_nerf.cu:3051-3052).  NULL: Perspective. */
int sng_set_render_lens(sng_ctx* ctx, const sng_lens* lens);
int sng_get_render_lens(sng_ctx* ctx, sng_lens* out);
/* Testbed::set_camera_to_training_view (testbed.cu:453-469): camera, relative focal length, screen centre
 * (1 - principal point) and render lens of training image `view`, render_with_lens_distortion on */
int sng_set_camera_to_training_view(sng_ctx* ctx, int32_t view);
/* Testbed::reset_network's training state: fp32 master weights from the current model, zero
 * moments, m_rng = pcg32(seed), density_grid_rng = pcg32(m_rng.next_uint()) (testbed.cu:3654-3667) */
int sng_train_reset(sng_ctx* ctx, uint64_t seed);
/* n_steps x (training_prep_nerf schedule + train_nerf_step + optimizer step); afterwards the EMA
 * weights and the trained density grid are the render path's model */
int sng_train(sng_ctx* ctx, uint32_t n_steps, sng_train_stats* stats);
/* snapshot fields of the trained model: params fp16 (tcnn order) and density_grid fp16 */
int sng_train_export(sng_ctx* ctx, uint16_t* params_out, uint64_t n_params, uint16_t* density_grid_out, uint64_t n_cells);
/* parity hook: run train_nerf_step up to `stage` (1 samples, 2 network outputs, 3 loss, 4 gradients)
 * without an optimizer step, then copy the named buffer ("ctrl", "ray_indices", "rays", "numsteps",
 * "coords", "mlp_out", "coords_c", "dloss", "loss", "grads", "acts", "grid", "master") to host */
int sng_train_debug(sng_ctx* ctx, int stage, const char* buffer, void* out, uint64_t capacity_bytes, uint64_t* size_bytes);

/* ---- multi-GPU step schedule --------------------------------------------------
 * trace_alt sizes each wavefront iteration from the FRAME-wide alive count
 * (n_steps = clamp(2^21 / n_alive, 1, 8), testbed_nerf.cu:2180-2190).  A rank that renders one row
 * band (sng_frame_params.row_begin/row_end) reproduces the single-GPU frame bit for bit only if it
 * uses that frame-wide count, so with a communicator or reducer attached each iteration sums the
 * alive rays of every band's own rows across ranks (one uint32 all-reduce) before stepping.
 * The bands of all ranks must tile [0, height) without overlap, and every rank renders every frame. */
#define SNG_COMM_ID_BYTES 128
/* ncclGetUniqueId: rank 0 calls it and broadcasts the bytes to the other ranks */
int sng_comm_unique_id(uint8_t out_id[SNG_COMM_ID_BYTES]);
/* ncclCommInitRank on the context's device (RCCL over xGMI); unique_id NULL detaches */
int sng_set_comm(sng_ctx* ctx, const uint8_t* unique_id, int rank, int world);
/* host-side alternative (tests, gloo): fn sums values[0..n) over all ranks in place, returns 0 on
 * success; called once per wavefront iteration after a stream sync.  fn NULL detaches. */
typedef int (*sng_sched_reduce_fn)(uint32_t* values, uint32_t n, void* user);
int sng_set_sched_reducer(sng_ctx* ctx, sng_sched_reduce_fn fn, void* user);
/* Schedule replay (profiling: one GPU times a band exactly as its rank renders it under sng_set_comm).
 * records: the reduced arrays of one frame in call order, each as {n, v[0..n)} -- what a host reducer
 * returns, e.g. recorded at world size 1 over the full frame.  Every reduction point of the following frames
 * copies its record to the device asynchronously on the context's stream (no host sync, no communicator);
 * the cursor restarts at each frame, and a frame whose reductions differ from the records fails with
 * SNG_ERR_STATE.  records NULL detaches; n_words 0 with records non-NULL is SNG_ERR_INVALID.  Excludes a
 * communicator or host reducer. */
int sng_set_sched_replay(sng_ctx* ctx, const uint32_t* records, uint64_t n_words);
/* Final composition of a banded frame ("a final RCCL gather to GPU 0 of RGBA8"): rank r's
 * final rows [bounds[r], bounds[r+1]) as RGBA8 (the sng_final_rgba8 encoding) go to rank 0 over the
 * attached communicator -- grouped ncclSend / ncclRecv, each band received straight into its rows of
 * d_frame (rank 0: device buffer of width x height uint32; ignored on other ranks).  bounds: world + 1
 * row boundaries, the same on every rank.  Enqueued on hip_stream (NULL: the context's stream); every
 * rank calls it once per frame.  The reference renders on one GPU; its per-view copy-back is
 * testbed.cu:5126-5127. */
int sng_gather_rgba8(sng_ctx* ctx, const int32_t* bounds, uint32_t* d_frame, void* hip_stream);
/* in-place sum of n uint32 on the device over the attached communicator (band balancing: per-rank times) */
int sng_comm_allreduce_u32(sng_ctx* ctx, uint32_t* d_values, uint64_t n, void* hip_stream);

int sng_synchronize(sng_ctx* ctx);
int sng_copy_to_host(sng_ctx* ctx, const void* d_src, void* h_dst, uint64_t n_bytes);
/* device-to-device copy on the caller's stream (frame tiles -> collective buffers) */
int sng_copy_device(sng_ctx* ctx, const void* d_src, void* d_dst, uint64_t n_bytes, void* hip_stream);
/* curandState_t arrays (init_rand_state, synerfgine/common.cu:22-26) as 6 x u32 (v0..v4, d) per pixel */
int sng_get_rng_states(sng_ctx* ctx, int which /*0 nerf,1 mesh*/, uint32_t* out, uint64_t n_states);
int sng_set_rng_states(sng_ctx* ctx, int which, const uint32_t* in, uint64_t n_states);

/* ---- host utilities (A13) -------------------------------------------------- */
/* TriangleBvhWithBranchingFactor<2>::build (triangle_bvh.cu:615-692): tris reordered in place */
int sng_bvh_build(float* tris /* n x 9 */, uint32_t n_tris, uint32_t prims_per_leaf, float* nodes_out /* cap x 8 */, uint32_t cap, uint32_t* n_nodes);

#ifdef __cplusplus
}
#endif
