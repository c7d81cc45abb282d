// host.h -- the host runtime's internal declarations: the context (struct sng_ctx, the C ABI's opaque handle),
// device buffers, the scene's host objects, and the functions the runtime's translation units share:
//   capi.cpp          the C ABI (include/sng.h), context create / destroy, small utilities
//   host_params.cpp   the parameter table (sng_set_param keys with their reference members)
//   host_scene.cpp    OBJ + BVH build, scene JSON (Engine::set_virtual_world), camera, animation
//   host_render.cpp   model upload, resize, the NeRF trace and the hybrid frame (Engine::frame)
//   host_train.cpp    online training (Testbed::train_nerf)
//   host_snapshot.cpp .ingp load / save (Testbed::load_snapshot / save_snapshot)
#pragma once
#include "../../include/sng.h"

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <mutex>
#include <sstream>
#include <stack>
#include <string>
#include <vector>

#include "json.h"
#include "sng_internal.h"
#include <array>
#include "train.h"

using namespace sng;

#define HIPCHK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) throw SngError(SNG_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

namespace sng_host {

extern thread_local std::string g_err;   // sng_last_error

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return SNG_OK;
    } catch (const SngError& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return SNG_ERR_INVALID;
    }
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void ensure(size_t n) {
        if (n <= bytes && p) return;
        if (p) HIPCHK(hipFree(p));
        p = nullptr;
        bytes = 0;
        if (n == 0) return;
        HIPCHK(hipMalloc(&p, n));
        bytes = n;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

uint16_t f2h_host(float f);
const std::vector<uint32_t>& xorwow_seq_tables();
void upload(DevBuf& b, const void* src, size_t n);
template <typename T>
std::vector<T> download(const DevBuf& b, size_t n) {
    std::vector<T> h(n);
    if (n) HIPCHK(hipMemcpy(h.data(), b.p, n * sizeof(T), hipMemcpyDeviceToHost));
    return h;
}

// scene (host_scene.cpp)
std::vector<Tri> load_obj(const std::string& path);
std::vector<BvhNode> build_bvh(std::vector<Tri>& tris, uint32_t ppl);
m3 inverse3(const m3& M);
m3 rolling_shutter_rotation(const m3& M);

// ---- animation: cam_path.cuh:30-143, light.cuh:39-49, virtual_object.cuh:53-64 ----
struct CamKeyframe { f3 view, at; float zoom; };
struct CamPathState {           // sng::CamPath
    std::vector<CamKeyframe> keys;
    int total_time_ms = 10000, fps = 24, total_frames = 0, frames_between = 1, current_frame = 0, current_keyframe = 0;
    bool playing = false, present = false;
};
struct LightAnim { bool on = false; f3 start{}, end{}; float ratio = 0.0f, step = 0.0f; };
struct ObjAnim { float angle = 0.0f; f3 axis{0.0f, 1.0f, 0.0f}, centre{0.0f, 0.0f, 0.0f}; };

struct HostObject {
    std::string file;
    std::vector<Tri> tris;
    std::vector<BvhNode> nodes;
    std::vector<BvhWide> wide;    // traversal layout of `nodes` (wide_bvh), empty if not representable
    int root_ref = 0;
    m3 rot;
    f3 pos;
    float scale = 1.0f;
    int mat = 0;
    ObjAnim anim;
    DevBuf d_nodes, d_tris, d_trit, d_wide;
};

bool wide_bvh(const std::vector<BvhNode>& nodes, std::vector<BvhWide>& wide, int& root_ref);
const std::map<std::string, double>& default_params();

}  // namespace sng_host

using namespace sng_host;

struct sng_ctx {
    int device = 0;
    int n_cus = 256;
    hipStream_t s_nerf = nullptr, s_rt = nullptr;
    hipEvent_t ev_start = nullptr, ev_rt0 = nullptr, ev_rt1 = nullptr, ev_nerf0 = nullptr, ev_nerf1 = nullptr, ev_shadow1 = nullptr, ev_end = nullptr, ev_rt_go = nullptr, ev_fused0 = nullptr, ev_fused1 = nullptr, ev_os0 = nullptr, ev_os1 = nullptr, ev_alive = nullptr, ev_brick = nullptr;
    std::vector<hipEvent_t> net_events;
    std::vector<hipEvent_t> train_events;   // train_kernel_times: the stages of a training step

    // model
    bool has_model = false;
    sng_nerf_config cfg{};
    NetworkDev net;
    DevBuf d_wfrag, d_grid, d_levels;
    std::vector<LevelInfo> levels;
    uint64_t n_params = 0;
    uint32_t max_cascade = 0;
    float cone = 0.0f;
    aabb box{};

    // occupancy
    bool has_bitfield = false;
    DevBuf d_bitfield, d_occ_linear, d_grid_f16, d_grid_f32, d_partial, d_mean;
    DevBuf d_occ_brick, d_occ_brick_aux;   // OccBrick blob (sng_math.h) + {4096 flags, n_bricks}
    uint32_t occ_brick_n = 0;              // occupied bricks (host copy, read back lazily)
    bool occ_brick_dirty = false;

    // camera (Testbed)
    float cam[12] = {1, 0, 0, 0, -1, 0, 0, 0, -1, 0.5f, 0.5f, 2.0f};
    // View::camera1 / rolling_shutter (testbed.h:1032,1042; Engine: camera1 = camera0 unless a camera
    // path renders with a shutter, testbed.cu:2849-2850): sng_set_motion_blur
    bool has_cam1 = false;
    float cam1[12] = {};
    float rolling_shutter[4] = {0.0f, 0.0f, 0.0f, 1.0f};
    // Testbed::Nerf::render_lens (testbed.h; the dataset's metadata[0].lens at load, testbed_nerf.cu:3051-3053),
    // applied when param render_with_lens_distortion is set (testbed_nerf.cu:2504)
    Lens render_lens{};
    float m_scale = 1.5f;
    // NerfDataset::scale / offset as the loaded snapshot held them (json_binding.h:108-132), written
    // back by save_snapshot; nerf_synthetic's values until a snapshot supplies its own
    double ds_scale = 0.33;
    f3 ds_offset = {0.5f, 0.5f, 0.5f};
    // animation state (Engine::m_camera_path, m_anim_speed / m_enable_animations, per light / object)
    CamPathState campath;
    std::vector<LightAnim> light_anim;
    std::vector<ObjAnim> obj_anim;
    float anim_speed = 0.0f;
    bool animations = false;
    uint64_t anim_frames = 0;
    // display stage (Display::present / save_image, display.cu:265-322)
    f3 clear_color{0.0f, 0.0f, 0.0f};   // Engine::m_default_clear_color (rendering.clear_color, engine.cu:161-163)
    std::string out_folder;             // output.folder (engine.cu:54-64)
    bool record = false;                // output.record
    int img_count = 0, img_count_max = 1;
    DevBuf display_rgb;
    f3 up = {0.0f, 1.0f, 0.0f};
    float rel_focal[2] = {0, 0};
    int fov_axis = 1;
    float zoom = 1.0f;
    float screen_center[2] = {0.5f, 0.5f};

    std::map<std::string, double> params = default_params();

    // window / resolution
    int win[2] = {0, 0};
    int nerf_res[2] = {0, 0}, mesh_res[2] = {0, 0};
    int vo_scale_eff = 1;
    int last_res_factor = -1;

    // buffers
    DevBuf nerf_rgba, nerf_depth, nerf_pos, nerf_nrm;
    DevBuf ray_ot[2], ray_di[2], ray_rgba[2], ray_depth[2], ray_mw[2], ray_lt[2], ray_lo[2], ray_kk[2];
    DevBuf samp, coords, net_out, ctrl;
    size_t ray_cap = 0, sample_cap = 0;
    DevBuf mesh_o, mesh_d, acc_rgba, acc_depth, final_rgba, final_depth;
    DevBuf rt_rec, rt_lc, rt_srec, rt_mask, rt_head, rt_work;   // deferred-shadow raytracer queues (+ work counters)
    DevBuf rt_plist, rt_pcount, rt_rval;   // per-pixel record lists + record colour terms (tile path kernel)
    DevBuf rt_tile_cost, rt_tile_order;   // previous frame's per-tile cost -> this frame's tile order
    DevBuf rt_started;                    // rt_first: the path kernel's landing flag (frame sequence number)
    uint32_t frame_seq = 0, rt_wait_seq = 0;
    DevBuf fused_work;                     // ray-queue cursor of the fused NeRF kernel
    DevBuf shadow_scratch;                 // NeRF shadow pass: light samples + terms per neighbour slot (launch_shadows)
    DevBuf tail_live;                      // tail iterations' alive counts as a difference array (reference slots)
    DevBuf sched_hint;                     // steps of every iteration of the last frame (sizes the msr rounds)
    uint64_t sched_hint_key = 0;           // the schedule the hints were written under (0: none; see trace_nerf)
    DevBuf msr_hist;                       // multi-step rounds: [4][MSR_KMAX] per-iteration deaths / samples
    DevBuf msr_alpha;                      // multi-step rounds: per-sample alpha, msr_count -> msr_commit
    DevBuf march_log;                      // diagnostics (param march_log): per iteration {alive, steps, samples}
    DevBuf spec_t;                         // speculative tail rounds: march t of every sample ([sample][ray])
    DevBuf spec_hint;                      // per NeRF pixel: 1 + the iteration its ray ended at last frame (u8, 0 unknown)
    uint64_t spec_hint_px = 0;
    uint64_t spec_hint_key = 0;            // the view the hints were written for (spec_view_key); another view reads none
    uint64_t spec_prev_view = 0;           // the last traced frame's view (spec_view_key); a repeat writes hints
    uint64_t model_epoch = 0;              // bumped when the model or its occupancy changes (part of that key)
    DevBuf spec_pre, spec_pre_depth;       // spec_prepare: per network sample {rgb, alpha} and depth
    DevBuf band_rgba8;                     // sng_gather_rgba8: this rank's band as RGBA8
    uint32_t spec_rounds = 0;              // rounds enqueued by the last trace
    uint32_t spec_rounds_next = 0;         // nerf_spec_adapt: the round count the next trace uses (0: nerf_spec_rounds)
    uint32_t msr_rounds = 0;               // multi-step speculative rounds of the last trace that committed iterations
    DevBuf rt_counts;                      // rt_count frames: path / shadow kernel {queries, box tests, triangle tests}
    bool fused_last = false;               // the last trace finished in the fused kernel
    uint32_t fused_k0 = 0;                 // ... from this iteration on
    DevBuf os_hist, os_state;              // one-step regime: death / no-sample histograms, OnestepState
    OnestepState* h_os = nullptr;          // pinned readback of the regime's length
    bool os_ran = false;                   // the last trace ran a one-step regime (ev_os0 .. ev_os1)
    uint32_t os_k = 0, os_J = 0;           // ... from iteration os_k for os_J iterations (all segments)
    uint64_t rt_tile_key = 0;             // band geometry the costs belong to

    DevBuf rng_nerf, rng_mesh;
    DevBuf rng_mesh_sp;            // rt_rng = 1: one XORWOW stream per (pixel, light sample), [6][n_px * samples]
    uint64_t rng_sp_key = 0;
    uint32_t n_rng_nerf = 0, n_rng_mesh = 0;
    DevBuf d_seq;
    MarchCtrl* h_ctrl = nullptr;
    uint32_t* h_alive = nullptr;  // pinned readback [chunk][2], [6] spec_ok, [7] occupancy brick count
    SchedComm sched_comm;         // frame-wide step schedule across ranks (comm.cpp)
    DevBuf d_params;              // the model's fp16 parameter blob (tcnn order), training source

    // ---- online training (train.hip; Testbed::train_nerf, testbed_nerf.cu:3298-3780)
    struct Train {
        bool ready = false;
        uint32_t step = 0, grid_ema_step = 0;
        uint32_t rays_per_batch = 1u << 12;            // testbed.h:509
        uint32_t measured = 0, measured_before = 0;
        // the device copy of those (TrainSched) is the one the steps read and update; the host fields above are pushed
        // when set on the host (reset, snapshot load) and pulled when train_steps returns
        DevBuf sched;
        bool sched_dirty = true;
        // pinned readbacks of the device's batch sizes every 8 steps into two slots; reusing a slot waits for its
        // previous copy, so the host queues at most ~16 steps ahead and the grid-size estimate lags by at most that
        TrainSched* h_sched = nullptr;                 // [2]
        hipEvent_t sched_ev[2] = {nullptr, nullptr};
        bool sched_pending[2] = {false, false};
        uint32_t sched_slot = 0;
        uint32_t n_rays_est = 1u << 12;                // grid sizes only (n_rays_grid)
        hipStream_t s_gen = nullptr;                   // train_overlap: the next step's generate
        hipEvent_t ev_gen = nullptr, ev_loss = nullptr;
        bool pregen = false;                           // the next step's samples are queued on s_gen (train_overlap_tail)
        Pcg32 rng{}, grid_rng{};
        int w = 0, h = 0, n_images = 0;
        DevBuf pixels, xforms, xforms_ray, focal, pp;
        DevBuf lens;                                   // [n_images] Lens (sng_train_set_lens); h_lens empty: all Perspective
        DevBuf tscr;                                   // generate's sample distances [NERF_STEPS][rays_per_batch]
        std::vector<Lens> h_lens;
        DevBuf master, grads, m1, m2, steps, ema, p_train, p_infer, wfrag_train, wfrag_t;
        DevBuf adam_corr;                              // Adam's bias correction per step count (launch_train_adam_corr)
        DevBuf grads_h;                                // fp16 hash-grid gradients (train_grid_grad_f16)
        bool grads_h_used = false;                     // the last step's grid gradients are in grads_h
        uint32_t adam_corr_n = 0;                      // valid entries 1..adam_corr_n
        DevBuf grid, grid_tmp, grid_coords, grid_idx, grid_out;
        DevBuf ctrl, ray_indices, rays, numsteps, coords, mlp_out, coords_c, dloss, loss, acts, partial, rayrec, cnt_i, cbase_i;
        uint32_t target = 1u << 18;                    // m_training_batch_size (testbed.h:1103)
        float last_loss = 0.0f;
    } tr;
    bool mesh_reset = true;

    // scene (Engine)
    std::vector<HostObject> objs;
    std::vector<sng_light> lights;
    std::vector<sng_material> mats;
    DevBuf d_objs, d_lights, d_mats;
    DevBuf d_scene_blob;          // every object's nodes + triangles (traversal kernels copy it to LDS)
    uint32_t scene_f4 = 0, bvh_depth = 0;
    uint32_t bvh_stack = 0;       // stack entries per lane the scene's walks need (depth + 2)
    bool scene_dirty = true;

    double p(const char* k) const { return params.at(k); }
};

namespace sng_host {
// ---- shared by the runtime's files (defined where the comment says)
// host_render.cpp
void compute_levels(sng_ctx* c);
void set_model(sng_ctx* c, const sng_nerf_config* cfg, const uint16_t* params, uint64_t n);
void set_density_grid(sng_ctx* c, const uint16_t* grid, uint64_t n_cells);
void build_occ_brick(sng_ctx* c, hipStream_t s);
Volume make_volume(const sng_ctx* c);
void resize(sng_ctx* c);
f2 focal_for(const sng_ctx* c, const int res[2]);
void render_frame(sng_ctx* c, const sng_frame_params* fp, sng_frame_result* out);
void render_nerf_ngp(sng_ctx* c, const sng_frame_params* fp, sng_frame_result* out);
void spec_adapt(sng_ctx* c);
// host_scene.cpp
f3 cam_col(const sng_ctx* c, int i);
void set_cam_col(sng_ctx* c, int i, f3 v);
f3 look_at(const sng_ctx* c);
void set_look_at(sng_ctx* c, f3 pos);
void set_scale(sng_ctx* c, float scale);
void set_view_dir(sng_ctx* c, f3 dir);
float fov_to_focal(float degrees);
void upload_scene(sng_ctx* c);
int n_point_lights(const sng_ctx* c);
void shadow_scene(sng_ctx* c, ShadowArgs& sa);
void load_scene(sng_ctx* c, const std::string& path);
void campath_set_to_frame(sng_ctx* c);
void animate(sng_ctx* c);
// host_snapshot.cpp
struct ParsedSnapshot {
    sng_nerf_config cfg{};
    std::vector<uint16_t> params, grid;
    JValue root;
};
ParsedSnapshot parse_snapshot(const std::string& path);
void load_snapshot(sng_ctx* c, const std::string& path);
void save_snapshot(sng_ctx* c, const std::string& path, bool include_opt, bool compress);
// host_train.cpp
void train_drop_pregen(sng_ctx::Train& t);
void train_reset(sng_ctx* c, uint64_t seed);
void train_density_update(sng_ctx* c, hipStream_t s);
void train_forward_backward(sng_ctx* c, int stage, hipStream_t s, hipEvent_t* ev = nullptr, bool generated = false, hipEvent_t ev_loss = nullptr);
void train_steps(sng_ctx* c, uint32_t n_steps, sng_train_stats* out);
}  // namespace sng_host
