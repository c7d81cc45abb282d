// capi.cpp -- host runtime (C++) behind the C-ABI in include/sng.h.
//
// Mirrors the reference's host objects on the hot path:
//   Testbed   : model/snapshot, density bitfield, camera (testbed.cu:405-425, 3562, 4133-4140, 4878-5015)
//   NerfTracer: the device-driven wavefront loop (testbed_nerf.cu:2128-2277)
//   RayTracer : mesh rays, path tracing, overlay (synerfgine/raytracer.cu:260-392)
//   Engine    : scene JSON, rendering.* keys, resize and frame (synerfgine/engine.cu:21-433)
//
// The runtime is split by subsystem (host.h lists its files); this file holds the C ABI itself, the context's
// creation and destruction, and the small utilities the others share.
#include "host.h"

namespace sng_host {

thread_local std::string g_err;

// ---- fp16 host conversion (RTE) ------------------------------------------------
uint16_t f2h_host(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
    if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00u);
    if (ax >= 0x47800000u) return (uint16_t)(sign | 0x7c00u);
    if (ax >= 0x38800000u) {
        uint32_t mant = ax & 0x7fffffu, e = (ax >> 23) - 127 + 15;
        uint32_t h = (e << 10) | (mant >> 13), rem = mant & 0x1fffu;
        if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
        return (uint16_t)(sign | h);
    }
    if (ax < 0x33000000u) return (uint16_t)sign;
    uint32_t e = ax >> 23, mant = (ax & 0x7fffffu) | 0x800000u, shift = 126 - e;
    uint32_t h = mant >> shift, rem = mant & ((1u << shift) - 1u), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
}

// ---- cuRAND XORWOW subsequence matrices M^(2^67 * 2^k), k < 32 -------------------
struct Gf2 { uint32_t col[160][5]; };
void gf2_apply(const Gf2& m, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int j = 0; j < 160; ++j)
        if ((in[j >> 5] >> (j & 31)) & 1u)
            for (int w = 0; w < 5; ++w) r[w] ^= m.col[j][w];
    std::memcpy(out, r, sizeof(r));
}
void gf2_square(const Gf2& a, Gf2& out) {
    Gf2 r;
    for (int j = 0; j < 160; ++j) gf2_apply(a, a.col[j], r.col[j]);
    out = r;
}
const std::vector<uint32_t>& xorwow_seq_tables() {
    static std::vector<uint32_t> tab;
    static std::once_flag once;
    std::call_once(once, [] {
        Gf2 m;
        for (int j = 0; j < 160; ++j) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[j >> 5] = 1u << (j & 31);
            uint32_t t = v[0] ^ (v[0] >> 2);
            v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
            v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
            std::memcpy(m.col[j], v, sizeof(v));
        }
        for (int i = 0; i < 67; ++i) gf2_square(m, m);
        tab.resize((size_t)32 * 160 * 5);
        for (int k = 0; k < 32; ++k) {
            std::memcpy(&tab[(size_t)k * 800], m.col, 800 * 4);
            gf2_square(m, m);
        }
    });
    return tab;
}

void upload(DevBuf& b, const void* src, size_t n) {
    b.ensure(n);
    if (n) HIPCHK(hipMemcpy(b.p, src, n, hipMemcpyHostToDevice));
}

void ctx_create(const sng_ctx_desc* desc, sng_ctx** out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw SngError(SNG_ERR_NOGPU, "no HIP device visible");
    int dev = desc ? desc->device_id : 0;
    if (dev < 0 || dev >= n) throw SngError(SNG_ERR_INVALID, "device_id out of range");
    HIPCHK(hipSetDevice(dev));
    auto* c = new sng_ctx();
    c->device = dev;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, dev));
    c->n_cus = prop.multiProcessorCount;
    // the NeRF wavefront (short, dependent launches) gets the higher queue priority so its
    // workgroups are dispatched ahead of the long raytracer grids it overlaps with
    int prio_lo = 0, prio_hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIPCHK(hipStreamCreateWithPriority(&c->s_nerf, hipStreamNonBlocking, prio_hi));
    HIPCHK(hipStreamCreateWithPriority(&c->s_rt, hipStreamNonBlocking, prio_lo));
    for (hipEvent_t* e : {&c->ev_start, &c->ev_rt0, &c->ev_rt1, &c->ev_nerf0, &c->ev_nerf1, &c->ev_shadow1, &c->ev_end, &c->ev_rt_go, &c->ev_fused0, &c->ev_fused1, &c->ev_os0, &c->ev_os1, &c->ev_alive, &c->ev_brick}) HIPCHK(hipEventCreate(e));
    HIPCHK(hipHostMalloc((void**)&c->h_ctrl, sizeof(MarchCtrl), hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&c->h_alive, 8 * sizeof(uint32_t), hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&c->h_os, sizeof(OnestepState), hipHostMallocDefault));
    float rf = fov_to_focal(50.625f);   // Testbed::reset_camera -> set_fov(50.625) (testbed.cu:480)
    c->rel_focal[0] = c->rel_focal[1] = rf;
    // reset_camera matrix: transpose(mat3x4{1,0,0,0.5; 0,-1,0,0.5; 0,0,-1,0.5}), then pos -= scale*dir
    c->m_scale = 1.5f;
    set_cam_col(c, 3, cam_col(c, 3) - cam_col(c, 2) * 0.0f);
    c->cam[9] = 0.5f; c->cam[10] = 0.5f; c->cam[11] = 0.5f;
    set_cam_col(c, 3, cam_col(c, 3) - c->m_scale * cam_col(c, 2));
    *out = c;
}

void ctx_destroy(sng_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    comm_destroy(c->sched_comm);
    for (auto& o : c->objs) { o.d_nodes.release(); o.d_tris.release(); o.d_trit.release(); o.d_wide.release(); }
    for (DevBuf* b : {&c->d_wfrag, &c->d_grid, &c->d_levels, &c->d_bitfield, &c->d_occ_linear, &c->d_grid_f16, &c->d_grid_f32, &c->d_partial, &c->d_mean, &c->nerf_rgba,
                      &c->nerf_depth, &c->nerf_pos, &c->nerf_nrm, &c->samp, &c->coords, &c->net_out, &c->ctrl, &c->mesh_o, &c->mesh_d, &c->acc_rgba,
                      &c->acc_depth, &c->final_rgba, &c->final_depth, &c->rt_rec, &c->rt_lc, &c->rt_srec, &c->rt_mask, &c->rt_head, &c->rt_plist, &c->rt_pcount, &c->rt_rval, &c->rt_work, &c->rt_tile_cost, &c->rt_tile_order, &c->fused_work, &c->rng_nerf, &c->rng_mesh, &c->rng_mesh_sp, &c->d_seq, &c->d_objs, &c->d_lights, &c->d_mats, &c->d_scene_blob,
                      &c->os_hist, &c->os_state, &c->d_occ_brick, &c->d_occ_brick_aux, &c->rt_counts, &c->spec_t, &c->tail_live, &c->sched_hint, &c->msr_hist, &c->march_log, &c->spec_pre, &c->spec_pre_depth, &c->band_rgba8, &c->display_rgb})
        b->release();
    for (int b = 0; b < 2; ++b) { c->ray_ot[b].release(); c->ray_di[b].release(); c->ray_rgba[b].release(); c->ray_depth[b].release(); c->ray_mw[b].release(); c->ray_lt[b].release(); c->ray_lo[b].release(); c->ray_kk[b].release(); }
    for (hipEvent_t e : {c->ev_start, c->ev_rt0, c->ev_rt1, c->ev_nerf0, c->ev_nerf1, c->ev_shadow1, c->ev_end, c->ev_rt_go, c->ev_fused0, c->ev_fused1, c->ev_os0, c->ev_os1, c->ev_alive, c->ev_brick}) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->net_events) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->train_events) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->tr.sched_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->tr.ev_gen) (void)hipEventDestroy(c->tr.ev_gen);
    if (c->tr.ev_loss) (void)hipEventDestroy(c->tr.ev_loss);
    if (c->tr.s_gen) (void)hipStreamDestroy(c->tr.s_gen);
    if (c->tr.h_sched) (void)hipHostFree(c->tr.h_sched);
    (void)hipHostFree(c->h_ctrl);
    (void)hipHostFree(c->h_alive);
    (void)hipHostFree(c->h_os);
    if (c->sched_comm.replay) (void)hipHostFree(c->sched_comm.replay);
    (void)hipStreamDestroy(c->s_nerf);
    (void)hipStreamDestroy(c->s_rt);
    delete c;
}


}  // namespace sng_host


// =====================================================================================
// C ABI
// =====================================================================================
extern "C" {

const char* sng_last_error(void) { return g_err.c_str(); }
int sng_abi_version(void) { return SNG_ABI_VERSION; }
int sng_device_count(int* out) {
    return guarded([&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        *out = n;
    });
}
int sng_ctx_create(const sng_ctx_desc* desc, sng_ctx** out) { return guarded([&] { ctx_create(desc, out); }); }
int sng_ctx_destroy(sng_ctx* ctx) { return guarded([&] { ctx_destroy(ctx); }); }

int sng_load_snapshot(sng_ctx* c, const char* path) { return guarded([&] { HIPCHK(hipSetDevice(c->device)); load_snapshot(c, path); }); }
int sng_frame_buffer(sng_ctx* c, const char* name, void* out, uint64_t cap, uint64_t* size) {
    return guarded([&] {
        if (!c || !name) throw SngError(SNG_ERR_INVALID, "null context or name");
        HIPCHK(hipSetDevice(c->device));
        const std::map<std::string, DevBuf*> bufs = {{"coords", &c->coords}, {"net_out", &c->net_out}, {"samp", &c->samp}, {"march_log", &c->march_log},
                                                       {"rt_tile_cost", &c->rt_tile_cost}, {"rt_tile_order", &c->rt_tile_order}};
        auto it = bufs.find(name);
        if (it == bufs.end()) throw SngError(SNG_ERR_INVALID, std::string("unknown frame buffer ") + name);
        HIPCHK(hipDeviceSynchronize());
        if (size) *size = it->second->bytes;
        if (out) HIPCHK(hipMemcpy(out, it->second->p, std::min<uint64_t>(cap, it->second->bytes), hipMemcpyDeviceToHost));
    });
}
int sng_rt_counters(sng_ctx* c, uint64_t* out) {
    return guarded([&] {
        if (!c || !out) throw SngError(SNG_ERR_INVALID, "null context or output");
        HIPCHK(hipSetDevice(c->device));
        std::memset(out, 0, 6 * sizeof(uint64_t));
        if (!c->rt_counts.p) return;
        HIPCHK(hipStreamSynchronize(c->s_rt));
        HIPCHK(hipMemcpy(out, c->rt_counts.p, 6 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
int sng_save_snapshot(sng_ctx* c, const char* path, int32_t include_optimizer_state, int32_t compress) {
    return guarded([&] {
        if (!c || !path) throw SngError(SNG_ERR_INVALID, "null context or path");
        HIPCHK(hipSetDevice(c->device));
        save_snapshot(c, path, include_optimizer_state != 0, compress != 0);
    });
}
int sng_snapshot_probe(const char* path, sng_nerf_config* cfg, uint64_t* n_params, uint64_t* n_grid_cells, uint16_t* params_out,
                       uint64_t params_cap, uint16_t* grid_out, uint64_t grid_cap) {
    return guarded([&] {
        ParsedSnapshot ps = parse_snapshot(path);
        if (cfg) *cfg = ps.cfg;
        if (n_params) *n_params = ps.params.size();
        if (n_grid_cells) *n_grid_cells = ps.grid.size();
        if (params_out) {
            if (params_cap < ps.params.size()) throw SngError(SNG_ERR_INVALID, "params buffer too small");
            std::memcpy(params_out, ps.params.data(), ps.params.size() * 2);
        }
        if (grid_out) {
            if (grid_cap < ps.grid.size()) throw SngError(SNG_ERR_INVALID, "grid buffer too small");
            std::memcpy(grid_out, ps.grid.data(), ps.grid.size() * 2);
        }
    });
}
uint64_t sng_nerf_param_count(const sng_nerf_config* cfg) {
    sng_ctx tmp;
    tmp.cfg = *cfg;
    compute_levels(&tmp);
    return tmp.n_params;
}
int sng_set_nerf_model(sng_ctx* c, const sng_nerf_config* cfg, const uint16_t* params, uint64_t n) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); set_model(c, cfg, params, n); });
}
int sng_set_density_grid(sng_ctx* c, const uint16_t* grid, uint64_t n) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); set_density_grid(c, grid, n); });
}
int sng_get_bitfield(sng_ctx* c, uint8_t* out, uint64_t n) {
    return guarded([&] {
        if (!c->has_bitfield) throw SngError(SNG_ERR_STATE, "no bitfield");
        if (n != c->d_bitfield.bytes) throw SngError(SNG_ERR_INVALID, "bitfield size is " + std::to_string(c->d_bitfield.bytes));
        HIPCHK(hipMemcpy(out, c->d_bitfield.p, n, hipMemcpyDeviceToHost));
    });
}
int sng_get_density_mean(sng_ctx* c, float* out) {
    return guarded([&] {
        if (!c->has_bitfield) throw SngError(SNG_ERR_STATE, "no bitfield");
        HIPCHK(hipMemcpy(out, c->d_mean.p, 4, hipMemcpyDeviceToHost));
    });
}
int sng_nerf_inference(sng_ctx* c, const float* coords, uint32_t stride, uint32_t n, uint16_t* out, int32_t layout, void* stream) {
    return guarded([&] {
        if (!c->has_model) throw SngError(SNG_ERR_STATE, "no model");
        if (stride < 7) throw SngError(SNG_ERR_INVALID, "NerfCoordinate stride must be >= 7 floats");
        if (layout < 0 || layout > 2) throw SngError(SNG_ERR_INVALID, "out_layout must be 0, 1 or 2");
        if (n == 0) return;
        launch_network(c->net, coords, stride, n, nullptr, out, layout, 0, (hipStream_t)stream);
        HIPCHK(hipGetLastError());
    });
}
int sng_hashgrid_encode(sng_ctx* c, const float* coords, uint32_t stride, uint32_t n, uint16_t* out, void* stream) {
    return guarded([&] {
        if (!c->has_model) throw SngError(SNG_ERR_STATE, "no model");
        if (stride < 3) throw SngError(SNG_ERR_INVALID, "stride must be >= 3 floats");
        launch_encode(c->net, coords, stride, n, out, (hipStream_t)stream);
        HIPCHK(hipGetLastError());
    });
}

int sng_sh_encode(sng_ctx* c, const float* coords, uint32_t stride, uint32_t dir_offset, uint32_t n, uint16_t* out, void* stream) {
    return guarded([&] {
        if (stride < dir_offset + 3) throw SngError(SNG_ERR_INVALID, "stride must cover dir_offset + 3 floats");
        HIPCHK(hipSetDevice(c->device));
        launch_sh_encode(coords, stride, dir_offset, n, out, (hipStream_t)stream);
        HIPCHK(hipGetLastError());
    });
}

int sng_load_virtual_scene(sng_ctx* c, const char* path) { return guarded([&] { load_scene(c, path); }); }
int sng_clear_virtual_scene(sng_ctx* c) {
    return guarded([&] {
        for (auto& o : c->objs) { o.d_nodes.release(); o.d_tris.release(); o.d_trit.release(); o.d_wide.release(); }
        c->objs.clear(); c->lights.clear(); c->mats.clear();
        c->scene_dirty = true;
    });
}
int sng_set_param(sng_ctx* c, const char* key, double v) {
    return guarded([&] {
        std::string k = key;
        if (k == "sshadows") k = "syn_shadow_samples";       // Engine::set_syn_samples (engine.cuh:29)
        else if (k == "nshadows") k = "nerf_shadow_samples"; // Engine::set_nerf_samples (engine.cuh:30-33)
        if (k == "animation_speed") {   // Engine::m_anim_speed / m_enable_animations (engine.cu:43-46)
            c->anim_speed = (float)v;
            c->animations = c->anim_speed > 0.0f;
            return;
        }
        if (k == "camera_path_playing") {   // CamPath::is_playing (Play / Pause)
            c->campath.playing = v != 0.0 && c->campath.keys.size() >= 2;
            return;
        }
        if (k == "record") { c->record = v != 0.0; return; }
        if (k == "img_count_max") { c->img_count_max = (int)v; return; }
        if (k == "camera_path_frame") {   // CamPath "Current Frame" slider -> set_to_frame
            c->campath.current_frame = std::max(0, (int)v);
            campath_set_to_frame(c);
            c->mesh_reset = true;
            return;
        }
        if (!default_params().count(k)) throw SngError(SNG_ERR_INVALID, "unknown parameter '" + k + "'");
        if (k == "rt_buffer_type" && !(v >= 0.0 && v <= 7.0 && v == std::floor(v)))
            throw SngError(SNG_ERR_INVALID, "rt_buffer_type is an ImgBufferType: 0 Final, 1 NextOrigin, 2 SrcOrigin, 3 NextDirection, 4 SrcDirection, 5 Normal, 6 Depth, 7 NerfShadow");
        if (k == "tonemap_curve" && !(v == 0.0 || v == 1.0 || v == 2.0 || v == 3.0))
            throw SngError(SNG_ERR_INVALID, "tonemap_curve is an ETonemapCurve: 0 Identity, 1 ACES, 2 Hable, 3 Reinhard");
        c->params[k] = v;
        c->mesh_reset = true;
        if (k == "rt_rng") c->rng_sp_key = 0;   // (re)setting it re-seeds the per-(pixel, sample) streams at the next frame
        if ((k == "fast_slab" || k == "scene_lds" || k == "bvh_wide") && !c->objs.empty()) upload_scene(c);
    });
}
int sng_get_param(sng_ctx* c, const char* key, double* v) {
    return guarded([&] {
        std::string k = key;
        if (k == "sshadows") k = "syn_shadow_samples";
        else if (k == "nshadows") k = "nerf_shadow_samples";
        if (k == "animation_speed") { *v = c->anim_speed; return; }
        if (k == "camera_path_playing") { *v = c->campath.playing ? 1.0 : 0.0; return; }
        if (k == "camera_path_frame") { *v = c->campath.current_frame; return; }
        if (k == "camera_path_total_frames") { *v = c->campath.present ? c->campath.total_frames : 0; return; }
        if (k == "record") { *v = c->record ? 1.0 : 0.0; return; }
        if (k == "img_count") { *v = c->img_count; return; }
        if (k == "img_count_max") { *v = c->img_count_max; return; }
        auto it = c->params.find(k);
        if (it == c->params.end()) throw SngError(SNG_ERR_INVALID, "unknown parameter '" + k + "'");
        *v = it->second;
    });
}
int sng_get_scene_counts(sng_ctx* c, uint32_t* no, uint32_t* nl, uint32_t* nm) {
    return guarded([&] {
        *no = (uint32_t)c->objs.size();
        *nl = (uint32_t)c->lights.size();
        *nm = (uint32_t)c->mats.size();
    });
}
int sng_get_object(sng_ctx* c, uint32_t i, sng_object_info* out) {
    return guarded([&] {
        if (i >= c->objs.size()) throw SngError(SNG_ERR_INVALID, "object index");
        const auto& o = c->objs[i];
        out->n_nodes = (uint32_t)o.nodes.size();
        out->n_tris = (uint32_t)o.tris.size();
        const f3 cols[3] = {o.rot.c0, o.rot.c1, o.rot.c2};
        for (int k = 0; k < 3; ++k) { out->rot[3 * k] = cols[k].x; out->rot[3 * k + 1] = cols[k].y; out->rot[3 * k + 2] = cols[k].z; }
        out->pos[0] = o.pos.x; out->pos[1] = o.pos.y; out->pos[2] = o.pos.z;
        out->scale = o.scale;
        out->mat_id = o.mat;
    });
}
int sng_get_object_bvh(sng_ctx* c, uint32_t i, float* nodes_out, float* tris_out) {
    return guarded([&] {
        if (i >= c->objs.size()) throw SngError(SNG_ERR_INVALID, "object index");
        const auto& o = c->objs[i];
        if (nodes_out) std::memcpy(nodes_out, o.nodes.data(), o.nodes.size() * sizeof(BvhNode));
        if (tris_out) std::memcpy(tris_out, o.tris.data(), o.tris.size() * sizeof(Tri));
    });
}
int sng_get_light(sng_ctx* c, uint32_t i, sng_light* out) {
    return guarded([&] { if (i >= c->lights.size()) throw SngError(SNG_ERR_INVALID, "light index"); *out = c->lights[i]; });
}
int sng_get_material(sng_ctx* c, uint32_t i, sng_material* out) {
    return guarded([&] { if (i >= c->mats.size()) throw SngError(SNG_ERR_INVALID, "material index"); *out = c->mats[i]; });
}

int sng_set_camera_view(sng_ctx* c, const float v[3], const float at[3], float scale) {
    return guarded([&] {
        set_view_dir(c, mk(v[0], v[1], v[2]));
        set_look_at(c, mk(at[0], at[1], at[2]));
        set_scale(c, scale);
        c->mesh_reset = true;
    });
}
int sng_set_camera_matrix(sng_ctx* c, const float m[12]) {
    return guarded([&] { std::memcpy(c->cam, m, 48); c->has_cam1 = false; c->mesh_reset = true; });
}
// Testbed::set_camera_to_training_view (testbed.cu:453-469): the training image's camera (its xform through
// get_xform_given_rolling_shutter at uv (0.5, 0.5), t 0: the quat round trip), relative focal length =
// focal / resolution[fov_axis], m_scale from the old look-at, render_with_lens_distortion on with the image's
// lens, screen centre 1 - principal point
int sng_set_camera_to_training_view(sng_ctx* c, int32_t view) {
    return guarded([&] {
        if (!c) throw SngError(SNG_ERR_INVALID, "null context");
        auto& t = c->tr;
        if (view < 0 || view >= t.n_images) throw SngError(SNG_ERR_INVALID, "no such training view");
        HIPCHK(hipSetDevice(c->device));
        const f3 old_look_at = look_at(c);
        float xf[12], fo[2], pp[2];
        HIPCHK(hipMemcpy(xf, t.xforms.as<float>() + 12 * (size_t)view, 48, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(fo, t.focal.as<float>() + 2 * (size_t)view, 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(pp, t.pp.as<float>() + 2 * (size_t)view, 8, hipMemcpyDeviceToHost));
        const m3 r = rolling_shutter_rotation({mk(xf[0], xf[1], xf[2]), mk(xf[3], xf[4], xf[5]), mk(xf[6], xf[7], xf[8])});
        set_cam_col(c, 0, r.c0); set_cam_col(c, 1, r.c1); set_cam_col(c, 2, r.c2); set_cam_col(c, 3, mk(xf[9], xf[10], xf[11]));
        c->has_cam1 = false;
        const float res = (float)(c->fov_axis == 0 ? t.w : t.h);
        c->rel_focal[0] = fo[0] / res;
        c->rel_focal[1] = fo[1] / res;
        c->m_scale = std::max(dot(old_look_at - cam_col(c, 3), cam_col(c, 2)), 0.1f);
        c->params["render_with_lens_distortion"] = 1.0;
        c->render_lens = t.h_lens.empty() ? Lens{} : t.h_lens[(size_t)view];
        c->screen_center[0] = 1.0f - pp[0];
        c->screen_center[1] = 1.0f - pp[1];
        c->mesh_reset = true;
    });
}
int sng_set_motion_blur(sng_ctx* c, const float camera1[12], const float rolling_shutter[4]) {
    return guarded([&] {
        c->has_cam1 = camera1 != nullptr;
        if (camera1) std::memcpy(c->cam1, camera1, 48);
        const float rs0[4] = {0.0f, 0.0f, 0.0f, 1.0f};
        std::memcpy(c->rolling_shutter, rolling_shutter ? rolling_shutter : rs0, 16);
    });
}
int sng_get_camera_matrix(sng_ctx* c, float m[12]) { return guarded([&] { std::memcpy(m, c->cam, 48); }); }
int sng_set_fov(sng_ctx* c, float deg) { return guarded([&] { c->rel_focal[0] = c->rel_focal[1] = fov_to_focal(deg); c->mesh_reset = true; }); }
int sng_get_focal_length(sng_ctx* c, int which, float out[2]) {
    return guarded([&] {
        // a pending res_factor change resizes first (the next frame would), so the focal length
        // reported is the one that frame uses
        if (c->win[0] > 0 && (int)c->p("res_factor") != c->last_res_factor) { HIPCHK(hipSetDevice(c->device)); resize(c); }
        const int* res = which == 0 ? c->nerf_res : c->mesh_res;
        f2 f = focal_for(c, res);
        out[0] = f.x; out[1] = f.y;
    });
}

int sng_set_window(sng_ctx* c, int32_t w, int32_t h) {
    return guarded([&] {
        if (w <= 0 || h <= 0) throw SngError(SNG_ERR_INVALID, "bad window size");
        HIPCHK(hipSetDevice(c->device));
        c->win[0] = w; c->win[1] = h;
        resize(c);
    });
}
int sng_get_resolution(sng_ctx* c, sng_resolution_info* out) {
    return guarded([&] {
        if (c->win[0] > 0 && (int)c->p("res_factor") != c->last_res_factor) { HIPCHK(hipSetDevice(c->device)); resize(c); }
        std::memset(out, 0, sizeof(*out));
        out->nerf_res[0] = c->nerf_res[0]; out->nerf_res[1] = c->nerf_res[1];
        out->mesh_res[0] = c->mesh_res[0]; out->mesh_res[1] = c->mesh_res[1];
        out->syn_px_scale = c->vo_scale_eff;
    });
}
int sng_render_nerf_ngp(sng_ctx* c, const sng_frame_params* p, sng_frame_result* out) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); render_nerf_ngp(c, p, out); });
}
// PNG (RGB8 / RGBA8, filter 0, zlib) -- the recording's stbi_write_png (display.cu:319)
void write_png(const std::string& path, const uint8_t* px, int w, int h, int ch) {
    if (w <= 0 || h <= 0 || (ch != 3 && ch != 4)) throw SngError(SNG_ERR_INVALID, "bad PNG image");
    std::vector<uint8_t> raw((size_t)h * ((size_t)w * ch + 1));
    for (int y = 0; y < h; ++y) {
        raw[(size_t)y * ((size_t)w * ch + 1)] = 0;
        std::memcpy(&raw[(size_t)y * ((size_t)w * ch + 1) + 1], px + (size_t)y * w * ch, (size_t)w * ch);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) throw SngError(SNG_ERR_IO, "zlib compress failed");
    z.resize(zlen);
    std::ofstream f(path, std::ios::binary);
    if (!f) throw SngError(SNG_ERR_IO, "cannot write " + path);
    auto be32 = [](uint32_t v) { return std::array<uint8_t, 4>{(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v}; };
    auto chunk = [&](const char* type, const std::vector<uint8_t>& data) {
        const auto len = be32((uint32_t)data.size());
        f.write(reinterpret_cast<const char*>(len.data()), 4);
        std::vector<uint8_t> td(type, type + 4);
        td.insert(td.end(), data.begin(), data.end());
        f.write(reinterpret_cast<const char*>(td.data()), (std::streamsize)td.size());
        const auto crc = be32((uint32_t)crc32(0L, td.data(), (uInt)td.size()));
        f.write(reinterpret_cast<const char*>(crc.data()), 4);
    };
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    f.write(reinterpret_cast<const char*>(sig), 8);
    std::vector<uint8_t> ihdr(13);
    const auto bw = be32((uint32_t)w), bh = be32((uint32_t)h);
    std::copy(bw.begin(), bw.end(), ihdr.begin());
    std::copy(bh.begin(), bh.end(), ihdr.begin() + 4);
    ihdr[8] = 8; ihdr[9] = ch == 4 ? 6 : 2; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    chunk("IHDR", ihdr);
    chunk("IDAT", z);
    chunk("IEND", {});
}

// Display::present (display.cu:265-303) of the last frame: FXAA + blend + RGB8 readback (display.hip)
void display_frame(sng_ctx* c, uint8_t* out, uint64_t cap) {
    const int W = c->mesh_res[0], H = c->mesh_res[1], OW = c->win[0], OH = c->win[1];
    if (W <= 0 || OW <= 0 || !c->final_rgba.p) throw SngError(SNG_ERR_STATE, "render a frame first");
    const size_t n = (size_t)OW * OH * 3;
    if (out && cap < n) throw SngError(SNG_ERR_INVALID, "display buffer too small");
    c->display_rgb.ensure(n);
    launch_display(c->final_rgba.as<float4>(), W, H, OW, OH, c->clear_color, c->display_rgb.as<uint8_t>(), c->s_nerf);
    HIPCHK(hipGetLastError());
    if (out) HIPCHK(hipMemcpyAsync(out, c->display_rgb.p, n, hipMemcpyDeviceToHost, c->s_nerf));
    HIPCHK(hipStreamSynchronize(c->s_nerf));
}

int sng_image_write_png(const char* path, const uint8_t* pixels, int32_t width, int32_t height, int32_t channels) {
    return guarded([&] {
        if (!path || !pixels) throw SngError(SNG_ERR_INVALID, "null argument");
        write_png(path, pixels, width, height, channels);
    });
}
int sng_display_frame(sng_ctx* c, uint8_t* rgb_out, uint64_t capacity) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); display_frame(c, rgb_out, capacity); });
}
int sng_save_image(sng_ctx* c, const char* folder, int32_t* written) {
    return guarded([&] {
        HIPCHK(hipSetDevice(c->device));
        if (written) *written = 0;
        if (c->img_count > c->img_count_max) return;   // Display::save_image (display.cu:305-306)
        const std::string dir = folder && *folder ? std::string(folder) : c->out_folder;
        if (dir.empty()) throw SngError(SNG_ERR_INVALID, "no output folder");
        std::vector<uint8_t> rgb((size_t)c->win[0] * c->win[1] * 3);
        display_frame(c, rgb.data(), rgb.size());
        char name[32];
        std::snprintf(name, sizeof(name), "/output-%03d.png", ++c->img_count);
        write_png(dir + name, rgb.data(), c->win[0], c->win[1], 3);
        if (written) *written = 1;
    });
}
int sng_animation_probe(const char* scene_json, uint32_t n_frames, int32_t playing, float animation_speed, float* cameras, float* light_pos,
                        uint32_t light_cap, float* object_pos, uint32_t object_cap, uint32_t* n_lights, uint32_t* n_objects) {
    return guarded([&] {
        if (!scene_json) throw SngError(SNG_ERR_INVALID, "null path");
        std::unique_ptr<sng_ctx> c(new sng_ctx());   // host state only: no device calls below
        c->params = default_params();
        load_scene(c.get(), scene_json);
        if (playing >= 0) c->campath.playing = playing != 0 && c->campath.keys.size() >= 2;
        if (animation_speed >= 0.0f) { c->anim_speed = animation_speed; c->animations = animation_speed > 0.0f; }
        const uint32_t nl = (uint32_t)c->lights.size(), no = (uint32_t)c->objs.size();
        if (n_lights) *n_lights = nl;
        if (n_objects) *n_objects = no;
        for (uint32_t f = 0; f < n_frames; ++f) {
            animate(c.get());
            if (cameras) std::memcpy(cameras + 12 * (size_t)f, c->cam, 12 * sizeof(float));
            if (light_pos && nl <= light_cap)
                for (uint32_t i = 0; i < nl; ++i) std::memcpy(light_pos + 3 * ((size_t)f * nl + i), c->lights[i].pos, 3 * sizeof(float));
            if (object_pos && no <= object_cap)
                for (uint32_t i = 0; i < no; ++i) {
                    float* q = object_pos + 3 * ((size_t)f * no + i);
                    q[0] = c->objs[i].pos.x; q[1] = c->objs[i].pos.y; q[2] = c->objs[i].pos.z;
                }
        }
        c->objs.clear();
    });
}
int sng_render_frame(sng_ctx* c, const sng_frame_params* p, sng_frame_result* out) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); render_frame(c, p, out); });
}
// 8-bit RGB / RGBA / grey(+alpha) non-interlaced PNG -> RGBA8 (the nerf_synthetic training images;
// the reference loads them through stb_image, nerf_loader.cu).  Host-only utility.
int sng_image_load_png(const char* path, uint8_t* out, uint64_t capacity, int32_t* width, int32_t* height) {
    return guarded([&] {
        std::ifstream f(path, std::ios::binary);
        if (!f) throw SngError(SNG_ERR_IO, std::string("cannot open ") + path);
        std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
        if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) throw SngError(SNG_ERR_IO, "not a PNG");
        auto be32 = [&](size_t o) { return (uint32_t)d[o] << 24 | (uint32_t)d[o + 1] << 16 | (uint32_t)d[o + 2] << 8 | d[o + 3]; };
        uint32_t w = 0, h = 0;
        int depth = 0, ctype = 0, interlace = 0;
        std::vector<uint8_t> idat;
        for (size_t o = 8; o + 8 <= d.size();) {
            const uint32_t len = be32(o);
            const std::string type(reinterpret_cast<const char*>(&d[o + 4]), 4);
            if (o + 12 + len > d.size()) throw SngError(SNG_ERR_IO, "truncated PNG");
            const uint8_t* p = &d[o + 8];
            if (type == "IHDR") {
                w = be32(o + 8); h = be32(o + 12); depth = p[8]; ctype = p[9]; interlace = p[12];
            } else if (type == "IDAT") {
                idat.insert(idat.end(), p, p + len);
            } else if (type == "IEND") {
                break;
            }
            o += 12 + len;
        }
        const int ch = ctype == 6 ? 4 : ctype == 2 ? 3 : ctype == 4 ? 2 : ctype == 0 ? 1 : 0;
        if (depth != 8 || ch == 0 || interlace != 0 || !w || !h) throw SngError(SNG_ERR_IO, "unsupported PNG (8-bit non-interlaced grey/RGB/RGBA only)");
        if (width) *width = (int32_t)w;
        if (height) *height = (int32_t)h;
        if (!out) return;
        if (capacity < (uint64_t)w * h * 4) throw SngError(SNG_ERR_INVALID, "output buffer too small");
        const size_t stride = (size_t)w * ch;
        std::vector<uint8_t> raw((stride + 1) * h);
        uLongf rl = (uLongf)raw.size();
        if (uncompress(raw.data(), &rl, idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size()) throw SngError(SNG_ERR_IO, "bad PNG data");
        std::vector<uint8_t> prev(stride, 0), cur(stride);
        for (uint32_t y = 0; y < h; ++y) {
            const uint8_t ft = raw[y * (stride + 1)];
            const uint8_t* src = &raw[y * (stride + 1) + 1];
            for (size_t i = 0; i < stride; ++i) {
                const int a = i >= (size_t)ch ? cur[i - ch] : 0, b = prev[i], cc = i >= (size_t)ch ? prev[i - ch] : 0;
                int v = src[i];
                if (ft == 1) v += a;
                else if (ft == 2) v += b;
                else if (ft == 3) v += (a + b) / 2;
                else if (ft == 4) {
                    const int pp = a + b - cc, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - cc);
                    v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc);
                }
                cur[i] = (uint8_t)v;
            }
            uint8_t* o = out + (size_t)y * w * 4;
            for (uint32_t x = 0; x < w; ++x) {
                const uint8_t* px = &cur[(size_t)x * ch];
                if (ch >= 3) { o[4 * x] = px[0]; o[4 * x + 1] = px[1]; o[4 * x + 2] = px[2]; o[4 * x + 3] = ch == 4 ? px[3] : 255; }
                else { o[4 * x] = o[4 * x + 1] = o[4 * x + 2] = px[0]; o[4 * x + 3] = ch == 2 ? px[1] : 255; }
            }
            std::swap(prev, cur);
        }
    });
}
int sng_train_set_dataset(sng_ctx* c, uint32_t n, uint32_t w, uint32_t h, const uint8_t* rgba, const float* xf, const float* focal, const float* pp) {
    return guarded([&] {
        if (!c || !rgba || !xf || !focal || !pp || !n || !w || !h) throw SngError(SNG_ERR_INVALID, "bad training dataset");
        HIPCHK(hipSetDevice(c->device));
        auto& t = c->tr;
        train_drop_pregen(t);   // a step generated ahead read the old images: wait for it, then regenerate
        upload(t.pixels, rgba, (size_t)n * w * h * 4);
        upload(t.xforms, xf, (size_t)n * 12 * 4);
        // generate_training_samples_nerf builds rays from get_xform_given_rolling_shutter (common_device.cuh:
        // 361-368): rotation through the glm quat round trip (start == end, no rolling shutter)
        std::vector<float> xr(xf, xf + (size_t)n * 12);
        for (uint32_t i = 0; i < n; ++i) {
            float* q = xr.data() + 12 * (size_t)i;
            const m3 r = rolling_shutter_rotation({mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8])});
            q[0] = r.c0.x; q[1] = r.c0.y; q[2] = r.c0.z; q[3] = r.c1.x; q[4] = r.c1.y; q[5] = r.c1.z; q[6] = r.c2.x; q[7] = r.c2.y; q[8] = r.c2.z;
        }
        upload(t.xforms_ray, xr.data(), (size_t)n * 12 * 4);
        upload(t.focal, focal, (size_t)n * 2 * 4);
        upload(t.pp, pp, (size_t)n * 2 * 4);
        t.w = (int)w; t.h = (int)h; t.n_images = (int)n;
        t.h_lens.clear();   // a new dataset is Perspective until sng_train_set_lens
    });
}
static_assert(sizeof(Lens) == sizeof(sng_lens), "Lens mirrors sng_lens");
int sng_train_set_lens(sng_ctx* c, const sng_lens* lenses, uint32_t n) {
    return guarded([&] {
        if (!c) throw SngError(SNG_ERR_INVALID, "null context");
        HIPCHK(hipSetDevice(c->device));
        auto& t = c->tr;
        train_drop_pregen(t);   // a step generated ahead used the old lenses
        if (!lenses || n == 0) { t.h_lens.clear(); return; }
        if ((int)n != t.n_images) throw SngError(SNG_ERR_INVALID, "one lens per training image (sng_train_set_dataset) expected");
        std::vector<Lens> h(n);
        for (uint32_t i = 0; i < n; ++i) {
            if (lenses[i].mode < 0 || lenses[i].mode > 5) throw SngError(SNG_ERR_INVALID, "unknown lens mode");
            h[i].mode = lenses[i].mode;
            for (int k = 0; k < 7; ++k) h[i].params[k] = lenses[i].params[k];
        }
        upload(t.lens, h.data(), (size_t)n * sizeof(Lens));
        t.h_lens = h;
    });
}
int sng_set_render_lens(sng_ctx* c, const sng_lens* lens) {
    return guarded([&] {
        if (!c) throw SngError(SNG_ERR_INVALID, "null context");
        Lens l{};
        if (lens) {
            if (lens->mode < 0 || lens->mode > 5) throw SngError(SNG_ERR_INVALID, "unknown lens mode");
            l.mode = lens->mode;
            for (int k = 0; k < 7; ++k) l.params[k] = lens->params[k];
        }
        c->render_lens = l;
    });
}
int sng_get_render_lens(sng_ctx* c, sng_lens* out) {
    return guarded([&] {
        if (!c || !out) throw SngError(SNG_ERR_INVALID, "null argument");
        out->mode = c->render_lens.mode;
        for (int k = 0; k < 7; ++k) out->params[k] = c->render_lens.params[k];
    });
}
int sng_train_reset(sng_ctx* c, uint64_t seed) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); train_reset(c, seed); });
}
int sng_train(sng_ctx* c, uint32_t n_steps, sng_train_stats* st) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); train_steps(c, n_steps, st); });
}
int sng_train_export(sng_ctx* c, uint16_t* params, uint64_t n_params, uint16_t* grid, uint64_t n_cells) {
    return guarded([&] {
        HIPCHK(hipSetDevice(c->device));
        if (!c->tr.ready) throw SngError(SNG_ERR_STATE, "no training state");
        if (params) {
            if (n_params != c->n_params) throw SngError(SNG_ERR_INVALID, "param count mismatch");
            HIPCHK(hipMemcpy(params, c->tr.p_infer.p, n_params * 2, hipMemcpyDeviceToHost));
        }
        if (grid) {
            const uint64_t nc = (uint64_t)GRID_CELLS * (c->max_cascade + 1);
            if (n_cells != nc) throw SngError(SNG_ERR_INVALID, "grid cell count mismatch");
            std::vector<float> f(nc);
            HIPCHK(hipMemcpy(f.data(), c->tr.grid.p, nc * 4, hipMemcpyDeviceToHost));
            for (uint64_t i = 0; i < nc; ++i) grid[i] = f2h(f[i]);
        }
    });
}
int sng_train_debug(sng_ctx* c, int stage, const char* name, void* out, uint64_t cap, uint64_t* size) {
    return guarded([&] {
        HIPCHK(hipSetDevice(c->device));
        if (!c->tr.ready) train_reset(c, 1337);
        auto& t = c->tr;
        if (t.n_images == 0) throw SngError(SNG_ERR_STATE, "no training images");
        if (stage > 0) {
            if (t.step == 0 && !c->has_bitfield) train_density_update(c, c->s_nerf);
            train_forward_backward(c, stage, c->s_nerf, nullptr, t.pregen);   // pregen: samples already generated on s_gen
            t.pregen = false;
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(c->s_nerf));
        if (!name) return;
        const std::string k = name;
        const std::map<std::string, DevBuf*> bufs = {{"ctrl", &t.ctrl}, {"ray_indices", &t.ray_indices}, {"rays", &t.rays}, {"numsteps", &t.numsteps},
                                                     {"coords", &t.coords}, {"mlp_out", &t.mlp_out}, {"coords_c", &t.coords_c}, {"dloss", &t.dloss},
                                                     {"loss", &t.loss}, {"grads", &t.grads}, {"acts", &t.acts}, {"grid", &t.grid}, {"master", &t.master},
                                                     {"m1", &t.m1}, {"m2", &t.m2}, {"steps", &t.steps}, {"ema", &t.ema}, {"p_infer", &t.p_infer}};
        auto it = bufs.find(k);
        if (it == bufs.end()) throw SngError(SNG_ERR_INVALID, "unknown training buffer " + k);
        const uint64_t n = it->second->bytes;
        if (size) *size = n;
        if (out && k == "grads" && t.grads_h_used) {   // f32 view: the fp16 grid gradients as the optimizer reads them
            const uint64_t n_mlp = 3072 + 7168, n_grid = c->n_params - n_mlp;
            std::vector<float> f(n / 4, 0.0f);
            std::vector<uint16_t> hg(n_grid);
            HIPCHK(hipMemcpy(f.data(), t.grads.p, n_mlp * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(hg.data(), t.grads_h.p, n_grid * 2, hipMemcpyDeviceToHost));
            for (uint64_t i = 0; i < n_grid && n_mlp + i < f.size(); ++i) f[n_mlp + i] = h2f(hg[i]);
            std::memcpy(out, f.data(), std::min(n, cap));
        } else if (out) {
            HIPCHK(hipMemcpy(out, it->second->p, std::min(n, cap), hipMemcpyDeviceToHost));
        }
    });
}
int sng_comm_unique_id(uint8_t* out) {
    return guarded([&] {
        if (!out) throw SngError(SNG_ERR_INVALID, "null id buffer");
        comm_unique_id(out);
    });
}
int sng_set_comm(sng_ctx* c, const uint8_t* id, int rank, int world) {
    return guarded([&] {
        if (!c) throw SngError(SNG_ERR_INVALID, "null context");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipStreamSynchronize(c->s_nerf));
        c->sched_hint_key = 0;   // hints of another schedule (trace_nerf)
        if (!id) { comm_destroy(c->sched_comm); return; }
        if (world < 1 || rank < 0 || rank >= world) throw SngError(SNG_ERR_INVALID, "bad rank/world");
        if (c->sched_comm.host_fn || c->sched_comm.replay) throw SngError(SNG_ERR_STATE, "a host schedule reducer or replay is attached");
        comm_init(c->sched_comm, id, rank, world);
    });
}
int sng_set_sched_reducer(sng_ctx* c, sng_sched_reduce_fn fn, void* user) {
    return guarded([&] {
        if (!c) throw SngError(SNG_ERR_INVALID, "null context");
        if (fn && (c->sched_comm.comm || c->sched_comm.replay)) throw SngError(SNG_ERR_STATE, "an RCCL communicator or replay is attached");
        c->sched_hint_key = 0;
        c->sched_comm.host_fn = fn;
        c->sched_comm.host_user = fn ? user : nullptr;
    });
}
int sng_set_sched_replay(sng_ctx* c, const uint32_t* records, uint64_t n_words) {
    return guarded([&] {
        if (!c) throw SngError(SNG_ERR_INVALID, "null context");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipStreamSynchronize(c->s_nerf));   // no copy from the old records is still queued
        SchedComm& sc = c->sched_comm;
        // attaching or detaching drops the step hints (another schedule wrote them); replacing the records of an
        // attached replay keeps them, as a rank keeps its frame-wide hints from one frame to the next
        if (!records || !sc.replay) c->sched_hint_key = 0;
        if (sc.replay) { (void)hipHostFree(sc.replay); sc.replay = nullptr; sc.replay_words = 0; }
        if (!records) return;
        // an empty replay would make every later frame fail with "diverged": detach with records = NULL instead
        if (n_words == 0) throw SngError(SNG_ERR_INVALID, "empty replay records (detach with records = NULL)");
        if (sc.comm || sc.host_fn) throw SngError(SNG_ERR_STATE, "an RCCL communicator or host reducer is attached");
        for (uint64_t at = 0; at < n_words; at += 1 + (uint64_t)records[at])
            if (records[at] == 0 || at + 1 + records[at] > n_words) throw SngError(SNG_ERR_INVALID, "malformed replay records");
        HIPCHK(hipHostMalloc((void**)&sc.replay, std::max<uint64_t>(1, n_words) * 4, hipHostMallocDefault));
        if (n_words) std::memcpy(sc.replay, records, n_words * 4);
        sc.replay_words = (size_t)n_words;
        sc.replay_cursor = 0;
    });
}
int sng_synchronize(sng_ctx* c) { return guarded([&] { HIPCHK(hipStreamSynchronize(c->s_nerf)); HIPCHK(hipStreamSynchronize(c->s_rt)); }); }
int sng_copy_to_host(sng_ctx* c, const void* src, void* dst, uint64_t n) {
    return guarded([&] { HIPCHK(hipSetDevice(c->device)); HIPCHK(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost)); });
}
int sng_copy_device(sng_ctx* c, const void* src, void* dst, uint64_t n, void* stream) {
    return guarded([&] {
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    });
}
int sng_gather_rgba8(sng_ctx* c, const int32_t* bounds, uint32_t* d_frame, void* stream) {
    return guarded([&] {
        if (!c || !bounds) throw SngError(SNG_ERR_INVALID, "null context or bounds");
        HIPCHK(hipSetDevice(c->device));
        if (!c->sched_comm.comm) throw SngError(SNG_ERR_STATE, "no communicator attached (sng_set_comm)");
        const int world = c->sched_comm.world, rank = c->sched_comm.rank;
        const int W = c->mesh_res[0], H = c->mesh_res[1];
        std::vector<size_t> off(world), size(world);
        for (int k = 0; k < world; ++k) {
            if (bounds[k] < 0 || bounds[k + 1] > H || bounds[k] > bounds[k + 1] || (k == 0 && bounds[0] != 0) || (k == world - 1 && bounds[world] != H))
                throw SngError(SNG_ERR_INVALID, "bounds must tile [0, height)");
            off[k] = (size_t)bounds[k] * W * 4;
            size[k] = (size_t)(bounds[k + 1] - bounds[k]) * W * 4;
        }
        if (rank == 0 && !d_frame) throw SngError(SNG_ERR_INVALID, "rank 0 needs the frame buffer");
        hipStream_t s = stream ? (hipStream_t)stream : c->s_nerf;
        c->band_rgba8.ensure(std::max<size_t>(4, size[rank]));
        if (size[rank]) launch_rgba8_band(c->final_rgba.as<float4>() + (size_t)bounds[rank] * W, (uint32_t)(size[rank] / 4), c->band_rgba8.as<uint32_t>(), s);
        HIPCHK(hipGetLastError());
        comm_gather_to_root(c->sched_comm, c->band_rgba8.p, d_frame, off.data(), size.data(), s);
    });
}
int sng_comm_allreduce_u32(sng_ctx* c, uint32_t* d, uint64_t n, void* stream) {
    return guarded([&] {
        if (!c || !d) throw SngError(SNG_ERR_INVALID, "null context or buffer");
        HIPCHK(hipSetDevice(c->device));
        if (!c->sched_comm.comm) throw SngError(SNG_ERR_STATE, "no communicator attached (sng_set_comm)");
        comm_allreduce_u32(c->sched_comm, d, d, (size_t)n, stream ? (hipStream_t)stream : c->s_nerf);
    });
}
int sng_final_rgba8(sng_ctx* c, int32_t row_begin, int32_t row_end, uint32_t* d_out, void* stream) {
    return guarded([&] {
        HIPCHK(hipSetDevice(c->device));
        const int W = c->mesh_res[0], H = c->mesh_res[1];
        if (!d_out || row_begin < 0 || row_end > H || row_begin > row_end) throw SngError(SNG_ERR_INVALID, "bad row band");
        launch_rgba8_band(c->final_rgba.as<float4>() + (size_t)row_begin * W, (uint32_t)((row_end - row_begin) * W), d_out, (hipStream_t)stream);
        HIPCHK(hipGetLastError());
    });
}
int sng_get_rng_states(sng_ctx* c, int which, uint32_t* out, uint64_t n) {
    return guarded([&] {
        DevBuf& b = which == 0 ? c->rng_nerf : c->rng_mesh;
        uint32_t cnt = which == 0 ? c->n_rng_nerf : c->n_rng_mesh;
        if (n != cnt) throw SngError(SNG_ERR_INVALID, "state count is " + std::to_string(cnt));
        std::vector<uint32_t> soa((size_t)n * 6);
        HIPCHK(hipMemcpy(soa.data(), b.p, soa.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < 6; ++k) out[6 * i + k] = soa[(size_t)k * n + i];
    });
}
int sng_set_rng_states(sng_ctx* c, int which, const uint32_t* in, uint64_t n) {
    return guarded([&] {
        DevBuf& b = which == 0 ? c->rng_nerf : c->rng_mesh;
        uint32_t cnt = which == 0 ? c->n_rng_nerf : c->n_rng_mesh;
        if (n != cnt) throw SngError(SNG_ERR_INVALID, "state count is " + std::to_string(cnt));
        std::vector<uint32_t> soa((size_t)n * 6);
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < 6; ++k) soa[(size_t)k * n + i] = in[6 * i + k];
        HIPCHK(hipMemcpy(b.p, soa.data(), soa.size() * 4, hipMemcpyHostToDevice));
    });
}
int sng_bvh_build(float* tris, uint32_t n, uint32_t ppl, float* nodes_out, uint32_t cap, uint32_t* n_nodes) {
    return guarded([&] {
        if (n == 0) throw SngError(SNG_ERR_INVALID, "no triangles");
        std::vector<Tri> t((Tri*)tris, (Tri*)tris + n);
        auto nodes = build_bvh(t, ppl);
        if (nodes.size() > cap) throw SngError(SNG_ERR_INVALID, "node capacity too small: need " + std::to_string(nodes.size()));
        std::memcpy(nodes_out, nodes.data(), nodes.size() * sizeof(BvhNode));
        std::memcpy(tris, t.data(), n * sizeof(Tri));
        *n_nodes = (uint32_t)nodes.size();
    });
}

}  // extern "C"
