// host_render.cpp -- the render path on the host: model and occupancy upload (Testbed), resize (Engine::resize),
// the device-driven NeRF trace (NerfTracer::trace_alt, testbed_nerf.cu:2128-2277), the hybrid frame (Engine::frame,
// engine.cu:352-433) and the instant-NGP render path (Testbed::render_nerf).
#include "host.h"

namespace sng_host {

void compute_levels(sng_ctx* c) {
    const auto& g = c->cfg;
    c->levels.clear();
    float log2_pls = std::log2(g.per_level_scale);
    uint32_t offset = 0;
    for (uint32_t i = 0; i < g.n_levels; ++i) {
        float scale = std::fma(std::exp2((float)i * log2_pls), (float)g.base_resolution, -1.0f);   // grid_scale [tcnn]
        uint32_t res = (uint32_t)std::ceil(scale) + 1;                                             // grid_resolution [tcnn]
        uint32_t max_params = 0xffffffffu / 2;
        uint32_t pil = std::pow((float)res, 3.0f) > (float)max_params ? max_params : res * res * res;
        pil = (pil + 7u) / 8u * 8u;
        pil = std::min(pil, 1u << g.log2_hashmap_size);
        // tcnn grid_index stride loop: dense index kept iff the loop ran all dims and stride <= size
        uint64_t stride = 1;
        uint32_t dims = 0;
        for (; dims < 3 && stride <= pil; ++dims) stride *= res;
        LevelInfo L{};
        L.offset = offset;
        L.size = pil;
        L.pow2_mask = (pil & (pil - 1)) == 0 ? pil - 1 : 0;
        L.dense = (dims == 3 && !(pil < stride)) ? 1u : 0u;
        L.res = res;
        L.res2 = res * res;
        L.scale = scale;
        c->levels.push_back(L);
        offset += pil;
    }
    c->n_params = 3072 + 7168 + (uint64_t)offset * g.n_features_per_level;
}

// A-fragment image of one layer: frag(lane, j) = W[16mb + (lane&15)][k(kb, lane>>4, j)]
void pack_layer(const uint16_t* W, int n_in, int mb, int kb, bool permuted, uint16_t* dst) {
    for (int lane = 0; lane < 64; ++lane) {
        int row = 16 * mb + (lane & 15), g = lane >> 4;
        for (int j = 0; j < 8; ++j) {
            int k = permuted ? 32 * kb + 16 * (j >= 4) + 4 * g + (j & 3) : 32 * kb + 8 * g + j;
            dst[lane * 8 + j] = W[row * n_in + k];
        }
    }
}

void set_model(sng_ctx* c, const sng_nerf_config* cfg, const uint16_t* params, uint64_t n) {
    if (!cfg) throw SngError(SNG_ERR_INVALID, "null config");
    if (cfg->n_levels * cfg->n_features_per_level != 32 || (cfg->n_features_per_level != 4 && cfg->n_features_per_level != 2))
        throw SngError(SNG_ERR_INVALID, "fused network supports L*F == 32 with F in {2,4} (base.json shape)");
    if (cfg->aabb_scale == 0 || (cfg->aabb_scale & (cfg->aabb_scale - 1)) || cfg->aabb_scale > 128)
        throw SngError(SNG_ERR_INVALID, "aabb_scale must be a power of two <= 128 (testbed_nerf.cu:3055-3067)");
    c->cfg = *cfg;
    compute_levels(c);
    if (n != c->n_params) throw SngError(SNG_ERR_INVALID, "param count mismatch: got " + std::to_string(n) + ", expected " + std::to_string(c->n_params));
    // weight fragments (network.hip header)
    std::vector<uint16_t> frag(20 * 64 * 8);
    const uint16_t* dW0 = params;
    const uint16_t* dW1 = dW0 + 64 * 32;
    const uint16_t* rW0 = params + 3072;
    const uint16_t* rW1 = rW0 + 64 * 32;
    const uint16_t* rW2 = rW1 + 64 * 64;
    int f = 0;
    for (int mb = 0; mb < 4; ++mb) pack_layer(dW0, 32, mb, 0, false, &frag[(f++) * 512]);
    for (int kb = 0; kb < 2; ++kb) pack_layer(dW1, 64, 0, kb, true, &frag[(f++) * 512]);
    for (int mb = 0; mb < 4; ++mb) pack_layer(rW0, 32, mb, 0, true, &frag[(f++) * 512]);
    for (int mb = 0; mb < 4; ++mb)
        for (int kb = 0; kb < 2; ++kb) pack_layer(rW1, 64, mb, kb, true, &frag[(f++) * 512]);
    for (int kb = 0; kb < 2; ++kb) pack_layer(rW2, 64, 0, kb, true, &frag[(f++) * 512]);
    upload(c->d_wfrag, frag.data(), frag.size() * 2);
    upload(c->d_grid, params + 3072 + 7168, (n - 3072 - 7168) * 2);
    upload(c->d_params, params, n * 2);
    c->tr.ready = false;
    upload(c->d_levels, c->levels.data(), c->levels.size() * sizeof(LevelInfo));
    c->net.F = (int)cfg->n_features_per_level;
    c->net.L = (int)cfg->n_levels;
    c->net.n_cus = c->n_cus;
    c->net.wfrag = c->d_wfrag.p;
    c->net.grid = c->d_grid.p;
    c->net.levels = c->d_levels.as<LevelInfo>();
    // load_nerf_post (testbed_nerf.cu:3069-3085)
    float half = 0.5f * (float)std::min(128u, cfg->aabb_scale);
    c->box = {mk(0.5f - half, 0.5f - half, 0.5f - half), mk(0.5f + half, 0.5f + half, 0.5f + half)};
    c->max_cascade = 0;
    while ((1u << c->max_cascade) < cfg->aabb_scale) ++c->max_cascade;
    c->cone = cfg->aabb_scale <= 1 ? 0.0f : 1.0f / 256.0f;
    c->has_model = true;
    c->has_bitfield = false;
    ++c->model_epoch;
}

void set_density_grid(sng_ctx* c, const uint16_t* grid, uint64_t n_cells) {
    if (!c->has_model) throw SngError(SNG_ERR_STATE, "set the model before the density grid");
    if (n_cells != (uint64_t)GRID_CELLS * (c->max_cascade + 1))
        throw SngError(SNG_ERR_INVALID, "Incompatible number of grid cascades.");   // testbed.cu:4932
    upload(c->d_grid_f16, grid, n_cells * 2);
    c->d_grid_f32.ensure(n_cells * 4);
    c->d_partial.ensure(1024 * sizeof(double));
    c->d_mean.ensure(sizeof(float));
    c->d_bitfield.ensure((size_t)GRID_CELLS / 8 * N_CASCADES);
    c->d_occ_linear.ensure((size_t)GRID_CELLS / 8 * N_CASCADES);   // every cascade (Volume::occ_lin_all)
    launch_bitfield(c->d_grid_f16.as<uint16_t>(), c->max_cascade, c->d_grid_f32.as<float>(), c->d_partial.as<double>(), c->d_mean.as<float>(),
                    c->d_bitfield.as<uint8_t>(), c->d_occ_linear.as<uint32_t>(), c->s_nerf);
    build_occ_brick(c, c->s_nerf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->s_nerf));
    c->has_bitfield = true;
}

// OccBrick blob of the current linear occupancy (render_frame reads the brick count back lazily)
void build_occ_brick(sng_ctx* c, hipStream_t s) {
    c->d_occ_brick.ensure((size_t)OCC_BRICK_CAP_WORDS * 4);
    c->d_occ_brick_aux.ensure((4096 + 4) * 4);
    launch_occ_brick(c->d_occ_linear.as<uint32_t>(), c->d_occ_brick_aux.as<uint32_t>(), c->d_occ_brick.as<uint32_t>(),
                     c->d_occ_brick_aux.as<uint32_t>() + 4096, s);
    // the brick count travels to pinned memory behind the rebuild; render_frame waits for this event only
    HIPCHK(hipMemcpyAsync(&c->h_alive[7], c->d_occ_brick_aux.as<uint32_t>() + 4096, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(c->ev_brick, s));
    c->occ_brick_dirty = true;
    ++c->model_epoch;
}

// the brick count of the last occupancy rebuild (build_occ_brick), read back behind it: the marchers stage the bricks in
// LDS only when the count is known
void resolve_occ_brick(sng_ctx* c) {
    if (c->occ_brick_dirty && c->d_occ_brick_aux.p) {
        HIPCHK(hipEventSynchronize(c->ev_brick));
        c->occ_brick_n = c->h_alive[7];
        c->occ_brick_dirty = false;
    }
}

Volume make_volume(const sng_ctx* c) {
    Volume v{};
    v.render_aabb = c->box;
    v.train_aabb = c->box;
    v.to_local = {mk(1, 0, 0), mk(0, 1, 0), mk(0, 0, 1)};
    v.to_local_identity = 1;
    v.cone = c->cone;
    v.ss = step_space(c->cone);
    v.max_mip = c->max_cascade;
    v.min_transmittance = (float)c->p("min_transmittance");
    v.bitfield = c->d_bitfield.as<uint8_t>();
    v.occ_linear = c->d_occ_linear.as<uint32_t>();
    if (c->p("occ_lin_all") != 0.0) v.occ_lin_all = v.occ_linear;   // the cascaded marchers' lookups without Morton encoding
    v.linear = (c->max_cascade == 0 && c->cone <= 1e-5f && c->p("linear_marcher") != 0.0) ? 1 : 0;
    // the bricks in LDS when they fit the budget (lego: 521 bricks, 41 KiB)
    const uint32_t words = (OCC_BRICK_HDR_WORDS + 16u * std::max(1u, c->occ_brick_n) + 3u) & ~3u;   // >= 1 brick: branch-free readers
    if (v.linear && c->d_occ_brick.p) v.occ_brick_g = c->d_occ_brick.as<uint32_t>();   // rebuilt in stream order with the bitfield
    if (v.linear && c->d_occ_brick.p && !c->occ_brick_dirty && c->p("occ_lds_kb") * 1024.0 >= 4.0 * words) {
        v.occ_brick = c->d_occ_brick.as<uint32_t>();
        v.occ_brick_words = words;
    }
    return v;
}

// ---- resize: Engine::resize (engine.cu:236-255) --------------------------------------
void resize(sng_ctx* c) {
    int res_factor = (int)c->p("res_factor");
    float factor = std::min(1.0f, 8.0f / (float)res_factor);
    auto clampi = [](int v, int lo, int hi) { return std::max(lo, std::min(hi, v)); };
    int nw = clampi((int)((float)c->win[0] * factor), c->win[0] / 16, c->win[0]);
    int nh = clampi((int)((float)c->win[1] * factor), c->win[1] / 16, c->win[1]);
    float vs = (float)(int)c->p("vo_scale");
    int rw = std::min(clampi((int)((float)nw * vs), nw / 16, nw * 16), c->win[0]);
    int rh = std::min(clampi((int)((float)nh * vs), nh / 16, nh * 16), c->win[1]);
    c->nerf_res[0] = nw; c->nerf_res[1] = nh;
    c->mesh_res[0] = rw; c->mesh_res[1] = rh;
    c->vo_scale_eff = std::max(1, rw / nw);
    c->params["vo_scale"] = c->vo_scale_eff;   // m_relative_vo_scale = rt_res.r / new_res.r
    c->last_res_factor = res_factor;
    size_t nn = (size_t)nw * nh, nm = (size_t)rw * rh;
    c->nerf_rgba.ensure(nn * 16);
    c->nerf_depth.ensure(nn * 4);
    c->nerf_pos.ensure(nn * 12);
    c->nerf_nrm.ensure(nn * 12);
    HIPCHK(hipMemset(c->nerf_rgba.p, 0, nn * 16));
    for (int b = 0; b < 2; ++b) {
        c->ray_ot[b].ensure(nn * 16);
        c->ray_di[b].ensure(nn * 16);
        c->ray_rgba[b].ensure(nn * 16);
        c->ray_depth[b].ensure(nn * 4);
        c->ray_mw[b].ensure(nn * 4);
        c->ray_lt[b].ensure(nn * 8);
        c->ray_lo[b].ensure(nn * 8);
        c->ray_kk[b].ensure(nn * 4);
    }
    c->samp.ensure(nn * 8);
    c->ray_cap = nn;
    c->ctrl.ensure(sizeof(MarchCtrl));
    c->mesh_o.ensure(nm * 16);
    c->mesh_d.ensure(nm * 16);
    c->acc_rgba.ensure(nm * 16);
    c->acc_depth.ensure(nm * 4);
    c->final_rgba.ensure(nm * 16);
    c->final_depth.ensure(nm * 4);
    // init_rand_state for NeRF px (engine.cu:246-247) and raytracer px (raytracer.cu:279)
    const auto& tab = xorwow_seq_tables();
    upload(c->d_seq, tab.data(), tab.size() * 4);
    c->rng_nerf.ensure(nn * 24);
    c->rng_mesh.ensure(nm * 24);
    c->n_rng_nerf = (uint32_t)nn;
    c->n_rng_mesh = (uint32_t)nm;
    launch_xorwow_init((uint32_t)nn, PT_SEED, c->d_seq.as<uint32_t>(), c->rng_nerf.as<uint32_t>(), c->s_nerf);
    launch_xorwow_init((uint32_t)nm, PT_SEED, c->d_seq.as<uint32_t>(), c->rng_mesh.as<uint32_t>(), c->s_nerf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->s_nerf));
    c->mesh_reset = true;
}

void ensure_samples(sng_ctx* c, uint32_t target) {
    // the speculative rounds' sample budget shares these buffers (nerf_spec_budget): a round marches at most kmax
    // iterations of 8 samples per ray, so a small frame (or a training-only context, ray_cap 0) needs no more
    const size_t kmax = (size_t)std::min<double>(SPEC_KMAX, std::max(1.0, c->p("nerf_spec_kmax")));
    const size_t spec = c->p("nerf_spec_rounds") > 0 ? std::min((size_t)std::max(1.0, c->p("nerf_spec_budget")),
                                                                MAX_STEPS_BETWEEN_COMPACTION * kmax * c->ray_cap) : 0;
    // the multi-step rounds' budget (nerf_msr_budget): at most kmax iterations of < 8 samples per ray
    const size_t mkmax = (size_t)std::min<double>(MSR_KMAX, std::max(1.0, c->p("nerf_msr_kmax")));
    const size_t msr = c->p("nerf_msr") != 0.0 ? std::min((size_t)std::max(1.0, c->p("nerf_msr_budget")),
                                                          (MAX_STEPS_BETWEEN_COMPACTION - 1) * mkmax * c->ray_cap) : 0;
    size_t cap = std::max(std::max(std::max<size_t>(target, c->ray_cap), spec), msr) + 64;
    if (cap > c->sample_cap) {
        c->coords.ensure(cap * 7 * 4);
        c->net_out.ensure(cap * 8);
        c->sample_cap = cap;
    }
}

CamDev cam_dev(const sng_ctx* c) { return {cam_col(c, 0), cam_col(c, 1), cam_col(c, 2), cam_col(c, 3)}; }
f2 focal_for(const sng_ctx* c, const int res[2]) {
    float r = (float)res[c->fov_axis];
    return {c->rel_focal[0] * r * c->zoom, c->rel_focal[1] * r * c->zoom};
}
f2 render_screen_center(const sng_ctx* c) {
    return {(0.5f - c->screen_center[0]) * c->zoom + 0.5f, (0.5f - c->screen_center[1]) * c->zoom + 0.5f};
}

// slots the reference would evaluate: sum over iterations of n_alive * n_steps padded to 256
// (testbed_nerf.cu:2210); the fused kernel only records the per-iteration alive counts
uint64_t ref_slots_of(const sng_ctx* c) {
    // generate_kernel / msr_schedule / the one-step schedule add the wavefront's iterations, tail_slots_kernel the tail's
    return c->h_ctrl->ref_slots;
}

// NerfTracer::init_rays_from_camera + trace_alt / trace (testbed_nerf.cu:2037-2401) for NeRF rows
// [tr0, tr1): device-driven wavefront, host readback of the alive count once per CHUNK iterations.
// on_chunk(k) runs after the k-th chunk is enqueued (render_frame starts the raytracer there).
// Returns the number of network launches.
// own0/own1: the NeRF rows this band owns (the bands of all ranks partition the frame's rows);
// only used when a schedule communicator is attached (Sched).
uint8_t* spec_hint_buf(sng_ctx* c);
bool spec_adapt_on(const sng_ctx* c, const TraceMode& mode);

// The view a frame's NeRF rays come from: camera0 / camera1 / rolling shutter, focal length, screen centre, NeRF
// resolution and the model (FNV-1a over the bytes).  The speculative rounds read the per-pixel look-ahead hints only
// when the hints were written for the same view: on a moving camera a pixel's last ray ended elsewhere, and the
// opacity policy (spec_k_of) sizes the look-ahead better (round 3: 1 deg/frame orbit 571 frames/s with hints read,
// 623 without).  They are written only by a frame that repeats the previous frame's view, so a moving camera
// makes none of their scattered byte stores.  The pixel jitter (spp) is not part of it: sub-pixel moves keep the hints close.
// the lens the NeRF rays of a frame go through: render_lens when render_with_lens_distortion is set, else Perspective
// (Testbed::render_nerf_with_buffers, testbed_nerf.cu:2504)
Lens frame_lens(const sng_ctx* c) {
    Lens l{};
    if (c->p("render_with_lens_distortion") != 0.0) l = c->render_lens;
    return l;
}
uint64_t spec_view_key(const sng_ctx* c, f2 focal, f2 sc) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    };
    mix(c->cam, sizeof(c->cam));
    mix(&c->has_cam1, sizeof(c->has_cam1));
    if (c->has_cam1) mix(c->cam1, sizeof(c->cam1));
    mix(c->rolling_shutter, sizeof(c->rolling_shutter));
    const Lens lens = frame_lens(c);
    mix(&lens, sizeof(lens));
    mix(&focal, sizeof(focal));
    mix(&sc, sizeof(sc));
    mix(c->nerf_res, sizeof(c->nerf_res));
    mix(&c->model_epoch, sizeof(c->model_epoch));
    return h | 1ull;   // never 0 (no hints)
}

// One reduction of the frame-wide schedule (sum over ranks of dev[0..n), in place on the NeRF stream):
// RCCL all-reduce, the host reducer (a stream sync + callback), or the next replay record (an async copy from
// pinned memory: a band timed on one GPU as its rank runs it, without a communicator).
// src: the values to sum when they are not already in dev (out of place: no copy into dev first).
void sched_reduce(sng_ctx* c, uint32_t* dev, uint32_t n, const uint32_t* src = nullptr) {
    SchedComm& sc = c->sched_comm;
    ++sc.replay_calls;
    if (sc.comm) {
        comm_allreduce_u32(sc, src ? src : dev, dev, n, c->s_nerf);
    } else if (sc.replay) {
        const size_t at = sc.replay_cursor;
        if (at >= sc.replay_words || sc.replay[at] != n || at + 1 + n > sc.replay_words)
            throw SngError(SNG_ERR_STATE, "schedule replay diverged at reduction " + std::to_string(sc.replay_calls) + " (" + std::to_string(n) + " values)");
        HIPCHK(hipMemcpyAsync(dev, sc.replay + at + 1, (size_t)n * 4, hipMemcpyHostToDevice, c->s_nerf));
        sc.replay_cursor = at + 1 + n;
    } else {
        std::vector<uint32_t> h(n);
        HIPCHK(hipMemcpyAsync(h.data(), src ? src : dev, (size_t)n * 4, hipMemcpyDeviceToHost, c->s_nerf));
        HIPCHK(hipStreamSynchronize(c->s_nerf));
        if (sc.host_fn(h.data(), n, sc.host_user) != 0) throw SngError(SNG_ERR_STATE, "schedule reducer failed");
        HIPCHK(hipMemcpyAsync(dev, h.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->s_nerf));
        HIPCHK(hipStreamSynchronize(c->s_nerf));   // h is a stack buffer
    }
}

uint32_t trace_nerf(sng_ctx* c, const sng_frame_params& P, const Volume& vol, const CamDev& cam, f2 sc, int tr0, int tr1, int own0, int own1,
                    TraceMode mode, uint32_t target, const std::function<void(int)>& on_chunk) {
    const int NW = c->nerf_res[0], NH = c->nerf_res[1];
    uint32_t net_launches = 0;
    MarchCtrl* ctrl = c->ctrl.as<MarchCtrl>();
    if (c->p("march_log") != 0.0) c->march_log.ensure(MARCH_LOG_CAP * 12);
    c->tail_live.ensure(TAIL_LIVE_CAP * 4);
    const bool gsched = c->sched_comm.active();
    // The msr rounds size K from the last frame's per-iteration steps (msr_shape).  Under the frame-wide schedule
    // every rank must see the same hints, so hints written under another schedule (a band's local one, another
    // target, before a communicator / reducer / replay was attached or detached) are dropped.
    const uint64_t hint_key = 1ull | (gsched ? 2ull : 0ull) | ((uint64_t)target << 2);
    if (!c->sched_hint.p || c->sched_hint_key != hint_key) {
        c->sched_hint.ensure(TAIL_LIVE_CAP);
        HIPCHK(hipMemsetAsync(c->sched_hint.p, 0, TAIL_LIVE_CAP, c->s_nerf));
        c->sched_hint_key = hint_key;
    }
    c->sched_comm.replay_cursor = 0;
    c->sched_comm.replay_calls = 0;
    launch_ctrl_init(ctrl, c->tail_live.as<int32_t>(), c->sched_hint.as<uint8_t>(), c->s_nerf, c->p("march_log") != 0.0 ? c->march_log.as<uint32_t>() : nullptr);
    NerfFrameArgs a{};
    a.vol = vol;
    a.cam = cam;
    // get_xform_given_rolling_shutter({camera0, camera1}, rolling_shutter, uv, motionblur_time) per pixel
    // (testbed_nerf.cu:1895): the quats of both cameras here, slerp / lerp in init_rays_kernel
    a.q0 = quat_from_m3({cam.c0, cam.c1, cam.c2});
    if (c->has_cam1) {
        const float* m = c->cam1;
        a.q1 = quat_from_m3({mk(m[0], m[1], m[2]), mk(m[3], m[4], m[5]), mk(m[6], m[7], m[8])});
        a.pos1 = mk(m[9], m[10], m[11]);
    } else {
        a.q1 = a.q0;
        a.pos1 = cam.c3;
    }
    for (int k = 0; k < 4; ++k) a.rolling_shutter[k] = c->rolling_shutter[k];
    a.lens = frame_lens(c);
    const int nres[2] = {NW, NH};
    a.focal = focal_for(c, nres);
    a.screen_center = sc;
    a.W = NW; a.H = NH; a.row0 = tr0; a.row1 = tr1;
    a.spp = P.spp;
    a.snap = 0;
    a.reset = P.reset_accumulation ? 1 : 0;
    a.target_n_queries = target;
    a.mode = mode;
    a.sched = {gsched ? 1 : 0, (uint32_t)own0 * (uint32_t)NW, (uint32_t)own1 * (uint32_t)NW};
    // sched_alive[q] <- sum over ranks of n_owned[q] (the frame-wide alive count of the next iteration)
    auto reduce_sched = [&](int q) {
        if (!gsched) return;
        sched_reduce(c, &ctrl->sched_alive[q], 1, &ctrl->n_owned[q]);
    };
    uint32_t* const sched_src = gsched ? &ctrl->sched_alive[0] : &ctrl->n_alive[0];   // counts the host loop reads
    // where network launch k records the sample count it read (timed frames; the per-launch roofline)
    auto net_rec = [&](uint32_t k) -> uint32_t* { return P.collect_kernel_times && k < 16 ? &ctrl->net_launch_samples[k] : nullptr; };
    RayBuf rb[2];
    for (int b = 0; b < 2; ++b)
        rb[b] = {c->ray_ot[b].as<float4>(), c->ray_di[b].as<float4>(), c->ray_rgba[b].as<float4>(), c->ray_depth[b].as<float>(), c->ray_mw[b].as<float>(),
                 c->ray_lt[b].as<float2>(), c->ray_lo[b].as<uint2>(), c->ray_kk[b].as<uint32_t>()};
    if (c->rt_wait_seq) {   // rt_first (render_frame)
        launch_rt_wait_started(c->rt_started.as<uint32_t>(), c->rt_wait_seq, (uint32_t)std::max(1.0, c->p("rt_first_timeout_us")), c->s_nerf);
        c->rt_wait_seq = 0;
    }
    launch_init_rays(a, rb[0], ctrl, c->nerf_rgba.as<float4>(), c->nerf_depth.as<float>(), c->nerf_pos.as<float>(), c->nerf_nrm.as<float>(),
                     (uint32_t)c->n_cus, c->s_nerf);
    reduce_sched(0);
    const uint32_t n_band = (uint32_t)(tr1 - tr0) * (uint32_t)NW;
    c->fused_last = false;
    c->fused_k0 = 0;
    c->msr_rounds = 0;
    // Hybrid schedule (fused.hip): the first `nerf_fused_after` iterations run as whole-GPU
    // wavefront launches (nearly every ray alive: throughput bound), the rest -- the latency-bound
    // tail -- in the ray-local fused kernel.  Valid when every iteration takes 8 steps, i.e. the
    // initial alive count satisfies n_alive * 8 <= target (it only shrinks).
    bool fuse = false;
    uint32_t fuse_after = 0;
    // Normals / EncodingVis rewrite the network input between the network and the compositor: wavefront only
    const bool probe = mode.ngp && (mode.render_mode == 2 || mode.render_mode == 10);
    // the glow visualisation is a wavefront-compositor term as well (the fused tail does not carry it)
    const bool wavefront_only = probe || (mode.ngp && mode.glow_mode != 0);
    // the decision needs the alive count after init_rays; when the tail starts after >= 1 whole-GPU
    // iteration the host reads it only once that first iteration is queued (no idle GPU while it waits)
    bool fuse_pending = false;
    // nerf_fused_after = 0 with speculative rounds: the tail is queued at once, ahead of its own check
    // (tail_prepare_kernel sets MarchCtrl::spec_ok; every tail kernel leaves all state untouched when it is 0),
    // and the host reads the check while the GPU runs the rounds -- no idle GPU waiting for init_rays' count
    bool tentative = false;
    if (c->p("nerf_fused") != 0.0 && !wavefront_only) {
        fuse_after = (uint32_t)std::max(0.0, c->p("nerf_fused_after"));
        if (fuse_after == 0 && c->p("nerf_spec_rounds") > 0) {
            fuse = true;
            tentative = true;
        } else if (fuse_after == 0) {
            HIPCHK(hipMemcpyAsync(c->h_alive, sched_src, 4, hipMemcpyDeviceToHost, c->s_nerf));
            HIPCHK(hipStreamSynchronize(c->s_nerf));
            fuse = (uint64_t)c->h_alive[0] * MAX_STEPS_BETWEEN_COMPACTION <= target;
        } else {
            HIPCHK(hipMemcpyAsync(c->h_alive, sched_src, 4, hipMemcpyDeviceToHost, c->s_nerf));
            HIPCHK(hipEventRecord(c->ev_alive, c->s_nerf));
            fuse_pending = true;
        }
    }
    const uint32_t blocks = std::max(1u, std::min((n_band + 255) / 256, (uint32_t)c->n_cus * 8));
    const uint32_t max_tiles = (uint32_t)((c->sample_cap + 15) / 16);
    // generate's grid: the marcher's DDA chains are long and uneven, so one trip over all rays (each
    // block waits for its slowest lane once) can beat the grid-stride cap
    const double gb = c->p("nerf_gen_blocks");
    const uint32_t gen_blocks = gb > 0 ? (uint32_t)gb : gb < 0 ? std::max(1u, (n_band + 255) / 256) : blocks;
    const int CHUNK = 4;
    int p = 0;
    uint32_t iter = 0;
    int chunk = 0;
    bool done = false;
    // trace_alt's one-step regime (fused.hip): tried at the first chunk boundary at which the alive
    // count may still exceed target / 2 (the boundary-sample caches are warm by then)
    bool os_open = !mode.ngp && c->p("nerf_onestep") != 0.0;
    const bool msr_on = !mode.ngp && c->p("nerf_msr") != 0.0;
    uint32_t& os_k = c->os_k;
    uint32_t& os_J = c->os_J;
    c->os_ran = false;
    // an upper bound of the current (schedule) alive count from the chunk readbacks; unknown before the first.
    // Every input of the decision is frame-wide, so all ranks of a banded frame take the same branch.
    uint32_t known_alive = UINT32_MAX;
    while (!done && iter < MARCH_ITER) {
        // a regime that reaches the speculative horizon continues with the next segment at once
        for (bool again = true; again && os_open && chunk >= 1 && !fuse && 2ull * known_alive > target;) {
            again = false;
            os_open = false;   // the count only shrinks: once the regime is over (or never was) it stays over
            HIPCHK(hipMemcpyAsync(c->h_ctrl, ctrl, sizeof(MarchCtrl), hipMemcpyDeviceToHost, c->s_nerf));
            HIPCHK(hipStreamSynchronize(c->s_nerf));
            const MarchCtrl& hc = *c->h_ctrl;
            const uint32_t ns = gsched ? hc.sched_alive[p] : hc.n_alive[p];
            if (ns > 0 && hc.i_step[p] < MARCH_ITER && steps_for(ns, target) == 1) {
                c->os_hist.ensure((size_t)3 * ONESTEP_HIST * 4);
                c->os_state.ensure(sizeof(OnestepState));
                OnestepArgs oa{};
                oa.vol = vol; oa.cam = cam; oa.sched = a.sched; oa.in = rb[p]; oa.out = rb[p ^ 1]; oa.ctrl = ctrl;
                oa.os = c->os_state.as<OnestepState>();
                oa.deaths_local = c->os_hist.as<uint32_t>();
                oa.deaths_sched = oa.deaths_local + ONESTEP_HIST;
                oa.nosample = oa.deaths_local + 2 * ONESTEP_HIST;
                oa.wfrag = c->net.wfrag; oa.grid_params = c->net.grid; oa.levels = c->net.levels;
                oa.frame_rgba = c->nerf_rgba.as<float4>(); oa.frame_depth = c->nerf_depth.as<float>(); oa.positions = c->nerf_pos.as<float>();
                oa.p = p; oa.target = target;
                if (!c->os_ran && P.collect_kernel_times) HIPCHK(hipEventRecord(c->ev_os0, c->s_nerf));
                const uint32_t horizon = (uint32_t)std::max(1.0, c->p("nerf_onestep_horizon"));
                launch_onestep_begin(oa, iter, horizon, c->os_ran ? 0 : 1, c->s_nerf);
                launch_onestep_pass(oa, c->net, 0, hc.n_alive[p], c->s_nerf);
                HIPCHK(hipGetLastError());
                if (gsched) sched_reduce(c, oa.deaths_sched, ONESTEP_HIST);   // own-row deaths summed over the ranks
                launch_onestep_schedule(oa, c->s_nerf);
                HIPCHK(hipMemcpyAsync(c->h_os, oa.os, sizeof(OnestepState), hipMemcpyDeviceToHost, c->s_nerf));
                HIPCHK(hipStreamSynchronize(c->s_nerf));
                const uint32_t J = c->h_os->J;
                launch_onestep_pass(oa, c->net, 1, hc.n_alive[p], c->s_nerf);
                HIPCHK(hipGetLastError());
                if (P.collect_kernel_times) HIPCHK(hipEventRecord(c->ev_os1, c->s_nerf));
                if (!c->os_ran) { os_k = c->h_os->k; os_J = 0; }
                c->os_ran = true;
                os_J += J;
                reduce_sched(p ^ 1);
                p ^= 1;
                iter += J;
                if (c->h_os->istep0 + J >= MARCH_ITER) break;
                if (J == c->h_os->H) { os_open = true; again = true; }   // horizon reached: n_steps may still be 1
            }
        }
        if (c->os_ran && c->h_os->istep0 + c->h_os->J >= MARCH_ITER) break;
        // multi-step speculative rounds (nerf.hip msr_*) while the step count is 2..7: each round commits the
        // iterations its guess S held for; a round whose first iteration does not take 2..7 steps is a no-op
        if (msr_on && chunk >= 1 && !fuse && (uint64_t)known_alive * MAX_STEPS_BETWEEN_COMPACTION > target) {
            c->msr_hist.ensure(4 * MSR_KMAX * 4);
            c->spec_t.ensure(c->sample_cap * 4);
            MsrArgs ma{};
            ma.vol = vol; ma.cam = cam; ma.sched = a.sched; ma.ctrl = ctrl; ma.target = target;
            ma.kmax = (uint32_t)std::min<double>(MSR_KMAX, std::max(1.0, c->p("nerf_msr_kmax")));
            // from the parameters and the frame size alone (ensure_samples' bound, so <= sample_cap), never from
            // sample_cap itself, which depends on the context's resize history: under the frame-wide schedule
            // every rank must choose the same round length K (msr_shape), or the ranks make different reductions
            ma.budget = (uint32_t)std::min<double>(std::max(1.0, c->p("nerf_msr_budget")),
                                                   (double)(MAX_STEPS_BETWEEN_COMPACTION - 1) * ma.kmax * (double)c->ray_cap);
            // rounds across step changes: fewer rounds (their fixed cost matters most on a thin band) for more
            // samples past the rays' ends; by default under the frame-wide schedule of a banded frame only
            const double span = c->p("nerf_msr_span");
            ma.span = span < 0 ? (gsched ? 1 : 0) : (span != 0.0 ? 1 : 0);
            c->msr_alpha.ensure(c->sample_cap * 4);
            ma.coords = c->coords.as<float>(); ma.samp = c->samp.as<uint2>(); ma.tbuf = c->spec_t.as<float>(); ma.net_out = c->net_out.as<uint2>();
            ma.abuf = c->msr_alpha.as<float>();
            ma.hist = c->msr_hist.as<uint32_t>();
            ma.frame_rgba = c->nerf_rgba.as<float4>(); ma.frame_depth = c->nerf_depth.as<float>(); ma.positions = c->nerf_pos.as<float>();
            const uint32_t mblocks = std::max(1u, std::min((n_band + 255) / 256, (uint32_t)c->n_cus * 8));
            while (true) {
                ma.in = rb[p]; ma.out = rb[p ^ 1]; ma.p = p;
                launch_msr_generate(ma, gen_blocks, c->s_nerf);
                if (P.collect_kernel_times) {
                    while (c->net_events.size() < 2 * (net_launches + 1)) { hipEvent_t e; HIPCHK(hipEventCreate(&e)); c->net_events.push_back(e); }
                }
                launch_network(c->net, c->coords.as<float>(), 7, 0, &ctrl->n_samples[p], c->net_out.as<uint16_t>(), 1, max_tiles, c->s_nerf,
                               P.collect_kernel_times ? c->net_events[2 * net_launches] : nullptr,
                               P.collect_kernel_times ? c->net_events[2 * net_launches + 1] : nullptr, net_rec(net_launches));
                launch_msr_count(ma, mblocks, c->s_nerf);
                if (gsched) sched_reduce(c, ma.hist + MSR_KMAX, MSR_KMAX);   // own-row deaths summed over the ranks
                launch_msr_schedule(ma, c->s_nerf);
                launch_msr_commit(ma, mblocks, c->s_nerf);
                HIPCHK(hipGetLastError());
                // the next round's frame-wide count is reduced before the one readback of the round (a no-op round's
                // reduction is unused; every rank makes it, as every rank sees the same no-op)
                reduce_sched(p ^ 1);
                HIPCHK(hipMemcpyAsync(c->h_ctrl, ctrl, sizeof(MarchCtrl), hipMemcpyDeviceToHost, c->s_nerf));
                HIPCHK(hipStreamSynchronize(c->s_nerf));
                const MarchCtrl& hc = *c->h_ctrl;
                if (hc.msr_K[p] == 0) break;   // no-op: the rays are still in buffer p
                ++net_launches;
                ++c->msr_rounds;
                p ^= 1;
                iter = hc.n_iter;
                // the (frame-wide) count the next round starts from
                known_alive = gsched ? hc.sched_alive[p] : hc.n_alive[p];
                if (known_alive == 0) { done = true; break; }
                if ((uint64_t)known_alive * MAX_STEPS_BETWEEN_COMPACTION <= target) {   // the 8-step tail's regime
                    if (!wavefront_only && c->p("nerf_fused") != 0.0) { fuse = true; fuse_after = iter; }
                    break;
                }
            }
            if (done) break;
        }
        if (fuse && iter >= fuse_after) {
            c->fused_work.ensure(16);
            c->fused_last = true;
            c->fused_k0 = iter;
            const int p_tail = p;
            const bool tentative_now = tentative;
            tentative = false;
            // speculative tail rounds (nerf.hip): each marches every alive ray K iterations ahead, one
            // whole-GPU network launch evaluates them, the compositor replays them exactly; the fused
            // kernel below then finishes whatever is still alive
            uint32_t rounds = (uint32_t)std::max(0.0, c->p("nerf_spec_rounds"));
            if (rounds > 1 && spec_adapt_on(c, mode) && c->spec_rounds_next) rounds = std::min(rounds, c->spec_rounds_next);
            uint8_t* hint_w = nullptr;   // the hints this frame writes (SpecArgs::hint), nullptr when it writes none
            c->spec_rounds = rounds;
            launch_tail_prepare(ctrl, c->fused_work.as<uint32_t>(), p, target, a.sched.global, c->s_nerf);
            if (tentative_now) {
                HIPCHK(hipMemcpyAsync(&c->h_alive[6], &ctrl->spec_ok, 4, hipMemcpyDeviceToHost, c->s_nerf));
                HIPCHK(hipEventRecord(c->ev_alive, c->s_nerf));
            }
            if (rounds) {
                c->spec_t.ensure(c->sample_cap * 4);
                // sample-parallel activations ahead of the compositing chain (not for the instant-NGP render modes
                // whose colour is not the network's: Positions, Depth, AO)
                const bool pre = c->p("nerf_spec_prepare") != 0.0 && !(mode.ngp && mode.render_mode != 1 && mode.render_mode != 6);
                if (pre) {
                    c->spec_pre.ensure(c->sample_cap * 16);
                    c->spec_pre_depth.ensure(c->sample_cap * 4);
                }
                SpecArgs sa{};
                sa.vol = vol; sa.cam = cam; sa.mode = mode; sa.ctrl = ctrl;
                sa.kmax = (uint32_t)std::min<double>(SPEC_KMAX, std::max(1.0, c->p("nerf_spec_kmax")));
                sa.budget = (uint32_t)std::min<double>(std::max(1.0, c->p("nerf_spec_budget")),
                                                       (double)MAX_STEPS_BETWEEN_COMPACTION * sa.kmax * (double)c->ray_cap);   // as ma.budget
                sa.coords = c->coords.as<float>(); sa.samp = c->samp.as<uint2>(); sa.tbuf = c->spec_t.as<float>();
                sa.net_out = c->net_out.as<uint2>();
                sa.frame_rgba = c->nerf_rgba.as<float4>(); sa.frame_depth = c->nerf_depth.as<float>(); sa.positions = c->nerf_pos.as<float>();
                sa.pre = pre ? c->spec_pre.as<float4>() : nullptr;
                sa.pre_depth = pre ? c->spec_pre_depth.as<float>() : nullptr;
                {   // hints are read when they were written for this view, and written only when the view repeats the
                    // last frame's (a moving camera neither reads nor writes them: no scattered byte stores for nothing)
                    uint8_t* hint = spec_hint_buf(c);
                    const uint64_t key = spec_view_key(c, a.focal, sc);
                    const bool any = c->p("nerf_spec_hint_any_view") != 0.0;
                    const bool read = hint && (key == c->spec_hint_key || any);
                    const bool write = hint && (read || any || key == c->spec_prev_view);
                    sa.hint = write ? hint : nullptr;
                    sa.hint_read = read ? 1 : 0;
                    if (write) c->spec_hint_key = key;
                }
                // rays alive after the head: at most the band's pixels (grid-stride over the device count)
                const uint32_t sblocks = std::max(1u, std::min((n_band + 255) / 256, (uint32_t)c->n_cus * 4));
                hint_w = sa.hint;
                for (uint32_t r = 0; r < rounds; ++r) {
                    sa.in = rb[p]; sa.out = rb[p ^ 1]; sa.p = p; sa.round = r;
                    // per-ray look-ahead in all but the last round (which then finishes nearly every ray)
                    sa.k_policy = (c->p("nerf_spec_k_policy") != 0.0 && r + 1 < rounds) ? 1 : 0;
                    launch_spec_generate(sa, sblocks, c->s_nerf);
                    if (P.collect_kernel_times) {
                        while (c->net_events.size() < 2 * (net_launches + 1)) { hipEvent_t e; HIPCHK(hipEventCreate(&e)); c->net_events.push_back(e); }
                    }
                    launch_network(c->net, c->coords.as<float>(), 7, 0, &ctrl->n_samples[p], c->net_out.as<uint16_t>(), 1, max_tiles, c->s_nerf,
                                   P.collect_kernel_times ? c->net_events[2 * net_launches] : nullptr,
                                   P.collect_kernel_times ? c->net_events[2 * net_launches + 1] : nullptr, net_rec(net_launches));
                    ++net_launches;
                    // render_frame gates the raytracer's path kernel on the head's network launch (the first round's)
                    if (r == 0) HIPCHK(hipEventRecord(c->ev_rt_go, c->s_nerf));
                    if (pre) launch_spec_prepare(sa, (uint32_t)c->n_cus * 4, c->s_nerf);
                    launch_spec_composite(sa, sblocks, c->s_nerf);
                    p ^= 1;
                }
                HIPCHK(hipGetLastError());
            }
            FusedArgs fa{};
            fa.vol = vol; fa.cam = cam; fa.mode = mode; fa.rays = rb[p]; fa.ctrl = ctrl; fa.p = p;
            fa.wfrag = c->net.wfrag; fa.grid_params = c->net.grid; fa.levels = c->net.levels;
            fa.frame_rgba = c->nerf_rgba.as<float4>(); fa.frame_depth = c->nerf_depth.as<float>(); fa.positions = c->nerf_pos.as<float>();
            fa.work = c->fused_work.as<uint32_t>();
            fa.lanes = (uint32_t)std::min(64.0, std::max(1.0, c->p("nerf_fused_lanes")));
            fa.hint = rounds ? hint_w : nullptr;
            // concurrent frames: the tail runs beside the raytracer on the CUs its grids leave free.  A
            // mid-frame switch (a long march, e.g. C4) happens long after the raytracer has finished: the
            // tail then gets the whole-GPU grid
            double fb = c->p("nerf_fused_blocks");
            const bool beside_rt = iter <= (uint32_t)std::max(0.0, c->p("nerf_fused_after"));
            if (fb < 0) fb = (beside_rt && c->p("concurrent_streams") != 0.0 && c->p("show_virtual_obj") != 0.0) ? 2.0 * std::max(1.0, c->p("rt_reserved_cus")) : 0.0;
            if (P.collect_kernel_times) HIPCHK(hipEventRecord(c->ev_fused0, c->s_nerf));
            launch_nerf_fused(fa, c->net, iter == 0 && !rounds ? std::min(c->h_alive[0], n_band) : n_band, (uint32_t)fb, c->s_nerf, rounds == 0);
            launch_tail_slots(ctrl, c->s_nerf);
            HIPCHK(hipGetLastError());
            if (P.collect_kernel_times) HIPCHK(hipEventRecord(c->ev_fused1, c->s_nerf));
            if (tentative_now) {
                HIPCHK(hipEventSynchronize(c->ev_alive));
                if (c->h_alive[6] == 0u) {   // not a tail: the queued kernels did nothing; march on as a wavefront
                    p = p_tail;
                    fuse = false;
                    c->fused_last = false;
                    c->spec_rounds = 0;
                    continue;
                }
            }
            HIPCHK(hipEventRecord(c->ev_nerf1, c->s_nerf));
            on_chunk(chunk + 1);
            break;
        }
        for (int k = 0; k < CHUNK && !(fuse && iter >= fuse_after); ++k, ++iter) {
            launch_generate(vol, rb[p], ctrl, p, target, iter, c->coords.as<float>(), c->samp.as<uint2>(), gen_blocks, mode.ngp, a.sched.global, c->s_nerf);
            if (P.collect_kernel_times) {
                while (c->net_events.size() < 2 * (net_launches + 1)) { hipEvent_t e; HIPCHK(hipEventCreate(&e)); c->net_events.push_back(e); }
            }
            // timing events recorded by the network kernel's own dispatch (hipExtLaunchKernelGGL)
            launch_network(c->net, c->coords.as<float>(), 7, 0, &ctrl->n_samples[p], c->net_out.as<uint16_t>(), 1, max_tiles, c->s_nerf,
                           P.collect_kernel_times ? c->net_events[2 * net_launches] : nullptr,
                           P.collect_kernel_times ? c->net_events[2 * net_launches + 1] : nullptr, net_rec(net_launches));
            if (probe)   // Normals / EncodingVis: input gradient or activation into the coordinates (testbed_nerf.cu:2363-2366)
                launch_field_probe(c->net, c->d_params.as<uint16_t>(), c->coords.as<float>(), &ctrl->n_samples[p], mode.render_mode,
                                   (int)c->p("visualized_layer"), (int)c->p("visualized_dimension"), c->s_nerf);
            HIPCHK(hipEventRecord(c->ev_rt_go, c->s_nerf));   // render_frame starts the raytracer after the head's network
            ++net_launches;
            launch_composite(vol, cam, mode, a.sched, rb[p], rb[p ^ 1], ctrl, p, target, iter, c->coords.as<float>(), c->samp.as<uint2>(), c->net_out.as<uint2>(),
                             c->nerf_rgba.as<float4>(), c->nerf_depth.as<float>(), c->nerf_pos.as<float>(), blocks, c->s_nerf, !fuse && !fuse_pending);
            reduce_sched(p ^ 1);
            p ^= 1;
            if (fuse_pending) {   // the first iteration is queued: now wait for init_rays' alive count
                HIPCHK(hipEventSynchronize(c->ev_alive));
                fuse = (uint64_t)c->h_alive[0] * MAX_STEPS_BETWEEN_COMPACTION <= target;
                fuse_pending = false;
            }
        }
        // readback of the alive count after this chunk; check the previous chunk's (already landed)
        HIPCHK(hipMemcpyAsync(&c->h_alive[2 * (chunk & 1)], sched_src, 8, hipMemcpyDeviceToHost, c->s_nerf));
        HIPCHK(hipGetLastError());
        if (chunk > 0) {
            // wait for the previous chunk's readback (the current chunk stays queued behind it)
            HIPCHK(hipEventSynchronize(c->ev_nerf1));
            const uint32_t* h = &c->h_alive[2 * ((chunk - 1) & 1)];
            known_alive = std::max(h[0], h[1]);
            if (h[0] == 0 && h[1] == 0) done = true;
            // once the alive count (it only shrinks) allows 8 steps per iteration, the rest of the march is
            // ray-local: hand it to the fused tail (the count read here is a chunk old, so it bounds the
            // count at `iter` from above)
            else if (!fuse && !wavefront_only && c->p("nerf_fused") != 0.0 && (uint64_t)std::max(h[0], h[1]) * MAX_STEPS_BETWEEN_COMPACTION <= target) {
                fuse = true;
                fuse_after = iter;
            }
        }
        HIPCHK(hipEventRecord(c->ev_nerf1, c->s_nerf));
        ++chunk;
        on_chunk(chunk);
    }
    if (c->sched_comm.replay && c->sched_comm.replay_cursor != c->sched_comm.replay_words)
        throw SngError(SNG_ERR_STATE, "schedule replay diverged: the frame made " + std::to_string(c->sched_comm.replay_calls) + " reductions, the records hold more");
    c->spec_prev_view = spec_view_key(c, a.focal, sc);
    return net_launches;
}

// the per-pixel look-ahead hints of the speculative rounds (nerf_spec_hint), zeroed whenever the NeRF
// resolution changes; nullptr when off
uint8_t* spec_hint_buf(sng_ctx* c) {
    if (c->p("nerf_spec_hint") == 0.0) return nullptr;
    const uint64_t px = (uint64_t)c->nerf_res[0] * (uint64_t)c->nerf_res[1];
    if (px != c->spec_hint_px) {
        c->spec_hint.ensure(px);
        HIPCHK(hipMemsetAsync(c->spec_hint.p, 0, px, c->s_nerf));
        c->spec_hint_px = px;
    }
    return c->spec_hint.as<uint8_t>();
}

// nerf_spec_adapt: the next trace's round count from this one's (MarchCtrl read back at the end of the frame).  A final
// round that evaluated fewer than nerf_spec_min_samples samples is dropped (its rays go to the fused kernel, which
// marches them ray-locally: C3's second round evaluates ~100 samples in a 15-us whole-GPU launch); a round comes back
// when the rays the fused kernel takes over would fill one (8 samples each, twice the threshold).  Only on hybrid
// frames whose NeRF tail runs beside the raytracer: the fused kernel's ray-local chain for those few rays is longer
// than the round it replaces (C3: 51 us), so it pays only where the NeRF stream is not the frame's critical path.
// The frame's bits do not depend on the count (the rounds are exact).
bool spec_adapt_on(const sng_ctx* c, const TraceMode& mode) {
    return c->p("nerf_spec_adapt") != 0.0 && !mode.ngp && c->p("concurrent_streams") != 0.0 && c->p("show_virtual_obj") != 0.0 && !c->objs.empty();
}
void spec_adapt(sng_ctx* c) {
    const uint32_t R = (uint32_t)std::max(0.0, c->p("nerf_spec_rounds")), r = c->spec_rounds;
    if (c->p("nerf_spec_adapt") == 0.0 || R < 2 || !c->fused_last || r == 0) { c->spec_rounds_next = 0; return; }
    const MarchCtrl& h = *c->h_ctrl;
    const double min_s = std::max(0.0, c->p("nerf_spec_min_samples"));
    uint32_t next = std::min(r, R);
    if (next > 1 && (double)h.spec_round_samples[std::min(next, 4u) - 1] < min_s) --next;
    else if (next < R && (double)h.fused_rays_in * MAX_STEPS_BETWEEN_COMPACTION >= 2.0 * min_s) ++next;
    c->spec_rounds_next = next;
}

// march statistics of the last trace (MarchCtrl read back at the end of the frame)
void march_stats(const sng_ctx* c, const sng_frame_params& P, sng_frame_result* out) {
    out->n_iterations = c->h_ctrl->n_iter;
    out->n_hit = c->h_ctrl->n_hit;
    out->n_samples = c->h_ctrl->total_samples;
    out->n_samples_network = c->h_ctrl->net_samples;
    out->n_samples_reused = c->h_ctrl->reused_samples;
    out->fused_from_iter = c->fused_last ? c->fused_k0 : c->h_ctrl->n_iter;
    out->onestep_from_iter = c->os_ran ? c->os_k : c->h_ctrl->n_iter;
    out->onestep_iterations = c->os_ran ? c->os_J : 0u;
    if (c->os_ran) {
        HIPCHK(hipMemcpy(c->h_os, c->os_state.p, sizeof(OnestepState), hipMemcpyDeviceToHost));
        out->onestep_field_evals = (uint32_t)c->h_os->evals[1];
    }
    out->n_reference_slots = ref_slots_of(c);
    out->spec_rounds = c->fused_last ? c->spec_rounds : 0u;
    out->spec_evals = (uint32_t)c->h_ctrl->spec_evals;
    out->spec_exec = (uint32_t)c->h_ctrl->spec_exec;
    out->msr_rounds = c->msr_rounds;
    out->msr_evals = (uint32_t)c->h_ctrl->msr_evals;
    out->msr_exec = (uint32_t)c->h_ctrl->msr_exec;
    out->sched_reductions = (uint32_t)c->sched_comm.replay_calls;
    std::memcpy(out->alive_per_iter, c->h_ctrl->alive_hist, sizeof(out->alive_per_iter));
    std::memcpy(out->steps_per_iter, c->h_ctrl->steps_hist, sizeof(out->steps_per_iter));
    std::memcpy(out->samples_per_iter, c->h_ctrl->samples_hist, sizeof(out->samples_per_iter));
}

// hipEvent durations of the network launches and of the fused tail (collect_kernel_times)
void network_times(sng_ctx* c, const sng_frame_params& P, uint32_t net_launches, sng_frame_result* out) {
    out->network_launches = net_launches;
    if (!P.collect_kernel_times) return;
    float tot = 0.0f;
    for (uint32_t k = 0; k < net_launches; ++k) {
        float ms = 0.0f;
        HIPCHK(hipEventElapsedTime(&ms, c->net_events[2 * k], c->net_events[2 * k + 1]));
        tot += ms;
    }
    out->ms_network = tot;
    out->n_launch_rec = std::min<uint32_t>(net_launches, 16u);
    for (uint32_t k = 0; k < out->n_launch_rec; ++k) {
        HIPCHK(hipEventElapsedTime(&out->ms_network_launch[k], c->net_events[2 * k], c->net_events[2 * k + 1]));
        out->samples_network_launch[k] = c->h_ctrl->net_launch_samples[k];
    }
    if (c->fused_last) HIPCHK(hipEventElapsedTime(&out->ms_fused_tail, c->ev_fused0, c->ev_fused1));
    if (c->os_ran) HIPCHK(hipEventElapsedTime(&out->ms_onestep, c->ev_os0, c->ev_os1));
}

void render_frame(sng_ctx* c, const sng_frame_params* fp, sng_frame_result* out) {
    if (c->win[0] <= 0) throw SngError(SNG_ERR_STATE, "sng_set_window first");
    if ((int)c->p("res_factor") != c->last_res_factor) resize(c);
    const bool show_nerf = c->p("show_nerf") != 0.0;
    if (show_nerf && !(c->has_model && c->has_bitfield)) throw SngError(SNG_ERR_STATE, "no NeRF model/density grid loaded");
    animate(c);
    if (c->scene_dirty) upload_scene(c);
    sng_frame_params P{};
    if (fp) P = *fp;
    const uint32_t target = P.target_n_queries ? P.target_n_queries : 2u * 1024u * 1024u;
    ensure_samples(c, target);
    const int MW = c->mesh_res[0], MH = c->mesh_res[1], NW = c->nerf_res[0], NH = c->nerf_res[1], S = c->vo_scale_eff;
    int y0 = P.row_begin, y1 = P.row_end;
    if (y0 == 0 && y1 == 0) { y0 = 0; y1 = MH; }
    if (y0 < 0 || y1 > MH || y0 >= y1) throw SngError(SNG_ERR_INVALID, "bad row band");
    const int radius = (int)c->p("nerf_shadow_samples") / 2;
    const bool shadows = c->p("shadow_on_nerf") != 0.0 && show_nerf;
    // NeRF rows: overlay needs [ny0, ny1); shadows need normals +-r; normals need positions +-2
    const int ny0 = std::min(NH, y0 / S), ny1 = std::min(NH, (y1 - 1) / S + 1);
    const int halo_n = shadows ? radius : 0;
    const int nr0 = std::max(0, ny0 - halo_n), nr1 = std::min(NH, ny1 + halo_n);
    const int tr0 = std::max(0, nr0 - 2), tr1 = std::min(NH, nr1 + 2);
    // owned NeRF rows: [ceil(y0 / S), ceil(y1 / S)) -- consecutive mesh bands partition the NeRF rows
    const int own0 = std::min(ny1, (y0 + S - 1) / S), own1 = ny1;
    // the raytracer's NeRF shadow test uses the density bitfield whether or not the NeRF is shown
    // (engine.cu:386-397 passes m_nerf.density_grid_bitfield unconditionally)
    Volume vol{};
    resolve_occ_brick(c);
    if (c->has_model && c->has_bitfield) vol = make_volume(c);
    else { vol.render_aabb = c->box; vol.train_aabb = c->box; vol.to_local = {mk(1, 0, 0), mk(0, 1, 0), mk(0, 0, 1)}; vol.to_local_identity = 1; }
    const CamDev cam = cam_dev(c);
    const f2 sc = render_screen_center(c);

    HIPCHK(hipEventRecord(c->ev_start, c->s_nerf));
    // The raytracer (s_rt) and the NeRF wavefront (s_nerf) are independent until the overlay.
    // concurrent_streams = 1: the raytracer starts after the first `rt_start_chunk` chunks of
    // wavefront iterations, i.e. once the NeRF's throughput-heavy head (nearly all rays alive)
    // has run on the whole GPU; it then overlaps the latency-bound tail iterations.
    const bool concurrent = c->p("concurrent_streams") != 0.0;
    int rt_start_chunk = (concurrent && show_nerf) ? (int)c->p("rt_start_chunk") : 0;
    if (rt_start_chunk < 0) rt_start_chunk = (y1 - y0) * 10 >= MH * 6 ? 1 : 0;
    bool rt_enqueued = false, rt_sorted = false;
    // rt_first: the path kernel's workgroups land before init_rays takes the CUs (the faster of the concurrent frame's two
    // dispatch orders): init_rays waits, on the device and bounded, for the first one
    const bool rt_first = concurrent && show_nerf && rt_start_chunk <= 0 && c->p("rt_first") != 0.0 && c->p("show_virtual_obj") != 0.0 &&
                          !c->objs.empty();
    if (rt_first) {
        if (!c->rt_started.p) {
            c->rt_started.ensure(256);
            HIPCHK(hipMemsetAsync(c->rt_started.p, 0, 256, c->s_rt));
        }
        c->rt_wait_seq = ++c->frame_seq;
        if (c->rt_wait_seq == 0) c->rt_wait_seq = ++c->frame_seq;   // 0 = no wait
    }
    // phase 0: everything after `after`; 1 (concurrent frames, at frame start): the work that does not
    // wait for the NeRF head -- mesh rays and the tile-order sort -- so it overlaps init_rays; 2: the
    // rest, gated on `after`
    auto enqueue_raytracer = [&](hipEvent_t after, int phase) {
        // ---- raytracer (RayTracer::render, raytracer.cu:312-370) on its own stream
        if (phase == 0) HIPCHK(hipStreamWaitEvent(c->s_rt, after, 0));
        if (phase != 2) HIPCHK(hipEventRecord(c->ev_rt0, c->s_rt));
        if (phase != 2 && (c->mesh_reset || P.reset_accumulation)) {
            const int mres[2] = {MW, MH};
            launch_mesh_rays(MW, MH, y0, y1, cam, focal_for(c, mres), sc, c->mesh_o.as<float4>(), c->mesh_d.as<float4>(), c->acc_rgba.as<float4>(),
                             c->acc_depth.as<float>(), c->s_rt);
            c->mesh_reset = false;
        }
        if (c->p("show_virtual_obj") != 0.0 && !c->objs.empty()) {
            RaytraceArgs ra{};
            c->params["rt_fused_shadow_used"] = 0;
            if (rt_first) { ra.started = c->rt_started.as<uint32_t>(); ra.started_seq = c->rt_wait_seq; }
            ra.vol = vol;
            ra.W = MW; ra.row0 = y0; ra.row1 = y1;
            ra.up = cam.c0;
            ra.objs = c->d_objs.as<ObjectGpu>(); ra.n_objs = (int)c->objs.size();
            ra.lights = c->d_lights.as<LightGpu>(); ra.n_lights = (int)c->lights.size();
            ra.mats = c->d_mats.as<MaterialGpu>();
            ra.samples = (uint32_t)c->p("light_samples");
            ra.bounces = (uint32_t)c->p("path_trace_depth");
            ra.shadow_iters = (uint32_t)c->p("syn_shadow_samples");
            ra.shadow_steps = (uint32_t)c->p("n_steps");
            ra.lens = (float)c->p("lens_size");
            ra.show_nerf_shadow = c->p("shadow_on_virtual_obj") != 0.0;
            ra.syn_shadow_factor = (float)c->p("syn_shadow_intensity");
            ra.scene_blob = c->d_scene_blob.as<float4>();
            ra.scene_f4 = c->scene_f4;
            // max stack use of the reference traversal is depth + 1; FixedStack<32> drops pushes at 31
            ra.stack_depth = std::min<uint32_t>(32u, c->bvh_stack);
            ra.bvh_flat = c->p("bvh_flat") != 0.0 ? 1 : 0;
            // blob + stacks in LDS: two 512-thread workgroups per CU (80 KB each), else one of 1024 threads
            // (one blob copy per CU, 160 KB); both give 16 waves per CU
            const uint64_t blob_b = (uint64_t)c->scene_f4 * 16;
            const bool lds_ok = c->p("scene_lds") != 0.0;
            ra.lds_tpb = 512;
            ra.scene_in_lds = 0;
            if (lds_ok && blob_b + (uint64_t)ra.stack_depth * 512 * 4 <= 80u * 1024u) ra.scene_in_lds = 1;
            else if (lds_ok && blob_b + (uint64_t)ra.stack_depth * 1024 * 4 <= 160u * 1024u) { ra.scene_in_lds = 1; ra.lds_tpb = 1024; }
            // persistent raytracer grids leave `rt_reserved_cus` CUs' worth of room for the NeRF
            // wavefront running beside them on the other stream (concurrent mode only)
            const int reserve = concurrent && show_nerf ? (int)c->p("rt_reserved_cus") : 0;
            ra.persistent_blocks = (uint32_t)std::max(1, c->n_cus - std::max(0, reserve));
            c->rt_work.ensure(RT_WORK_WORDS * sizeof(uint32_t));
            ra.work = c->rt_work.as<uint32_t>();
            if (c->p("rt_count") != 0.0 && phase != 1) {   // counting frame: traversal counters (sng_rt_counters)
                c->rt_counts.ensure(8 * sizeof(unsigned long long));
                HIPCHK(hipMemsetAsync(c->rt_counts.p, 0, 8 * sizeof(unsigned long long), c->s_rt));
                ra.counts = c->rt_counts.as<unsigned long long>();
                ra.count_waves = c->p("rt_count") == 2.0 ? 1 : 0;
            }
            // tile width 1, 2, 4 or 8 pixels (else 8); height 1..8 (0: square), at most 64 pixels per wave
            {
                const int tw = (int)c->p("rt_tile"), th = (int)c->p("rt_tile_h");
                ra.tile = (tw == 1 || tw == 2 || tw == 4) ? tw : 8;
                ra.tile_h = (th >= 1 && th <= 8) ? th : ra.tile;
            }
            ra.buffer_type = (int)c->p("rt_buffer_type");
            ra.spread = c->p("rt_spread") != 0.0 ? 1 : 0;
            if (c->p("rt_tile_order") != 0.0) {
                const uint32_t n_tiles = (uint32_t)((MW + ra.tile - 1) / ra.tile) * (uint32_t)((y1 - y0 + ra.tile_h - 1) / ra.tile_h);
                const uint64_t key = ((uint64_t)MW << 40) ^ ((uint64_t)y0 << 20) ^ (uint64_t)y1 ^ ((uint64_t)ra.tile << 60) ^ ((uint64_t)ra.tile_h << 56);
                if (phase != 2) {
#ifdef RT_CHAIN_PROBE
                    c->rt_tile_cost.ensure((size_t)n_tiles * 4 * 9);   // + the chain probe's 8 words per tile
#else
                    c->rt_tile_cost.ensure((size_t)n_tiles * 4);
#endif
                    c->rt_tile_order.ensure((size_t)(n_tiles + 64) * 4);   // + launch_tile_sort's 64 aux words
                    rt_sorted = key == c->rt_tile_key;
                    if (rt_sorted) launch_tile_sort(c->rt_tile_cost.as<uint32_t>(), n_tiles, c->rt_tile_order.as<uint32_t>(),
                                                    c->rt_tile_order.as<uint32_t>() + n_tiles, c->s_rt);
                    c->rt_tile_key = key;
                }
                if (rt_sorted) {
                    ra.tile_order = c->rt_tile_order.as<uint32_t>();
                    ra.prio_tiles = (uint32_t)(std::max(0.0, c->p("rt_prio_frac")) * n_tiles);
                    ra.prio2_tiles = (uint32_t)(std::max(0.0, c->p("rt_prio2_frac")) * n_tiles);
                }
                ra.tile_cost = c->rt_tile_cost.as<uint32_t>();
            }
            if (phase == 1) return;
            if (phase == 2) HIPCHK(hipStreamWaitEvent(c->s_rt, after, 0));
            // deferred shadow rays (wavefront) whenever the path has point-light shadow tests and the
            // worst-case queues (every pixel hits on every sample and bounce) fit the budget
            uint32_t n_point = 0;
            for (auto& l : c->lights) n_point += l.type == 0 ? 1u : 0u;
            const uint64_t n_px = (uint64_t)(y1 - y0) * (uint64_t)MW;
            const uint64_t cap = n_px * ra.samples * ra.bounces;
            RtQueue q{};
            q.nls = (uint32_t)c->lights.size() * ra.shadow_iters;
            q.nps = n_point * ra.shadow_iters;
            q.rec_stride = 2;
            const uint64_t bytes = cap * (16ull * q.rec_stride + 16ull * q.nls + 16ull * q.nps + 4ull * q.nps) + (uint64_t)MW * MH * 4;
            // (the ImgBufferType debug views come from the one-kernel path, which carries their sums)
            const bool wavefront = c->p("rt_wavefront") != 0.0 && ra.buffer_type == 0 && ra.show_nerf_shadow && q.nps > 0 && cap > 0 && cap < (1ull << 31) &&
                                   bytes <= (uint64_t)(c->p("rt_queue_gb") * 1073741824.0);
            if (wavefront) {
                c->rt_rec.ensure(cap * 16ull * q.rec_stride);
                c->rt_srec.ensure(cap * 16ull * q.nps);
                c->rt_lc.ensure(cap * 16ull * std::max<uint32_t>(1u, q.nls));
                c->rt_mask.ensure(cap * 4ull * q.nps);
                c->rt_head.ensure((uint64_t)MW * MH * 4);
                q.rec = c->rt_rec.as<float4>(); q.lc = c->rt_lc.as<float4>(); q.srec = c->rt_srec.as<float4>(); q.mask = c->rt_mask.as<float>();
                q.head = c->rt_head.as<int>(); q.count = ra.work + RT_REC_COUNT; q.cap = (uint32_t)cap;
                // shadow-ray grid: the CUs the path kernel leaves to the NeRF tail too when rt_shadow_all_cus
                // (by then the tail has mostly finished)
                const uint32_t sb = c->p("rt_shadow_all_cus") != 0.0 ? (uint32_t)c->n_cus * 1024u / ra.lds_tpb : 0u;
                const uint64_t max_hits = (uint64_t)ra.samples * ra.bounces;
                const uint64_t stage_b = 16ull * (64ull * q.rec_stride + (64ull * q.nps + 3) / 4);   // rt_record_colour_kernel's LDS per wave
                if (c->p("rt_plist") != 0.0 && max_hits <= 255 && stage_b <= 64ull * 1024) {
                    // per-pixel record lists: the colour replay reads each pixel's records directly instead of
                    // walking their chain (one dependent load per record)
                    c->rt_plist.ensure(n_px * max_hits * 4);
                    c->rt_pcount.ensure(n_px);
                    c->rt_rval.ensure(cap * 16);
                    q.plist = c->rt_plist.as<int>();
                    q.pcount = c->rt_pcount.as<uint8_t>();
                    q.rval = c->rt_rval.as<float4>();
                    q.max_hits = (uint32_t)max_hits;
                }
                // banded frames (at most rt_fused_tiles_per_wave tiles per path-kernel wave): the waves past their tiles
                // trace the shadow rays as the records appear, and the shadow-ray kernel is not launched
                {
                    const uint32_t n_tiles = (uint32_t)((MW + ra.tile - 1) / ra.tile) * (uint32_t)((y1 - y0 + ra.tile_h - 1) / ra.tile_h);
                    const uint32_t tpb = ra.scene_in_lds ? ra.lds_tpb : 512u;
                    const size_t lds_need = (ra.scene_in_lds ? (size_t)ra.scene_f4 * 16 : 0) + (size_t)ra.stack_depth * tpb * 4 + RT_FQ_WORDS * 4;
                    ra.fused_shadow = c->p("rt_fused_shadow") != 0.0 && ra.spread && !ra.counts && n_tiles <= (uint32_t)(c->p("rt_fused_tiles_per_wave") * ra.persistent_blocks * 16u) &&
                                      lds_need <= 160u * 1024u ? 1 : 0;
                    c->params["rt_fused_shadow_used"] = ra.fused_shadow;
                }
                uint32_t* rng = c->rng_mesh.as<uint32_t>();
                uint32_t n_rng = c->n_rng_mesh;
                if (c->p("rt_rng") != 0.0) {   // per-(pixel, sample) streams, the sample-parallel path kernel
                    if (!q.plist || ra.counts || ra.bounces > RT_SP_MAX_BOUNCES || ra.samples < 1 || ra.samples > 64)
                        throw SngError(SNG_ERR_INVALID, "rt_rng 1 needs the record lists (rt_plist), no counting frame, path_trace_depth <= 4 "
                                                        "and 1..64 light_samples");
                    const uint64_t n_sp = (uint64_t)MW * MH * ra.samples;
                    if (n_sp >= (1ull << 32)) throw SngError(SNG_ERR_INVALID, "rt_rng 1: too many (pixel, sample) streams");
                    const uint64_t key = n_sp ^ ((uint64_t)ra.samples << 40);
                    if (key != c->rng_sp_key) {   // curand_init(1999, pixel * samples + s, 0)
                        c->rng_mesh_sp.ensure(n_sp * 24);
                        launch_xorwow_init((uint32_t)n_sp, PT_SEED, c->d_seq.as<uint32_t>(), c->rng_mesh_sp.as<uint32_t>(), c->s_rt);
                        c->rng_sp_key = key;
                    }
                    rng = c->rng_mesh_sp.as<uint32_t>();
                    n_rng = (uint32_t)n_sp;
                    ra.sample_par = 1;
                    ra.fused_shadow = 0;
                    c->params["rt_fused_shadow_used"] = 0;
                }
                launch_raytrace_wavefront(ra, q, c->mesh_o.as<float4>(), c->mesh_d.as<float4>(), rng, n_rng,
                                          c->acc_rgba.as<float4>(), c->acc_depth.as<float>(), sb, c->s_rt);
            } else {
                launch_raytrace(ra, c->mesh_o.as<float4>(), c->mesh_d.as<float4>(), c->rng_mesh.as<uint32_t>(), c->n_rng_mesh, c->acc_rgba.as<float4>(),
                                c->acc_depth.as<float>(), c->s_rt);
            }
        }
        if (phase == 1) return;
        if (phase == 2 && !(c->p("show_virtual_obj") != 0.0 && !c->objs.empty())) HIPCHK(hipStreamWaitEvent(c->s_rt, after, 0));
        HIPCHK(hipEventRecord(c->ev_rt1, c->s_rt));
        rt_enqueued = true;
    };
    if (rt_start_chunk <= 0) enqueue_raytracer(c->ev_start, 0);
    else enqueue_raytracer(nullptr, 1);
    if (!concurrent) HIPCHK(hipStreamWaitEvent(c->s_nerf, c->ev_rt1, 0));

    // ---- NeRF (Testbed::render SyNeRFgine overload, testbed.cu:4353-4404)
    HIPCHK(hipEventRecord(c->ev_nerf0, c->s_nerf));
    uint32_t net_launches = 0;
    if (show_nerf) {
        TraceMode mode{0, 1, 1.0f};
        net_launches = trace_nerf(c, P, vol, cam, sc, tr0, tr1, own0, own1, mode, target, [&](int chunk) {
            // gated on the last network launch of the head (ev_rt_go, trace_nerf), not the chunk's end
            if (!rt_enqueued && chunk == rt_start_chunk) enqueue_raytracer(c->ev_rt_go, 2);
        });
        // write_normals_to_buffer (testbed_nerf.cu:1523-1612): the G-buffer only the NeRF shadow pass reads; without
        // shadow_on_nerf no output depends on it (nerf_gbuffer = 1 keeps it for sng_frame_buffer("nerf_normals"))
        if (shadows || c->p("nerf_gbuffer") != 0.0) launch_normals(NW, NH, nr0, nr1, c->nerf_pos.as<float>(), c->nerf_nrm.as<float>(), c->s_nerf);
    }
    c->rt_wait_seq = 0;
    if (!rt_enqueued) {
        HIPCHK(hipEventRecord(c->ev_rt_go, c->s_nerf));
        enqueue_raytracer(c->ev_rt_go, rt_start_chunk <= 0 ? 0 : 2);
    }
    HIPCHK(hipEventRecord(c->ev_shadow1, c->s_nerf));   // end of the trace
    if (shadows && !c->objs.empty()) {
        ShadowArgs sa{};
        sa.vol = vol;
        sa.W = NW; sa.H = NH; sa.row0 = ny0; sa.row1 = ny1;
        sa.radius = radius;
        sa.intensity = (float)c->p("nerf_shadow_intensity");
        sa.threshold = (float)c->p("nerf_on_nerf_shadow_threshold");
        sa.objs = c->d_objs.as<ObjectGpu>(); sa.n_objs = (int)c->objs.size();
        sa.lights = c->d_lights.as<LightGpu>(); sa.n_lights = (int)c->lights.size();
        sa.n_point = n_point_lights(c);
        shadow_scene(c, sa);
        c->shadow_scratch.ensure(shadow_scratch_bytes(sa));
        launch_shadows(sa, c->nerf_rgba.as<float4>(), c->nerf_pos.as<float>(), c->nerf_nrm.as<float>(), c->rng_nerf.as<uint32_t>(), c->n_rng_nerf,
                       c->shadow_scratch.p, c->s_nerf);
    } else if (shadows) {
        ShadowArgs sa{};
        sa.vol = vol;
        sa.W = NW; sa.H = NH; sa.row0 = ny0; sa.row1 = ny1;
        sa.radius = radius;
        sa.intensity = (float)c->p("nerf_shadow_intensity");
        sa.threshold = (float)c->p("nerf_on_nerf_shadow_threshold");
        sa.objs = c->d_objs.as<ObjectGpu>(); sa.n_objs = 0;
        sa.lights = c->d_lights.as<LightGpu>(); sa.n_lights = (int)c->lights.size();
        sa.n_point = n_point_lights(c);
        shadow_scene(c, sa);
        c->shadow_scratch.ensure(shadow_scratch_bytes(sa));
        launch_shadows(sa, c->nerf_rgba.as<float4>(), c->nerf_pos.as<float>(), c->nerf_nrm.as<float>(), c->rng_nerf.as<uint32_t>(), c->n_rng_nerf,
                       c->shadow_scratch.p, c->s_nerf);
    }
    HIPCHK(hipEventRecord(c->ev_nerf1, c->s_nerf));
    // ---- overlay (RayTracer::overlay, raytracer.cu:372-392) after both streams
    HIPCHK(hipStreamWaitEvent(c->s_nerf, c->ev_rt1, 0));
    launch_overlay(MW, y0, y1, S, MW / S, NW * NH, show_nerf ? 1 : 0, (float)c->p("depth_offset"), std::pow(2.0f, (float)c->p("exposure")), (int)c->p("srgb"),
                   (int)c->p("tonemap_curve"),
                   c->acc_rgba.as<float4>(), c->acc_depth.as<float>(), c->nerf_rgba.as<float4>(), c->nerf_depth.as<float>(), c->final_rgba.as<float4>(),
                   c->final_depth.as<float>(), c->s_nerf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev_end, c->s_nerf));
    if (show_nerf) HIPCHK(hipMemcpyAsync(c->h_ctrl, c->ctrl.p, sizeof(MarchCtrl), hipMemcpyDeviceToHost, c->s_nerf));
    HIPCHK(hipStreamSynchronize(c->s_nerf));
    if (show_nerf) spec_adapt(c);

    if (out) {
        std::memset(out, 0, sizeof(*out));
        out->d_final_rgba = c->final_rgba.as<float>();
        out->d_final_depth = c->final_depth.as<float>();
        out->d_nerf_rgba = c->nerf_rgba.as<float>();
        out->d_nerf_depth = c->nerf_depth.as<float>();
        out->d_nerf_positions = c->nerf_pos.as<float>();
        out->d_nerf_normals = c->nerf_nrm.as<float>();
        out->d_syn_rgba = c->acc_rgba.as<float>();
        out->d_syn_depth = c->acc_depth.as<float>();
        if (show_nerf) march_stats(c, P, out);
        HIPCHK(hipEventElapsedTime(&out->ms_frame, c->ev_start, c->ev_end));
        HIPCHK(hipEventElapsedTime(&out->ms_raytrace, c->ev_rt0, c->ev_rt1));
        HIPCHK(hipEventElapsedTime(&out->ms_nerf, c->ev_nerf0, c->ev_shadow1));
        HIPCHK(hipEventElapsedTime(&out->ms_shadow, c->ev_shadow1, c->ev_nerf1));
        float ov = 0.0f;
        HIPCHK(hipEventElapsedTime(&ov, c->ev_nerf1, c->ev_end));
        out->ms_overlay = ov;
        network_times(c, P, net_launches, out);
    }
}

// Testbed::render_nerf (testbed_nerf.cu:2679-2837): the instant-NGP render path --
// NerfTracer::trace + composite_kernel_nerf + shade_kernel_nerf into the NeRF frame buffer, with
// ERenderMode "render_mode" (0 AO, 1 Shade, 3 Positions, 4 Depth, 6 Cost, 10 EncodingVis) and
// "depth_scale" (1 / dataset.scale).  NeRF only: no mesh, shadows or overlay.
void render_nerf_ngp(sng_ctx* c, const sng_frame_params* fp, sng_frame_result* out) {
    if (c->win[0] <= 0) throw SngError(SNG_ERR_STATE, "sng_set_window first");
    if ((int)c->p("res_factor") != c->last_res_factor) resize(c);
    if (!(c->has_model && c->has_bitfield)) throw SngError(SNG_ERR_STATE, "no NeRF model/density grid loaded");
    const int vdim = (int)c->p("visualized_dimension"), vlayer = (int)c->p("visualized_layer");
    const int rm = vdim > -1 ? 10 : (int)c->p("render_mode");   // testbed_nerf.cu:2491
    if (!(rm == 0 || rm == 1 || rm == 2 || rm == 3 || rm == 4 || rm == 6 || rm == 10))
        throw SngError(SNG_ERR_INVALID, "render_mode " + std::to_string(rm) + " is not supported by the instant-NGP path (AO, Shade, Normals, Positions, Depth, Cost, EncodingVis)");
    if (rm == 10) {   // tcnn visualize_activation's range checks (NerfNetwork::width, base.json: 1 density + 2 rgb hidden layers)
        static const int width[5] = {32, 64, 32, 64, 64};
        if (vlayer < 0 || vlayer > 4 || vdim < 0 || vdim >= width[vlayer])
            throw SngError(SNG_ERR_INVALID, "EncodingVis: visualized layer " + std::to_string(vlayer) + " / dimension " + std::to_string(vdim) + " out of range");
    }
    sng_frame_params P{};
    if (fp) P = *fp;
    const uint32_t target = P.target_n_queries ? P.target_n_queries : 2u * 1024u * 1024u;
    ensure_samples(c, target);
    const int NH = c->nerf_res[1];
    int r0 = P.row_begin, r1 = P.row_end;
    if (r0 == 0 && r1 == 0) { r0 = 0; r1 = NH; }
    if (r0 < 0 || r1 > NH || r0 >= r1) throw SngError(SNG_ERR_INVALID, "bad row band");
    const Volume vol = make_volume(c);
    const CamDev cam = cam_dev(c);
    const f2 sc = render_screen_center(c);
    const TraceMode mode{1, rm, (float)c->p("depth_scale"), (int)c->p("glow_mode"), (float)c->p("glow_y_cutoff")};
    HIPCHK(hipEventRecord(c->ev_start, c->s_nerf));
    HIPCHK(hipEventRecord(c->ev_nerf0, c->s_nerf));
    const uint32_t net_launches = trace_nerf(c, P, vol, cam, sc, r0, r1, r0, r1, mode, target, [](int) {});
    HIPCHK(hipEventRecord(c->ev_end, c->s_nerf));
    HIPCHK(hipMemcpyAsync(c->h_ctrl, c->ctrl.p, sizeof(MarchCtrl), hipMemcpyDeviceToHost, c->s_nerf));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->s_nerf));
    spec_adapt(c);
    if (out) {
        std::memset(out, 0, sizeof(*out));
        out->d_nerf_rgba = c->nerf_rgba.as<float>();
        out->d_nerf_depth = c->nerf_depth.as<float>();
        march_stats(c, P, out);
        HIPCHK(hipEventElapsedTime(&out->ms_frame, c->ev_start, c->ev_end));
        out->ms_nerf = out->ms_frame;
        network_times(c, P, net_launches, out);
    }
}

}  // namespace sng_host
