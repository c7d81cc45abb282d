// host_snapshot.cpp -- .ingp snapshots: Testbed::load_snapshot (testbed.cu:4878-5015; zlib(msgpack), 244-270) and
// Testbed::save_snapshot (testbed.cu:4812-4876).
#include "host.h"

namespace sng_host {

// ---- .ingp snapshot (Testbed::load_snapshot, testbed.cu:4878-5015; zlib(msgpack), 244-270) ----
std::vector<uint8_t> inflate_all(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw SngError(SNG_ERR_IO, "Network snapshot '" + path + "' does not exist.");
    std::vector<uint8_t> in((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    bool compressed = path.size() >= 5 && path.substr(path.size() - 5) == ".ingp";
    if (!compressed) return in;
    z_stream zs{};
    if (inflateInit2(&zs, 15 + 32) != Z_OK) throw SngError(SNG_ERR_IO, "zlib init failed");
    std::vector<uint8_t> out;
    std::vector<uint8_t> buf(1 << 20);
    zs.next_in = in.data();
    zs.avail_in = (uInt)in.size();
    int r;
    do {
        zs.next_out = buf.data();
        zs.avail_out = (uInt)buf.size();
        r = inflate(&zs, Z_NO_FLUSH);
        if (r != Z_OK && r != Z_STREAM_END) { inflateEnd(&zs); throw SngError(SNG_ERR_IO, "zlib inflate failed"); }
        out.insert(out.end(), buf.data(), buf.data() + (buf.size() - zs.avail_out));
    } while (r != Z_STREAM_END);
    inflateEnd(&zs);
    return out;
}
float jnum(const JValue& v, float dflt) { return v.type == JValue::Null ? dflt : v.as_float(); }
// tcnn vec/mat JSON: arrays; mat4x3 as 4 columns of 3 or 3 rows of 4 [tcnn vec_json.h, unvendored]
void read_mat43(const JValue& m, float out[12]) {
    if (m.size() == 4 && m[0].size() == 3) {
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 3; ++j) out[3 * i + j] = m[i][j].as_float();
    } else if (m.size() == 3 && m[0].size() == 4) {
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 3; ++j) out[3 * i + j] = m[j][i].as_float();
    } else throw SngError(SNG_ERR_IO, "unexpected camera matrix encoding");
}
// Testbed::load_snapshot (testbed.cu:4878-5015): zlib(msgpack) -> model config, fp16 params,
// fp16 density grid and camera.  Host-only parse, shared by sng_load_snapshot and sng_snapshot_probe.
ParsedSnapshot parse_snapshot(const std::string& path) {
    ParsedSnapshot ps;
    std::vector<uint8_t> raw = inflate_all(path);
    ps.root = MsgpackParser(raw.data(), raw.size()).parse();
    const JValue& root = ps.root;
    if (!root.contains("snapshot")) throw SngError(SNG_ERR_IO, "not a snapshot");
    const JValue& snap = root["snapshot"];
    if (!snap.contains("version") || snap["version"].as_num() < 1) throw SngError(SNG_ERR_IO, "Snapshot uses an old format and can not be loaded.");
    if (!root.contains("encoding")) throw SngError(SNG_ERR_IO, "snapshot has no encoding config");
    const JValue& enc = root["encoding"];
    sng_nerf_config& cfg = ps.cfg;
    cfg.n_levels = (uint32_t)enc["n_levels"].as_num();
    cfg.n_features_per_level = enc.contains("n_features_per_level") ? (uint32_t)enc["n_features_per_level"].as_num() : 2u;
    cfg.log2_hashmap_size = enc.contains("log2_hashmap_size") ? (uint32_t)enc["log2_hashmap_size"].as_num() : 15u;
    cfg.base_resolution = (uint32_t)enc["base_resolution"].as_num();
    cfg.per_level_scale = enc["per_level_scale"].as_float();
    cfg.aabb_scale = (uint32_t)snap["nerf"]["aabb_scale"].as_num();
    const JValue& pb = snap["params_binary"];
    std::string ptype = snap.contains("params_type") ? snap["params_type"].as_str() : std::string("__half");
    if (ptype == "__half") {
        ps.params.resize(pb.str.size() / 2);
        std::memcpy(ps.params.data(), pb.str.data(), ps.params.size() * 2);
    } else if (ptype == "float") {
        std::vector<float> fp(pb.str.size() / 4);
        std::memcpy(fp.data(), pb.str.data(), fp.size() * 4);
        for (float v : fp) ps.params.push_back(f2h_host(v));
    } else throw SngError(SNG_ERR_IO, "unsupported params_type " + ptype);
    if (snap.contains("density_grid_binary")) {
        const JValue& dg = snap["density_grid_binary"];
        ps.grid.resize(dg.str.size() / 2);
        std::memcpy(ps.grid.data(), dg.str.data(), ps.grid.size() * 2);
    }
    return ps;
}

// The optimizer state of a snapshot saved with include_optimizer_state (save_snapshot below; tcnn
// Trainer::deserialize): Adam moments and per-parameter steps, EMA weights, the step counter and the
// batch counters.  With snapshot.sng (this library's extension) also the fp32 master weights, the fp32
// density grid and the pcg32 states, so training resumes exactly; without it the master weights are
// the fp16 params and the grid the fp16 density grid (what a reference snapshot carries).
// whether the snapshot's optimizer block has every key and size restore_training_state reads (the tcnn key
// names are restated, not pinned; a block written by another tcnn version must not break a render-only load)
bool training_state_usable(const sng_ctx* c, const JValue& snap, std::string& why) {
    const uint64_t n = c->n_params;
    const uint64_t n_cells = (uint64_t)GRID_CELLS * (c->max_cascade + 1);
    auto bin_ok = [&](const JValue& parent, const char* key, uint64_t bytes) {
        if (!parent.contains(key)) { why = std::string("missing ") + key; return false; }
        const JValue& v = parent[key];
        if (v.type != JValue::Binary || v.str.size() != bytes) { why = std::string(key) + " has the wrong type or size"; return false; }
        return true;
    };
    const JValue& opt = snap["optimizer"];
    if (opt.type != JValue::Object) { why = "optimizer is not a map"; return false; }
    if (!bin_ok(opt, "weights_ema_binary", n * 4)) return false;
    if (!opt.contains("nested") || !opt["nested"].contains("nested")) { why = "missing optimizer.nested.nested (Adam)"; return false; }
    const JValue& adam = opt["nested"]["nested"];
    if (!bin_ok(adam, "first_moments_binary", n * 4) || !bin_ok(adam, "second_moments_binary", n * 4) || !bin_ok(adam, "param_steps_binary", n * 4))
        return false;
    if (!adam.contains("current_step") || adam["current_step"].type == JValue::Binary) { why = "missing current_step"; return false; }
    if (snap.contains("sng")) {
        const JValue& x = snap["sng"];
        if (!bin_ok(x, "master_binary", n * 4) || !bin_ok(x, "density_grid_f32_binary", n_cells * 4) || !bin_ok(x, "rng_binary", 32)) return false;
        if (!x.contains("grid_ema_step")) { why = "missing sng.grid_ema_step"; return false; }
    }
    return true;
}

void restore_training_state(sng_ctx* c, const JValue& snap) {
    const uint64_t n = c->n_params;
    const uint32_t n_cells = GRID_CELLS * (c->max_cascade + 1);
    auto bin = [](const JValue& v, size_t bytes) -> const void* {
        if (v.type != JValue::Binary || v.str.size() != bytes) throw SngError(SNG_ERR_IO, "snapshot optimizer state has the wrong size");
        return v.str.data();
    };
    const JValue& opt = snap["optimizer"];
    const JValue& adam = opt["nested"]["nested"];
    train_reset(c, 1337);   // allocations; master = ema = float(params), zero moments
    auto& t = c->tr;
    HIPCHK(hipMemcpy(t.ema.p, bin(opt["weights_ema_binary"], n * 4), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.m1.p, bin(adam["first_moments_binary"], n * 4), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.m2.p, bin(adam["second_moments_binary"], n * 4), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.steps.p, bin(adam["param_steps_binary"], n * 4), n * 4, hipMemcpyHostToDevice));
    t.step = (uint32_t)adam["current_step"].as_num();
    if (snap.contains("nerf") && snap["nerf"].contains("rgb")) {
        const JValue& r = snap["nerf"]["rgb"];
        t.rays_per_batch = (uint32_t)r["rays_per_batch"].as_num();
        t.measured = (uint32_t)r["measured_batch_size"].as_num();
        t.measured_before = (uint32_t)r["measured_batch_size_before_compaction"].as_num();
    }
    if (snap.contains("loss")) t.last_loss = snap["loss"].as_float();
    std::vector<float> master(n), grid(n_cells);
    if (snap.contains("sng")) {
        const JValue& x = snap["sng"];
        std::memcpy(master.data(), bin(x["master_binary"], n * 4), n * 4);
        std::memcpy(grid.data(), bin(x["density_grid_f32_binary"], (size_t)n_cells * 4), (size_t)n_cells * 4);
        uint64_t rng[4];
        std::memcpy(rng, bin(x["rng_binary"], sizeof(rng)), sizeof(rng));
        t.rng.state = rng[0]; t.rng.inc = rng[1]; t.grid_rng.state = rng[2]; t.grid_rng.inc = rng[3];
        t.grid_ema_step = (uint32_t)x["grid_ema_step"].as_num();
    } else {
        HIPCHK(hipMemcpy(master.data(), t.master.p, n * 4, hipMemcpyDeviceToHost));
        const std::vector<uint16_t> g16 = download<uint16_t>(c->d_grid_f16, n_cells);
        for (uint32_t i = 0; i < n_cells; ++i) grid[i] = h2f(g16[i]);
        t.grid_ema_step = t.step;
    }
    std::vector<uint16_t> p_train(n);
    for (uint64_t i = 0; i < n; ++i) p_train[i] = f2h_host(master[i]);
    HIPCHK(hipMemcpy(t.master.p, master.data(), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.p_train.p, p_train.data(), n * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.p_infer.p, c->d_params.p, n * 2, hipMemcpyDeviceToDevice));
    HIPCHK(hipMemcpy(t.grid.p, grid.data(), (size_t)n_cells * 4, hipMemcpyHostToDevice));
    // the training marcher's bitfield and density mean from the f32 grid (train_density_update's tail)
    HIPCHK(hipMemcpy(c->d_grid_f32.p, t.grid.p, (size_t)n_cells * 4, hipMemcpyDeviceToDevice));
    launch_bitfield(nullptr, c->max_cascade, c->d_grid_f32.as<float>(), c->d_partial.as<double>(), c->d_mean.as<float>(), c->d_bitfield.as<uint8_t>(),
                    c->d_occ_linear.as<uint32_t>(), c->s_nerf);
    build_occ_brick(c, c->s_nerf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->s_nerf));
    c->has_bitfield = true;
}

// from_json(Lens) (json_binding.h:65-95)
Lens lens_from_json(const JValue& j) {
    Lens l{};
    auto num = [&](const char* k) { return j[k].as_float(); };
    if (j.contains("k1")) {
        if (j.contains("is_fisheye") && j["is_fisheye"].as_bool()) {
            l.mode = LENS_OPENCV_FISHEYE;
            l.params[0] = num("k1"); l.params[1] = num("k2"); l.params[2] = num("k3"); l.params[3] = num("k4");
        } else {
            l.mode = LENS_OPENCV;
            l.params[0] = num("k1"); l.params[1] = num("k2"); l.params[2] = num("p1"); l.params[3] = num("p2");
        }
    } else if (j.contains("ftheta_p0")) {
        l.mode = LENS_FTHETA;
        const char* kf[7] = {"ftheta_p0", "ftheta_p1", "ftheta_p2", "ftheta_p3", "ftheta_p4", "w", "h"};
        for (int i = 0; i < 7; ++i) l.params[i] = num(kf[i]);
    } else if (j.contains("latlong")) {
        l.mode = LENS_LATLONG;
    } else if (j.contains("equirectangular")) {
        l.mode = LENS_EQUIRECTANGULAR;
    }
    return l;
}

void load_snapshot(sng_ctx* c, const std::string& path) {
    ParsedSnapshot ps = parse_snapshot(path);
    const JValue& snap = ps.root["snapshot"];
    set_model(c, &ps.cfg, ps.params.data(), ps.params.size());
    if (!ps.grid.empty()) set_density_grid(c, ps.grid.data(), ps.grid.size());
    if (snap.contains("nerf") && snap["nerf"].contains("dataset")) {
        const JValue& ds = snap["nerf"]["dataset"];
        if (ds.contains("scale")) c->ds_scale = ds["scale"].as_num();
        if (ds.contains("offset")) c->ds_offset = mk(ds["offset"][0].as_float(), ds["offset"][1].as_float(), ds["offset"][2].as_float());
        // load_nerf_post: render_lens = metadata[0].lens (testbed_nerf.cu:3051-3052; NerfDataset from_json reads the global
        // "lens" default, then the image's own, json_binding.h:141-160); render_with_lens_distortion is left as it is
        c->render_lens = Lens{};
        // the legacy key "camera_distortion" overrides "lens" at both levels, as in from_json(NerfDataset)
        if (ds.contains("lens")) c->render_lens = lens_from_json(ds["lens"]);
        if (ds.contains("camera_distortion")) c->render_lens = lens_from_json(ds["camera_distortion"]);
        if (ds.contains("metadata") && ds["metadata"].size() > 0) {
            const JValue& m0 = ds["metadata"][0];
            if (m0.contains("lens")) c->render_lens = lens_from_json(m0["lens"]);
            if (m0.contains("camera_distortion")) c->render_lens = lens_from_json(m0["camera_distortion"]);
        }
    }
    if (snap.contains("up_dir")) c->up = mk(snap["up_dir"][0].as_float(), snap["up_dir"][1].as_float(), snap["up_dir"][2].as_float());
    if (snap.contains("camera")) {
        const JValue& cam = snap["camera"];
        if (cam.contains("matrix")) read_mat43(cam["matrix"], c->cam);
        if (cam.contains("fov_axis")) c->fov_axis = (int)cam["fov_axis"].as_num();
        if (cam.contains("relative_focal_length")) {
            const JValue& r = cam["relative_focal_length"];
            if (r.type == JValue::Array) { c->rel_focal[0] = r[0].as_float(); c->rel_focal[1] = r[1].as_float(); }
            else c->rel_focal[0] = c->rel_focal[1] = r.as_float();
        }
        if (cam.contains("screen_center")) { c->screen_center[0] = cam["screen_center"][0].as_float(); c->screen_center[1] = cam["screen_center"][1].as_float(); }
        if (cam.contains("zoom")) c->zoom = cam["zoom"].as_float();
        if (cam.contains("scale")) c->m_scale = cam["scale"].as_float();
    }
    if (snap.contains("exposure")) c->params["exposure"] = snap["exposure"].as_num();
    // the optimizer chain's state (include_optimizer_state): restored for training when every key and size is
    // as written; otherwise the inference model stays loaded and the training state is not touched
    // (optimizer_state_loaded: 1 restored, 0 skipped or malformed, -1 none in the file)
    c->params["optimizer_state_loaded"] = -1.0;
    if (snap.contains("optimizer")) {
        std::string why;
        if (c->p("load_optimizer_state") != 0.0 && training_state_usable(c, snap, why)) {
            restore_training_state(c, snap);
            c->params["optimizer_state_loaded"] = 1.0;
        } else {
            c->params["optimizer_state_loaded"] = 0.0;
            if (!why.empty()) std::fprintf(stderr, "sng_load_snapshot: optimizer state not restored (%s); inference model loaded\n", why.c_str());
        }
    }
}

// ---- Testbed::save_snapshot (testbed.cu:4812-4876) ------------------------------------------------
// m_network_config (base.json, with the model's encoding) + "snapshot": tcnn Trainer::serialize (n_params,
// params_type, params_binary = the inference (EMA) params; with include_optimizer_state the optimizer
// chain Ema -> ExponentialDecay -> Adam: weights_ema / first_moments / second_moments / param_steps /
// current_step [tcnn, unvendored: key names restated from its source, parity unpinned]) and the Testbed
// fields the reference writes.  Extension (ignored by the reference's loader): snapshot.sng holds what an
// exact resume needs beyond those -- the fp32 master weights, the fp32 density grid and both pcg32 states.
// .ingp: gzip-wrapped deflate (zstr::ostream; Z_NO_COMPRESSION when compress = 0); else plain msgpack.
void put_vec3(MsgpackWriter& w, f3 v) { const float a[3] = {v.x, v.y, v.z}; w.nums(a, 3); }
void put_mat43(MsgpackWriter& w, const float m[12]) {   // tcnn mat json: an array of the 4 columns
    w.arr(4);
    for (int i = 0; i < 4; ++i) w.nums(m + 3 * i, 3);
}
void put_aabb(MsgpackWriter& w, const aabb& b) { w.map(2); w.key("min"); put_vec3(w, b.lo); w.key("max"); put_vec3(w, b.hi); }
// to_json(Lens) (json_binding.h:37-63)
void put_lens(MsgpackWriter& w, const Lens& l) {
    const char* k4[4] = {"k1", "k2", l.mode == LENS_OPENCV_FISHEYE ? "k3" : "p1", l.mode == LENS_OPENCV_FISHEYE ? "k4" : "p2"};
    if (l.mode == LENS_OPENCV || l.mode == LENS_OPENCV_FISHEYE) {
        w.map(5);
        w.key("is_fisheye"); w.boolean(l.mode == LENS_OPENCV_FISHEYE);
        for (int i = 0; i < 4; ++i) { w.key(k4[i]); w.num(l.params[i]); }
    } else if (l.mode == LENS_FTHETA) {
        const char* kf[7] = {"ftheta_p0", "ftheta_p1", "ftheta_p2", "ftheta_p3", "ftheta_p4", "w", "h"};
        w.map(7);
        for (int i = 0; i < 7; ++i) { w.key(kf[i]); w.num(l.params[i]); }
    } else if (l.mode == LENS_LATLONG) {
        w.map(1); w.key("latlong"); w.boolean(true);
    } else if (l.mode == LENS_EQUIRECTANGULAR) {
        w.map(1); w.key("equirectangular"); w.boolean(true);
    } else {
        w.map(0);
    }
}
void put_network_config(MsgpackWriter& w, const sng_nerf_config& g) {
    w.key("loss"); w.map(1); w.key("otype"); w.str("Huber");
    w.key("optimizer"); w.map(3); w.key("otype"); w.str("Ema"); w.key("decay"); w.num(0.95);
    w.key("nested"); w.map(5); w.key("otype"); w.str("ExponentialDecay"); w.key("decay_start"); w.uint(20000); w.key("decay_interval"); w.uint(10000);
    w.key("decay_base"); w.num(0.33);
    w.key("nested"); w.map(6); w.key("otype"); w.str("Adam"); w.key("learning_rate"); w.num(1e-2); w.key("beta1"); w.num(0.9); w.key("beta2"); w.num(0.99);
    w.key("epsilon"); w.num(1e-15); w.key("l2_reg"); w.num(1e-6);
    w.key("encoding"); w.map(6); w.key("otype"); w.str("HashGrid"); w.key("n_levels"); w.uint(g.n_levels); w.key("n_features_per_level"); w.uint(g.n_features_per_level);
    w.key("log2_hashmap_size"); w.uint(g.log2_hashmap_size); w.key("base_resolution"); w.uint(g.base_resolution);
    w.key("per_level_scale"); w.num(g.per_level_scale);   // testbed.cu:3740 writes it back into the config
    for (const char* name : {"network", "rgb_network"}) {
        w.key(name); w.map(5); w.key("otype"); w.str("FullyFusedMLP"); w.key("activation"); w.str("ReLU"); w.key("output_activation"); w.str("None");
        w.key("n_neurons"); w.uint(64); w.key("n_hidden_layers"); w.uint(name[0] == 'n' ? 1 : 2);
    }
    w.key("dir_encoding"); w.map(2); w.key("otype"); w.str("Composite");
    w.key("nested"); w.arr(2); w.map(3); w.key("n_dims_to_encode"); w.uint(3); w.key("otype"); w.str("SphericalHarmonics"); w.key("degree"); w.uint(4);
    w.map(1); w.key("otype"); w.str("Identity");
}
void save_snapshot(sng_ctx* c, const std::string& path, bool include_opt, bool compress) {
    if (!c->has_model) throw SngError(SNG_ERR_STATE, "no model to save");
    HIPCHK(hipStreamSynchronize(c->s_nerf));
    const uint64_t n = c->n_params;
    auto& t = c->tr;
    const uint32_t n_cells = GRID_CELLS * (c->max_cascade + 1);
    const std::vector<uint16_t> params = download<uint16_t>(c->d_params, n);
    // m_nerf.density_grid (f32) -> fp16: the trained grid when training ran, else the loaded one
    std::vector<float> grid32;
    std::vector<uint16_t> grid16(n_cells, 0);
    if (t.ready && t.grid.p) {
        grid32 = download<float>(t.grid, n_cells);
        for (uint32_t i = 0; i < n_cells; ++i) grid16[i] = f2h_host(grid32[i]);
    } else if (c->has_bitfield && c->d_grid_f16.p) {
        grid16 = download<uint16_t>(c->d_grid_f16, n_cells);
    }
    const bool opt = include_opt && t.ready;
    MsgpackWriter w;
    w.map(7);
    put_network_config(w, c->cfg);
    w.key("snapshot");
    w.map(opt ? 21 : 19);
    w.key("n_params"); w.uint(n);
    w.key("params_type"); w.str("__half");
    w.key("params_binary"); w.bin(params.data(), n * 2);
    if (opt) {
        const std::vector<float> ema = download<float>(t.ema, n), m1 = download<float>(t.m1, n), m2 = download<float>(t.m2, n);
        const std::vector<uint32_t> ps = download<uint32_t>(t.steps, n);
        w.key("optimizer"); w.map(2);
        w.key("weights_ema_binary"); w.bin(ema.data(), n * 4);
        w.key("nested"); w.map(1); w.key("nested"); w.map(5);
        w.key("current_step"); w.uint(t.step);
        w.key("base_learning_rate"); w.num(1e-2);
        w.key("first_moments_binary"); w.bin(m1.data(), n * 4);
        w.key("second_moments_binary"); w.bin(m2.data(), n * 4);
        w.key("param_steps_binary"); w.bin(ps.data(), n * 4);
        const std::vector<float> master = download<float>(t.master, n);
        w.key("sng"); w.map(5);
        w.key("master_binary"); w.bin(master.data(), n * 4);
        w.key("density_grid_f32_binary"); w.bin(grid32.data(), grid32.size() * 4);
        const uint64_t rng[4] = {t.rng.state, t.rng.inc, t.grid_rng.state, t.grid_rng.inc};
        w.key("rng_binary"); w.bin(rng, sizeof(rng));
        w.key("grid_ema_step"); w.uint(t.grid_ema_step);
        w.key("loss_scalar"); w.num(t.last_loss);
    }
    w.key("version"); w.uint(1);   // SNAPSHOT_FORMAT_VERSION
    w.key("mode"); w.str("Nerf");
    w.key("density_grid_size"); w.uint(GRID_SIZE);
    w.key("density_grid_binary"); w.bin(grid16.data(), grid16.size() * 2);
    const float ident[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    w.key("nerf"); w.map(6);
    w.key("aabb_scale"); w.uint(c->cfg.aabb_scale);
    w.key("cam_pos_offset"); w.arr(0);
    w.key("cam_rot_offset"); w.arr(0);
    w.key("extra_dims_opt"); w.arr(0);
    w.key("rgb"); w.map(3);
    w.key("rays_per_batch"); w.uint(t.rays_per_batch);
    w.key("measured_batch_size"); w.uint(t.measured);
    w.key("measured_batch_size_before_compaction"); w.uint(t.measured_before);
    w.key("dataset");
    {   // NerfDataset to_json (json_binding.h:108-132); images are not part of a snapshot
        const int ni = t.n_images;
        std::vector<float> xf = ni ? download<float>(t.xforms, (size_t)ni * 12) : std::vector<float>();
        std::vector<float> fo = ni ? download<float>(t.focal, (size_t)ni * 2) : std::vector<float>();
        std::vector<float> pp = ni ? download<float>(t.pp, (size_t)ni * 2) : std::vector<float>();
        w.map(ni ? 15 : 13);
        w.key("n_images"); w.uint((uint64_t)ni);
        w.key("paths"); w.arr((uint32_t)ni); for (int i = 0; i < ni; ++i) w.str("");
        if (ni) {
            w.key("metadata"); w.arr((uint32_t)ni);
            for (int i = 0; i < ni; ++i) {
                w.map(5);
                w.key("focal_length"); w.nums(&fo[2 * i], 2);
                w.key("lens"); put_lens(w, t.h_lens.empty() ? Lens{} : t.h_lens[i]);
                w.key("principal_point"); w.nums(&pp[2 * i], 2);
                const float rs[4] = {0, 0, 0, 0};
                w.key("rolling_shutter"); w.nums(rs, 4);
                w.key("resolution"); w.arr(2); w.uint((uint64_t)t.w); w.uint((uint64_t)t.h);
            }
            w.key("xforms"); w.arr((uint32_t)ni);
            for (int i = 0; i < ni; ++i) { w.map(2); w.key("start"); put_mat43(w, &xf[12 * i]); w.key("end"); put_mat43(w, &xf[12 * i]); }
        }
        w.key("render_aabb"); put_aabb(w, c->box);
        w.key("render_aabb_to_local"); w.arr(3); for (int i = 0; i < 3; ++i) w.nums(ident + 3 * i, 3);
        w.key("up"); put_vec3(w, c->up);
        w.key("offset"); put_vec3(w, c->ds_offset);
        w.key("envmap_resolution"); w.arr(2); w.uint(0); w.uint(0);
        w.key("scale"); w.num(c->ds_scale);
        w.key("aabb_scale"); w.uint(c->cfg.aabb_scale);
        w.key("from_mitsuba"); w.boolean(false);
        w.key("is_hdr"); w.boolean(false);
        w.key("wants_importance_sampling"); w.boolean(true);
        w.key("n_extra_learnable_dims"); w.uint(0);
    }
    w.key("training_step"); w.uint(t.step);
    w.key("loss"); w.num(t.last_loss);
    w.key("aabb"); put_aabb(w, c->box);
    w.key("bounding_radius"); w.num(1.0);
    w.key("render_aabb_to_local"); w.arr(3); for (int i = 0; i < 3; ++i) w.nums(ident + 3 * i, 3);
    w.key("render_aabb"); put_aabb(w, c->box);
    w.key("up_dir"); put_vec3(w, c->up);
    w.key("sun_dir"); put_vec3(w, normalize(mk(1.0f, 1.0f, 1.0f)));
    w.key("exposure"); w.num(c->p("exposure"));
    const float bg[4] = {0, 0, 0, 0};
    w.key("background_color"); w.nums(bg, 4);
    w.key("camera"); w.map(10);
    w.key("matrix"); put_mat43(w, c->cam);
    w.key("fov_axis"); w.sint(c->fov_axis);
    w.key("relative_focal_length"); w.nums(c->rel_focal, 2);
    w.key("screen_center"); w.nums(c->screen_center, 2);
    w.key("zoom"); w.num(c->zoom);
    w.key("scale"); w.num(c->m_scale);
    w.key("aperture_size"); w.num(0.0);
    w.key("autofocus"); w.boolean(false);
    const float af[3] = {0.5f, 0.5f, 0.5f};
    w.key("autofocus_target"); w.nums(af, 3);
    w.key("autofocus_depth"); w.num(0.0);
    std::ofstream f(path, std::ios::binary);
    if (!f) throw SngError(SNG_ERR_IO, "cannot write '" + path + "'");
    const bool ingp = path.size() >= 5 && path.substr(path.size() - 5) == ".ingp";
    if (!ingp) {
        f.write(reinterpret_cast<const char*>(w.out.data()), (std::streamsize)w.out.size());
    } else {
        z_stream zs{};
        if (deflateInit2(&zs, compress ? Z_DEFAULT_COMPRESSION : Z_NO_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK)
            throw SngError(SNG_ERR_IO, "zlib init failed");
        std::vector<uint8_t> buf(1 << 20);
        zs.next_in = w.out.data();
        zs.avail_in = (uInt)w.out.size();
        int r;
        do {
            zs.next_out = buf.data();
            zs.avail_out = (uInt)buf.size();
            r = deflate(&zs, Z_FINISH);
            if (r == Z_STREAM_ERROR) { deflateEnd(&zs); throw SngError(SNG_ERR_IO, "zlib deflate failed"); }
            f.write(reinterpret_cast<const char*>(buf.data()), (std::streamsize)(buf.size() - zs.avail_out));
        } while (r != Z_STREAM_END);
        deflateEnd(&zs);
    }
    if (!f) throw SngError(SNG_ERR_IO, "write failed '" + path + "'");
}

}  // namespace sng_host
