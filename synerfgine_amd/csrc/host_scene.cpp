// host_scene.cpp -- virtual objects and scene description: OBJ loading and the triangle BVH build
// (triangle_bvh.cu), the traversal layout, the scene JSON (Engine::set_virtual_world, engine.cu:21-78, and its
// rendering.* keys), the camera (testbed.cu:405-425) and animation (engine.cu:80-127, 365-372).
#include "host.h"

namespace sng_host {

// ---- OBJ (tinyobj::LoadObj subset: v + polygon faces, fan-triangulated) ----------
std::vector<Tri> load_obj(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw SngError(SNG_ERR_IO, "Error loading file: " + path);
    std::vector<f3> verts;
    std::vector<Tri> tris;
    std::string line;
    while (std::getline(f, line)) {
        if (line.size() < 2) continue;
        if (line[0] == 'v' && line[1] == ' ') {
            std::istringstream ss(line.substr(2));
            float x, y, z;
            ss >> x >> y >> z;
            verts.push_back({x, y, z});
        } else if (line[0] == 'f' && line[1] == ' ') {
            std::istringstream ss(line.substr(2));
            std::string tok;
            std::vector<int> idx;
            while (ss >> tok) {
                int vi = std::stoi(tok.substr(0, tok.find('/')));
                idx.push_back(vi > 0 ? vi - 1 : (int)verts.size() + vi);
            }
            for (size_t k = 1; k + 1 < idx.size(); ++k) tris.push_back({verts.at(idx[0]), verts.at(idx[k]), verts.at(idx[k + 1])});
        }
    }
    return tris;
}

// ---- TriangleBvhWithBranchingFactor<2>::build (triangle_bvh.cu:615-692) ----------
std::vector<BvhNode> build_bvh(std::vector<Tri>& tris, uint32_t ppl) {
    struct BB { f3 lo, hi; };
    auto bb_of = [](std::vector<Tri>::iterator b, std::vector<Tri>::iterator e) {
        BB bb{b->a, b->a};
        auto grow = [&](f3 p) {
            bb.lo = mk(fminf(bb.lo.x, p.x), fminf(bb.lo.y, p.y), fminf(bb.lo.z, p.z));
            bb.hi = mk(fmaxf(bb.hi.x, p.x), fmaxf(bb.hi.y, p.y), fmaxf(bb.hi.z, p.z));
        };
        for (auto it = b; it != e; ++it) { grow(it->a); grow(it->b); grow(it->c); }
        return bb;
    };
    auto centroid = [](const Tri& t) { return (t.a + t.b + t.c) / 3.0f; };
    auto centroid_axis = [](const Tri& t, int ax) {
        const float* a = &t.a.x; const float* b = &t.b.x; const float* c = &t.c.x;
        return (a[ax] + b[ax] + c[ax]) / 3;
    };
    auto set_bb = [](BvhNode& n, const BB& bb) {
        n.lo[0] = bb.lo.x; n.lo[1] = bb.lo.y; n.lo[2] = bb.lo.z;
        n.hi[0] = bb.hi.x; n.hi[1] = bb.hi.y; n.hi[2] = bb.hi.z;
    };
    std::vector<BvhNode> nodes(1);
    set_bb(nodes[0], bb_of(tris.begin(), tris.end()));
    struct BuildNode { int node_idx; std::vector<Tri>::iterator begin, end; };
    std::stack<BuildNode> st;
    st.push({0, tris.begin(), tris.end()});
    while (!st.empty()) {
        BuildNode curr = st.top();
        st.pop();
        BuildNode ch[2];
        ch[0].begin = curr.begin;
        ch[0].end = curr.end;
        {
            auto& c = ch[0];
            f3 mean = splat(0.0f);
            for (auto it = c.begin; it != c.end; ++it) mean = mean + centroid(*it);
            mean = mean / (float)std::distance(c.begin, c.end);
            f3 var = splat(0.0f);
            for (auto it = c.begin; it != c.end; ++it) { f3 d = centroid(*it) - mean; var = var + d * d; }
            var = var / (float)std::distance(c.begin, c.end);
            float mv = std::max(std::max(var.x, var.y), var.z);
            int axis = var.x == mv ? 0 : (var.y == mv ? 1 : 2);
            auto mid = c.begin + std::distance(c.begin, c.end) / 2;
            std::nth_element(c.begin, mid, c.end, [&](const Tri& a, const Tri& b) { return centroid_axis(a, axis) < centroid_axis(b, axis); });
            ch[1].end = c.end;
            ch[0].end = ch[1].begin = mid;
        }
        nodes[curr.node_idx].left = (int)nodes.size();
        for (int i = 0; i < 2; ++i) {
            ch[i].node_idx = (int)nodes.size();
            nodes.emplace_back();
            set_bb(nodes.back(), bb_of(ch[i].begin, ch[i].end));
            if ((uint32_t)std::distance(ch[i].begin, ch[i].end) <= ppl) {
                nodes.back().left = -(int)std::distance(tris.begin(), ch[i].begin) - 1;
                nodes.back().right = -(int)std::distance(tris.begin(), ch[i].end) - 1;
            } else {
                st.push(ch[i]);
            }
        }
        nodes[curr.node_idx].right = (int)nodes.size();
    }
    return nodes;
}

// glm-style adjugate inverse (tcnn::inverse(mat3)) -- column-major m.c[i] = column i
m3 inverse3(const m3& M) {
    auto e = [&](int i, int j) { const f3& c = i == 0 ? M.c0 : (i == 1 ? M.c1 : M.c2); return j == 0 ? c.x : (j == 1 ? c.y : c.z); };
    float det = e(0, 0) * (e(1, 1) * e(2, 2) - e(2, 1) * e(1, 2)) - e(1, 0) * (e(0, 1) * e(2, 2) - e(2, 1) * e(0, 2)) +
                e(2, 0) * (e(0, 1) * e(1, 2) - e(1, 1) * e(0, 2));
    float r[3][3];
    r[0][0] = +(e(1, 1) * e(2, 2) - e(2, 1) * e(1, 2));
    r[1][0] = -(e(1, 0) * e(2, 2) - e(2, 0) * e(1, 2));
    r[2][0] = +(e(1, 0) * e(2, 1) - e(2, 0) * e(1, 1));
    r[0][1] = -(e(0, 1) * e(2, 2) - e(2, 1) * e(0, 2));
    r[1][1] = +(e(0, 0) * e(2, 2) - e(2, 0) * e(0, 2));
    r[2][1] = -(e(0, 0) * e(2, 1) - e(2, 0) * e(0, 1));
    r[0][2] = +(e(0, 1) * e(1, 2) - e(1, 1) * e(0, 2));
    r[1][2] = -(e(0, 0) * e(1, 2) - e(1, 0) * e(0, 2));
    r[2][2] = +(e(0, 0) * e(1, 1) - e(1, 0) * e(0, 1));
    return {mk(r[0][0] / det, r[0][1] / det, r[0][2] / det), mk(r[1][0] / det, r[1][1] / det, r[1][2] / det),
            mk(r[2][0] / det, r[2][1] / det, r[2][2] / det)};
}

// get_xform_given_rolling_shutter(start == end, t = 0) rotation: glm quat round trip
// (common_device.cuh:361-368) [tcnn quat, unvendored]
m3 rolling_shutter_rotation(const m3& M) {
    const q4 q = quat_from_m3(M);
    return shutter_rotation(q, q, 0.0f);
}

// BvhWide records of the inner nodes of a TriangleBvhNode array (children at left, left + 1).
// Returns false when a leaf range does not fit the reference encoding (the walk then uses nodes).
bool wide_bvh(const std::vector<BvhNode>& nodes, std::vector<BvhWide>& wide, int& root_ref) {
    std::vector<int> id(nodes.size(), -1);
    int n_inner = 0;
    for (size_t i = 0; i < nodes.size(); ++i)
        if (nodes[i].left >= 0) id[i] = n_inner++;
    bool ok = true;
    auto ref_of = [&](int i) -> int {
        const BvhNode& n = nodes[i];
        if (n.left >= 0) return id[i];
        const int b = -n.left - 1, e = -n.right - 1;
        if (b < 0 || e < b || (uint32_t)b >= WIDE_MAX_BEGIN || (uint32_t)(e - b) > WIDE_MAX_COUNT) { ok = false; return 0; }
        if (((uint32_t)b | ((uint32_t)(e - b) << 24)) == 0x7FFFFFFFu) { ok = false; return 0; }   // would collide with WIDE_DONE
        return (int)~((uint32_t)b | ((uint32_t)(e - b) << 24));
    };
    wide.assign(n_inner, BvhWide{});
    for (size_t i = 0; i < nodes.size(); ++i) {
        const BvhNode& n = nodes[i];
        if (n.left < 0) continue;
        if ((size_t)n.left + 1 >= nodes.size()) return false;
        BvhWide& w = wide[id[i]];
        const BvhNode &c0 = nodes[n.left], &c1 = nodes[n.left + 1];
        for (int k = 0; k < 3; ++k) { w.s0[2 * k] = c0.lo[k]; w.s0[2 * k + 1] = c0.hi[k]; w.s1[2 * k] = c1.lo[k]; w.s1[2 * k + 1] = c1.hi[k]; }
        w.ref0 = ref_of(n.left);
        w.ref1 = ref_of(n.left + 1);
    }
    root_ref = nodes.empty() ? 0 : ref_of(0);
    if (!ok) wide.clear();
    return ok;
}
// ---- camera (testbed.cu:405-425) -------------------------------------------------
f3 cam_col(const sng_ctx* c, int i) { return mk(c->cam[3 * i], c->cam[3 * i + 1], c->cam[3 * i + 2]); }
// Every write of camera0 drops an explicit camera1 (sng_set_motion_blur): the reference re-derives
// camera1 from camera0 each frame (testbed.cu:2850), so a blur set for one pose never applies to another.
void set_cam_col(sng_ctx* c, int i, f3 v) {
    c->cam[3 * i] = v.x; c->cam[3 * i + 1] = v.y; c->cam[3 * i + 2] = v.z;
    c->has_cam1 = false;
}
f3 look_at(const sng_ctx* c) { return cam_col(c, 3) + cam_col(c, 2) * c->m_scale; }
void set_look_at(sng_ctx* c, f3 pos) { set_cam_col(c, 3, cam_col(c, 3) + (pos - look_at(c))); }
void set_scale(sng_ctx* c, float scale) {
    f3 prev = look_at(c);
    set_cam_col(c, 3, (cam_col(c, 3) - prev) * (scale / c->m_scale) + prev);
    c->m_scale = scale;
}
void set_view_dir(sng_ctx* c, f3 dir) {
    f3 old = look_at(c);
    f3 c0 = normalize(cross(dir, c->up));
    set_cam_col(c, 0, c0);
    set_cam_col(c, 1, normalize(cross(dir, c0)));
    set_cam_col(c, 2, normalize(dir));
    set_look_at(c, old);
}
float fov_to_focal(float degrees) { return 0.5f * 1.0f / std::tan(0.5f * degrees * 3.14159265358979323846f / 180.0f); }

// ---- scene JSON (Engine::set_virtual_world, engine.cu:21-78; Engine::init keys 148-228) ----
std::string read_file(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    if (!f) throw SngError(SNG_ERR_IO, "JSON File not found: " + p);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}
bool file_exists(const std::string& p) { std::ifstream f(p); return (bool)f; }

// depth of a BVH built by build_bvh (root depth 0)
uint32_t bvh_depth(const std::vector<BvhNode>& nodes) {
    std::vector<uint32_t> d(nodes.size(), 0);
    uint32_t m = 0;
    for (size_t i = 0; i < nodes.size(); ++i)
        if (nodes[i].left >= 0) {
            d[nodes[i].left] = d[nodes[i].left + 1] = d[i] + 1;
            m = std::max(m, d[i] + 1);
        }
    return m;
}

void upload_scene(sng_ctx* c) {
    std::vector<ObjectGpu> og;
    // scene blob: per object [nodes or wide records][traversal triangles], each array 16-B aligned
    std::vector<uint8_t> blob;
    auto append = [&](const void* p, size_t bytes) {
        const size_t off = blob.size();
        blob.resize((off + bytes + 15) / 16 * 16, 0);
        std::memcpy(blob.data() + off, p, bytes);
        return (uint32_t)off;
    };
    c->bvh_depth = 0;
    c->bvh_stack = 0;
    for (auto& o : c->objs) {
        upload(o.d_nodes, o.nodes.data(), o.nodes.size() * sizeof(BvhNode));
        upload(o.d_tris, o.tris.data(), o.tris.size() * sizeof(Tri));
        std::vector<TriT> trit(o.tris.size());
        for (size_t i = 0; i < o.tris.size(); ++i) trit[i] = make_trit(o.tris[i]);
        upload(o.d_trit, trit.data(), trit.size() * sizeof(TriT));
        ObjectGpu g{};
        g.nodes = o.d_nodes.as<BvhNode>();
        g.tris = o.d_tris.as<Tri>();
        g.trit = o.d_trit.as<TriT>();
        g.rot = o.rot;
        g.pos = o.pos;
        g.scale = o.scale;
        g.mat_id = o.mat;
        m3 msc = {mk(1.0f / o.scale, 0.0f / o.scale, 0.0f / o.scale), mk(0.0f / o.scale, 1.0f / o.scale, 0.0f / o.scale),
                  mk(0.0f / o.scale, 0.0f / o.scale, 1.0f / o.scale)};
        g.world_to_obj = mulm(msc, inverse3(o.rot));   // m_scale * m_rotate (triangle_bvh.cu:313-319)
        float max_coord = 0.0f;
        for (const BvhNode& n : o.nodes)
            for (int k = 0; k < 3; ++k) max_coord = std::max(max_coord, std::max(std::fabs(n.lo[k]), std::fabs(n.hi[k])));
        g.fast_slab = (c->p("fast_slab") != 0.0 && max_coord < SLAB_FAST_MAX_COORD) ? 1 : 0;
        const bool wide = c->p("bvh_wide") != 0.0 && wide_bvh(o.nodes, o.wide, o.root_ref);
        if (wide) {
            upload(o.d_wide, o.wide.data(), std::max<size_t>(1, o.wide.size()) * sizeof(BvhWide));
            g.wide = o.d_wide.as<BvhWide>();
            g.lds_wide = append(o.wide.data(), o.wide.size() * sizeof(BvhWide));
            g.root_ref = o.root_ref;
            g.lds_nodes = 0;   // the node array is not needed by the traversal
        } else {
            g.lds_nodes = append(o.nodes.data(), o.nodes.size() * sizeof(BvhNode));
        }
        g.lds_trit = append(trit.data(), trit.size() * sizeof(TriT));
        c->bvh_depth = std::max(c->bvh_depth, bvh_depth(o.nodes));
        c->bvh_stack = std::max(c->bvh_stack, c->bvh_depth + 2u);
        og.push_back(g);
    }
    upload(c->d_objs, og.data(), og.size() * sizeof(ObjectGpu));
    if (blob.empty()) blob.resize(16, 0);
    upload(c->d_scene_blob, blob.data(), blob.size());
    c->scene_f4 = (uint32_t)(blob.size() / 16);
    std::vector<LightGpu> lg;
    for (auto& l : c->lights) lg.push_back({mk(l.pos[0], l.pos[1], l.pos[2]), l.intensity, l.size, l.type});
    upload(c->d_lights, lg.data(), lg.size() * sizeof(LightGpu));
    std::vector<MaterialGpu> mg;
    for (auto& m : c->mats)
        mg.push_back({mk(m.ka[0], m.ka[1], m.ka[2]), mk(m.kd[0], m.kd[1], m.kd[2]), mk(m.ks[0], m.ks[1], m.ks[2]), m.n, m.rg, m.spec_angle, m.type});
    upload(c->d_mats, mg.data(), mg.size() * sizeof(MaterialGpu));
    c->scene_dirty = false;
}

// lights whose shadow term draws a light sample (Light::sample, type 0)
int n_point_lights(const sng_ctx* c) {
    int n = 0;
    for (const auto& l : c->lights) n += l.type == 0 ? 1 : 0;
    return n;
}

// the NeRF shadow pass's mesh queries: the raytracer's scene blob, in LDS when it fits (2 x 512 or 1 x 1024 threads
// per CU with their stacks, 16 waves per CU), else traversed from global memory
void shadow_scene(sng_ctx* c, ShadowArgs& sa) {
    sa.scene_blob = c->d_scene_blob.as<float4>();
    sa.scene_f4 = c->scene_f4;
    sa.stack_depth = std::min<uint32_t>(32u, c->bvh_stack);
    sa.bvh_flat = c->p("bvh_flat") != 0.0 ? 1 : 0;
    const uint64_t blob_b = (uint64_t)c->scene_f4 * 16;
    const bool lds_ok = c->p("scene_lds") != 0.0 && sa.scene_blob != nullptr;
    sa.tpb = 512;
    sa.scene_in_lds = 0;
    if (lds_ok && blob_b + (uint64_t)sa.stack_depth * 512 * 4 <= 80u * 1024u) sa.scene_in_lds = 1;
    else if (lds_ok && blob_b + (uint64_t)sa.stack_depth * 1024 * 4 <= 160u * 1024u) { sa.scene_in_lds = 1; sa.tpb = 1024; }
    sa.blocks = (uint32_t)c->n_cus * (1024u / sa.tpb);
}

void load_scene(sng_ctx* c, const std::string& path) {
    JValue cfg = JsonParser(read_file(path)).parse();
    std::string dir = path.find('/') == std::string::npos ? std::string(".") : path.substr(0, path.find_last_of('/'));
    if (cfg.contains("camera")) {
        const JValue& cc = cfg["camera"];
        f3 view = splat(0.0f), at = splat(0.0f);
        float zoom = 1.0f;
        if (cc.contains("view")) view = mk(cc["view"][0].as_float(), cc["view"][1].as_float(), cc["view"][2].as_float());
        if (cc.contains("at")) at = mk(cc["at"][0].as_float(), cc["at"][1].as_float(), cc["at"][2].as_float());
        if (cc.contains("zoom")) zoom = cc["zoom"].as_float();
        if (cc.contains("vo_scale")) c->params["vo_scale"] = cc["vo_scale"].as_num();
        // Engine::set_virtual_world (engine.cu:43-49): animation_speed, CamPath(cam_conf) (cam_path.cuh:97-115)
        c->anim_speed = 0.0f;
        c->animations = false;
        if (cc.contains("animation_speed")) {
            c->anim_speed = cc["animation_speed"].as_float();
            c->animations = c->anim_speed > 0.0f;
        }
        c->campath = CamPathState{};
        if (cc.contains("path")) {
            CamPathState& cp = c->campath;
            auto key = [](const JValue& f) {
                return CamKeyframe{mk(f["view"][0].as_float(), f["view"][1].as_float(), f["view"][2].as_float()),
                                   mk(f["at"][0].as_float(), f["at"][1].as_float(), f["at"][2].as_float()), f["zoom"].as_float()};
            };
            if (cc.contains("frames"))
                for (size_t i = 0; i < cc["frames"].size(); ++i) cp.keys.push_back(key(cc["frames"][i]));
            if (!cc.contains("total_time_ms")) throw SngError(SNG_ERR_INVALID, "camera path without total_time_ms");
            cp.total_time_ms = (int)cc["total_time_ms"].as_num();
            if (cc.contains("fps")) cp.fps = (int)cc["fps"].as_num();
            cp.total_frames = cp.total_time_ms * cp.fps / 1000;
            if (cc.contains("move_on_start")) cp.playing = cc["move_on_start"].as_num() != 0.0;
            for (size_t i = 0; i < cc["path"].size(); ++i) cp.keys.push_back(key(cc["path"][i]));
            // total_frames / (keyframes - 1); the reference divides by zero in set_to_frame when that is 0
            cp.frames_between = std::max(1, cp.total_frames / std::max((int)cp.keys.size() - 1, 1));
            cp.present = true;
        }
        if (dot(view, view) != 0.0f) {   // Engine::init (engine.cu:148-152)
            set_view_dir(c, view);
            set_look_at(c, at);
            set_scale(c, zoom);
        }
    }
    if (cfg.contains("rendering")) {
        const JValue& r = cfg["rendering"];
        static const char* numeric[] = {"res_factor", "exposure", "smooth_threshold", "path_trace_depth", "light_samples", "nerf_shadow_samples",
                                        "nerf_shadow_intensity", "syn_shadow_samples", "syn_shadow_intensity", "attenuation", "lens_size",
                                        "nerf_on_nerf_shadow_threshold", "max_shadow_variance", "nerf_ao_intensity", "shadow_on_virtual_obj",
                                        "shadow_on_nerf", "show_virtual_obj", "show_nerf", "depth_offset"};
        for (const char* k : numeric)
            if (r.contains(k)) c->params[k] = r[k].as_num();
        if (r.contains("clear_color")) c->clear_color = mk(r["clear_color"][0].as_float(), r["clear_color"][1].as_float(), r["clear_color"][2].as_float());
        if (r.contains("nerf_filter") && r["nerf_filter"].as_str() != "Shade")
            throw SngError(SNG_ERR_INVALID, "nerf_filter '" + r["nerf_filter"].as_str() + "' is not on the accelerated path (Shade only)");
        if (r.contains("syn_filter") && r["syn_filter"].as_str() != "Final")
            throw SngError(SNG_ERR_INVALID, "syn_filter '" + r["syn_filter"].as_str() + "' is not on the accelerated path (Final only)");
    }
    // output (engine.cu:52-65): recording folder, record flag, image budget (img_count or the camera path's frames)
    c->img_count = 0;
    c->record = false;
    c->img_count_max = std::max(1, c->campath.present ? c->campath.total_frames : 0);
    if (cfg.contains("output")) {
        const JValue& oc = cfg["output"];
        if (oc.contains("folder")) {
            c->out_folder = oc["folder"].as_str();
            if (!c->out_folder.empty() && c->out_folder[0] != '/') c->out_folder = dir + "/" + c->out_folder;
        }
        if (oc.contains("img_count")) c->img_count_max = (int)oc["img_count"].as_num();
        if (oc.contains("record")) c->record = oc["record"].as_num() != 0.0;
    }
    std::vector<sng_material> mats;
    for (size_t i = 0; i < cfg["materials"].size(); ++i) {   // Material(id, json) (material.cuh:26-48)
        const JValue& m = cfg["materials"][i];
        sng_material mm{};
        mm.ks[0] = mm.ks[1] = mm.ks[2] = 1.0f;
        const std::string& t = m["type"].as_str();
        for (int k = 0; k < 3; ++k) mm.kd[k] = m["kd"][k].as_float();
        if (m.contains("ka")) for (int k = 0; k < 3; ++k) mm.ka[k] = m["ka"][k].as_float();
        if (m.contains("ks")) for (int k = 0; k < 3; ++k) mm.ks[k] = m["ks"][k].as_float();
        mm.n = m["n"].as_float();
        mm.rg = m.contains("rg") ? m["rg"].as_float() : 0.0f;
        if (t == "lambertian") { mm.type = 0; mm.spec_angle = 0.0f; }
        else if (t == "glossy") { mm.type = 1; mm.spec_angle = m.contains("spec_angle") ? m["spec_angle"].as_float() : 0.001f; }
        else throw SngError(SNG_ERR_INVALID, "Material type " + t + " not supported");
        mats.push_back(mm);
    }
    std::vector<HostObject> objs;
    for (size_t i = 0; i < cfg["objfile"].size(); ++i) {   // VirtualObject(id, json) (virtual_object.cu:7-88)
        const JValue& o = cfg["objfile"][i];
        HostObject ho;
        ho.file = o["file"].as_str();
        std::string fp = ho.file;
        if (!file_exists(fp)) fp = dir + "/" + ho.file;
        ho.scale = o.contains("scale") ? o["scale"].as_float() : 1.0f;
        uint32_t ppl = o.contains("primitives-per-leaf") ? (uint32_t)o["primitives-per-leaf"].as_num() : 4u;
        ho.pos = o.contains("pos") ? mk(o["pos"][0].as_float(), o["pos"][1].as_float(), o["pos"][2].as_float()) : splat(0.0f);
        ho.rot = {mk(1, 0, 0), mk(0, 1, 0), mk(0, 0, 1)};
        if (o.contains("rot")) {
            const JValue& a = o["rot"];
            ho.rot = {mk(a[0].as_float(), a[1].as_float(), a[2].as_float()), mk(a[3].as_float(), a[4].as_float(), a[5].as_float()),
                      mk(a[6].as_float(), a[7].as_float(), a[8].as_float())};
        }
        ho.mat = (int)o["material"].as_num();
        if (o.contains("anim")) {   // virtual_object.cu:27-33
            const JValue& an = o["anim"];
            ho.anim.centre = mk(an["rot_center"][0].as_float(), an["rot_center"][1].as_float(), an["rot_center"][2].as_float());
            ho.anim.axis = mk(an["rot_axis"][0].as_float(), an["rot_axis"][1].as_float(), an["rot_axis"][2].as_float());
            ho.anim.angle = an["rot_angle"].as_float();
        }
        ho.tris = load_obj(fp);
        if (ho.tris.empty()) throw SngError(SNG_ERR_IO, "mesh has no triangles: " + fp);
        ho.nodes = build_bvh(ho.tris, ppl);
        objs.push_back(std::move(ho));
    }
    std::vector<sng_light> lights;
    std::vector<LightAnim> light_anims;
    for (size_t i = 0; i < cfg["lights"].size(); ++i) {   // Light(id, json) (light.cuh:17-37)
        const JValue& l = cfg["lights"][i];
        sng_light ll{};
        for (int k = 0; k < 3; ++k) ll.pos[k] = l["pos"][k].as_float();
        ll.intensity = l["intensity"].as_float();
        ll.size = l["size"].as_float();
        ll.type = 0;
        if (l.contains("type")) {
            const std::string& t = l["type"].as_str();
            if (t == "point") ll.type = 0;
            else if (t == "directional") ll.type = 1;
            else throw SngError(SNG_ERR_INVALID, t + " light not recognized");
        }
        LightAnim la;
        if (l.contains("anim")) {   // light.cuh:31-36
            la.on = true;
            la.start = mk(ll.pos[0], ll.pos[1], ll.pos[2]);
            la.end = mk(l["anim"]["end"][0].as_float(), l["anim"]["end"][1].as_float(), l["anim"]["end"][2].as_float());
            la.step = l["anim"]["step"].as_float();
            la.ratio = 0.0f;
        }
        light_anims.push_back(la);
        lights.push_back(ll);
    }
    for (auto& o : objs)
        if (o.mat < 0 || (size_t)o.mat >= mats.size()) throw SngError(SNG_ERR_INVALID, "object material index out of range");
    for (auto& o : c->objs) { o.d_nodes.release(); o.d_tris.release(); o.d_trit.release(); o.d_wide.release(); }
    c->objs = std::move(objs);
    c->mats = mats;
    c->lights = lights;
    c->light_anim = light_anims;
    c->anim_frames = 0;
    c->scene_dirty = true;
    c->mesh_reset = true;
}

// ---- animation: Engine::frame's m_camera_path.update + update_world_objects (engine.cu:365-372, 80-127) ----
// CamPath::set_to_frame (cam_path.cuh:121-130) + CamKeyframe::interpolate (cam_path.cuh:30-39)
void campath_set_to_frame(sng_ctx* c) {
    CamPathState& cp = c->campath;
    if (cp.keys.size() < 2) return;   // the reference reads keyframes[1] past the end here
    cp.current_keyframe = cp.current_frame / cp.frames_between;
    uint32_t next = (uint32_t)cp.current_keyframe + 1;
    if (next >= cp.keys.size()) {
        cp.current_frame = 0;
        cp.current_keyframe = 0;
        next = 1;
    }
    const CamKeyframe& a = cp.keys[cp.current_keyframe];
    const CamKeyframe& b = cp.keys[next];
    const float k = (float)(cp.current_frame % cp.frames_between) / (float)cp.frames_between;
    const float invk = 1.0f - k;
    set_view_dir(c, invk * a.view + k * b.view);
    set_look_at(c, invk * a.at + k * b.at);
    set_scale(c, invk * a.zoom + k * b.zoom);
}
// Light::next_frame (light.cuh:39-49); lights without "anim" do not move (the reference leaves
// their step uninitialised)
void light_next_frame(sng_light& l, LightAnim& a) {
    if (!a.on || a.step == 0.0f) return;
    float next = a.ratio + a.step;
    if (next > 1.0f || next < 0.0f) {
        a.step = -a.step;
        next = a.ratio + a.step;
    }
    a.ratio = next;
    const f3 p = (1.0f - a.ratio) * a.start + a.ratio * a.end;
    l.pos[0] = p.x; l.pos[1] = p.y; l.pos[2] = p.z;
}
// VirtualObject::next_frame (virtual_object.cuh:53-64), including its rotation matrix as written
// (third column uses ax.z*ax.y) and pos = R_next * (rot * (pos - centre)) + centre
void object_next_frame(HostObject& o, float speed) {
    const ObjAnim& an = o.anim;
    if (an.angle == 0.0f) return;
    const f3 ax = an.axis;
    const float cost = std::cos(an.angle * speed), sint = std::sin(an.angle * speed);
    const m3 R = {mk(cost + ax.x * ax.x * (1.0f - cost), ax.x * ax.y * (1.0f - cost) - ax.z * sint, ax.x * ax.z * (1.0f - cost) + ax.y * sint),
                  mk(ax.x * ax.y * (1.0f - cost) + ax.z * sint, cost + ax.y * ax.y * (1.0f - cost), ax.y * ax.z * (1.0f - cost) - ax.x * sint),
                  mk(ax.z * ax.y * (1.0f - cost) - ax.y * sint, ax.z * ax.y * (1.0f - cost) + ax.x * sint, cost + ax.z * ax.z * (1.0f - cost))};
    o.pos = mul(R, mul(o.rot, o.pos - an.centre)) + an.centre;
}
// one frame of animation, in the reference's order: camera path, then objects, then lights
void animate(sng_ctx* c) {
    if (c->campath.playing) {
        c->campath.current_frame += 1;   // CamPath::advance_frame (cam_path.cuh:132-135)
        campath_set_to_frame(c);
        c->mesh_reset = true;
    }
    if (c->animations) {
        for (auto& o : c->objs) object_next_frame(o, c->anim_speed);
        for (size_t i = 0; i < c->lights.size() && i < c->light_anim.size(); ++i) light_next_frame(c->lights[i], c->light_anim[i]);
        c->scene_dirty = true;
        c->mesh_reset = true;
    }
    ++c->anim_frames;
}

}  // namespace sng_host
