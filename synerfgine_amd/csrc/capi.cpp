// capi.cpp -- host runtime (C++) behind the C-ABI in include/sng.h.
//
// Mirrors the reference's host objects on the hot path:
//   Testbed   : model/snapshot, density bitfield, camera (testbed.cu:405-425, 3562, 4133-4140, 4878-5015)
//   NerfTracer: the device-driven wavefront loop (testbed_nerf.cu:2128-2277)
//   RayTracer : mesh rays, path tracing, overlay (synerfgine/raytracer.cu:260-392)
//   Engine    : scene JSON, rendering.* keys, resize and frame (synerfgine/engine.cu:21-433)
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

namespace {

thread_local std::string g_err;

#define HIPCHK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) throw SngError(SNG_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

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

const std::map<std::string, double>& default_params() {
    static const std::map<std::string, double> d = {
        {"res_factor", 64},                     // Testbed::m_fixed_res_factor (testbed.h:656)
        {"vo_scale", 4},                        // Engine::m_relative_vo_scale (engine.cuh:113)
        {"exposure", 0.0},                      // Testbed::m_exposure
        {"tonemap_curve", 0},                   // Testbed::m_tonemap_curve (engine.cu:406): 0 Identity, 1 ACES, 2 Hable, 3 Reinhard
        {"rt_buffer_type", 0},                  // RayTracer::m_buffer_to_show (raytracer.cuh:20,179): 0 Final, 1 NextOrigin, 2 SrcOrigin,
                                                //   3 NextDirection, 4 SrcDirection, 5 Normal, 6 Depth, 7 NerfShadow
        {"path_trace_depth", 2},                // RayTracer::m_ray_iters (raytracer.cuh:160)
        {"light_samples", 2},                   // RayTracer::m_samples
        {"syn_shadow_samples", 4},              // RayTracer::m_shadow_iters
        {"syn_shadow_intensity", 1.0},          // RayTracer::m_syn_shadow_factor
        {"attenuation", 1.0},                   // RayTracer::m_attenuation_coeff (unused by raytrace)
        {"lens_size", 0.009},                   // RayTracer::m_lens_angle_constant
        {"depth_offset", 0.1},                  // RayTracer::m_depth_offset (overlay z-test)
        {"n_steps", 8},                         // RayTracer::m_n_steps (NeRF shadow steps on meshes)
        {"nerf_shadow_samples", 1},             // Testbed::sng_position_kernel_size (testbed.h:686)
        {"nerf_shadow_intensity", 2.0},         // Engine::m_nerf_shadow_intensity (engine.cuh:117)
        {"nerf_ao_intensity", 2.0},             // Engine::m_nerf_ao_intensity
        {"nerf_on_nerf_shadow_threshold", 0.3}, // Engine::m_nerf_self_shadow_threshold
        {"shadow_on_nerf", 1},                  // Engine::m_view_syn_shadow
        {"shadow_on_virtual_obj", 1},           // RayTracer::m_view_nerf_shadow
        {"show_virtual_obj", 1},                // RayTracer::m_show_virtual_obj
        {"show_nerf", 1},                       // Engine::m_show_nerf
        {"min_transmittance", 0.01},            // render_min_transmittance (testbed.h:867)
        {"srgb", 1},                            // EColorSpace::SRGB passed to overlay (engine.cu:406)
        {"smooth_threshold", 1.0},              // sng_position_kernel_threshold (unused by the path)
        {"max_shadow_variance", 0.0},           // sng_shadow_depth_variance (unused by the path)
        {"concurrent_streams", 1},              // 1: raytracer and NeRF streams overlap (engine.cu:386-405 run them back to back)
        {"rt_start_chunk", 0},                  // concurrent mode: 0 the raytracer starts at frame start beside init_rays; k > 0 its path
                                                //   kernel waits for the head's network launch (the first speculative round's, or the
                                                //   wavefront's of chunk k); -1: 1 for bands of >= 60 % of the rows, else 0.  C3 A/B
                                                //   (round 5, 4 alternating pairs): 0 -> 295-298 frames/s, 1 -> 271-272 (the path kernel,
                                                //   the frame's critical path, idles ~0.3 ms behind init_rays + generate + network)
        {"rt_reserved_cus", 32},                // concurrent mode: CUs (4 per XCD) the persistent raytracer grids leave to the NeRF stream
        {"linear_marcher", 1},                  // exact unit-cube fast path of the occupancy march
        {"occ_lin_all", 1},                     // cascaded marchers read every cascade's occupancy from x-fastest rows (same bits, no Morton code)
        {"fast_slab", 1},                       // exact reciprocal-multiply BVH box tests
        {"rt_wavefront", 1},                    // deferred shadow-ray queues for the path tracer
        {"bvh_wide", 1},                        // traversal layout with both child boxes per record (exact)
        {"bvh_flat", 1},                        // BvhWide walk keeping the nearer child in a register (exact)
        {"rt_tile", 8},                         // path-kernel tile width: 8 (8x8 pixels per wave) or 4 (4x4, shorter chains)
        {"rt_tile_h", 0},                       // path-kernel tile height: 0 = rt_tile; 4 with rt_tile 8: 8x4 (32 lanes per wave)
        {"scene_lds", 1},                       // BVH nodes + triangles staged in LDS per workgroup when they fit
        {"rt_tile_order", 1},                   // visit raytracer tiles in descending previous-frame cost
        {"rt_prio_frac", 0.1},                  // the costliest fraction of the path tiles (last frame's order) at wave priority 3
        {"rt_prio2_frac", 0.25},                // ... the tiles up to this fraction of the order at priority 2
        {"rt_first", 1},                        // concurrent frames: init_rays waits (device-side, bounded) for the path kernel's first workgroup
        {"rt_first_timeout_us", 100},           // ... at most this long
        {"rt_fused_shadow", 1},                 // banded frames: the path kernel's idle waves trace the shadow rays (mesh.hip fq_consume)
        {"rt_fused_tiles_per_wave", 1},         // ... when the band has at most this many path tiles per wave (a full queue is traced in place)
        {"rt_fused_shadow_used", 0},            // (output) 1 when the last frame's path kernel traced its shadow rays itself
        {"rt_spread", 1},
        {"rt_rng", 0},                          // 1: a measurement mode, NOT the reference's RNG order -- each (pixel, sample) its own XORWOW
                                                //   subsequence, a pixel's samples traced on adjacent lanes (raytrace_sp_kernel); same
                                                //   expectation, other noise (tests/test_gpu_rt_rng.py); for the band-scaling question                       // the path kernel's first tiles dealt across all CUs (costliest one per CU / SIMD)
        {"nerf_gbuffer", 0},                    // 1: NeRF normals every frame (otherwise only when shadow_on_nerf needs them)
        {"rt_plist", 1},                        // per-pixel hit-record lists for the colour replay (rt_accumulate_kernel)
        {"glow_mode", 0},                       // Testbed::Nerf::glow_mode (testbed.h:871): bits 1 green grid, 2 cut line, 4 mask to alpha,
                                                // 8 radial, 16 grid mode -- instant-NGP path only (testbed_nerf.cu:638-734)
        {"glow_y_cutoff", 0},                   // Testbed::Nerf::glow_y_cutoff (testbed.h:870)
        {"render_mode", 1},                     // ERenderMode of the instant-NGP path (sng_render_nerf_ngp): Shade
        {"visualized_layer", 0},                // Testbed::m_visualized_layer (testbed.h:1024)
        {"visualized_dimension", -1},           // Testbed::m_visualized_dimension (testbed.h:1023); > -1 selects EncodingVis (testbed_nerf.cu:2491)
        {"train_grid_est", 0},                  // > 0: the per-ray training kernels' grid sized for this many rays (tests of their grid-stride loops)
        {"train_overlap", 1},                   // the next step's generate on a second stream beside this step's gradients / optimizer
        {"train_overlap_tail", 0},              // tests: sng_train also generates the next step ahead, for the parity hook
        {"train_grid_morton", 1},               // density-grid update: the uniform samples in the Morton order of their cells (same samples, same grid)
        {"train_gen_bricks", 0},                // training generator's occupancy: 0 the linear words (measured fastest, tools/train_ab.py), 1 the OccBrick blob (LDS when it fits, else global)
        {"train_grid_grad_f16", 1},             // hash-grid gradients in fp16 with packed atomics, tcnn's grad_t (__half2 atomicAdd); 0: f32
        {"train_grid_density_only", 1},         // density-grid update: the density MLP alone (NerfNetwork::density), not the full network
        {"train_dw_pipe", 1},                   // dW kernel: the next tile's operands in flight during the current tile's MFMAs (0: load, then multiply)
        {"train_dw_blocks_per_cu", 2},          // dW kernel: workgroups per CU (tools/train_ab.py)
        {"train_gen_lanes", 8},                 // lanes per ray of the training generator's speculative march (8 or 16; 1: one lane per ray; tools/train_ab.py)
        {"train_kernel_times", 0},              // 1: sng_train times the stages of every step with HIP events (sng_train_stats.ms_*)
        {"render_with_lens_distortion", 0},     // Testbed::Nerf::render_with_lens_distortion (testbed_nerf.cu:2504): NeRF rays through
                                                //   render_lens (sng_set_render_lens; the snapshot dataset's first lens)
        {"depth_scale", 1.0},                   // 1 / dataset.scale (testbed_nerf.cu:2748)
        {"rt_queue_gb", 48},                    // device-memory budget for the deferred-shadow queues
        {"train_batch", 262144},                // m_training_batch_size (testbed.h:1103)
        {"train_random_bg", 1},                 // m_nerf.training.random_bg_color (testbed.h:790)
        {"train_debug", 0},                     // parity hook: generate writes per-ray step counts (sng_train_debug)
        {"nerf_fused", 1},                      // ray-local fused NeRF kernel for the tail iterations (fused.hip)
        {"nerf_fused_after", 0},                // ... after this many whole-GPU wavefront iterations (0: the speculative tail
                                                //   from the first iteration, queued ahead of its device check; C2 1311 -> 1483
                                                //   frames/s against 1, C3 unchanged)
        {"nerf_spec_rounds", 2},                // speculative tail rounds before the fused kernel finishes the stragglers (nerf.hip)
        {"nerf_spec_budget", 16777216},         // samples one round may generate (K = clamp(budget / (8 n_alive), 1, kmax)); the
                                                //   sample buffers are sized for it (16.8 M x 60 B ~ 1 GB of the 288 GB)
        {"nerf_spec_hint", 1},                  // a ray looks ahead as far as its pixel's ray lived last frame (exact; 0: opacity policy)
        {"nerf_spec_hint_any_view", 0},         // 1: read the hints whatever view wrote them (tests: exact for any hint)
        {"nerf_spec_kmax", 16},                 // iterations one round marches ahead (<= 16)
        {"nerf_spec_k_policy", 1},              // per-ray look-ahead from the ray's opacity in all rounds but the last (exact)
        {"nerf_spec_prepare", 1},               // sample-parallel activations before the spec compositor (exact; 0: in the chain)
        {"occ_lds_kb", 64},                     // LDS budget for the occupancy bricks in the linear marchers (0: global loads)
        {"load_optimizer_state", 1},            // sng_load_snapshot restores a snapshot's optimizer state (0: inference model only)
        {"optimizer_state_loaded", -1},         // set by sng_load_snapshot: 1 restored, 0 skipped / malformed, -1 none in the file
        {"nerf_fused_lanes", 64},               // rays per wave in the fused kernel
        {"nerf_fused_blocks", -1},              // workgroup cap of the fused kernel (0: 2 per CU; -1: 2 per reserved CU when concurrent)
        {"nerf_gen_blocks", -1},                 // generate grid (256-thread units): 0 = min(rays, 8 per CU); -1 = all rays in one trip
        {"rt_shadow_all_cus", 1},               // shadow-ray kernel on every CU: the NeRF tail has mostly finished by then (C3 +2 %; 0: the path kernel grid)
        {"rt_count", 0},                        // count BVH queries / box / triangle tests of the deferred raytracer (sng_rt_counters); 2: wave iterations
        {"nerf_msr", 1},                        // multi-step speculative rounds while n_steps is 2..7 (nerf.hip msr_*; exact)
        {"nerf_msr_budget", 16777216},          // samples one such round may generate (K = clamp(budget / (S n_alive), 1, kmax))
        {"nerf_msr_kmax", 16},                  // iterations one such round marches ahead (<= 16)
        {"nerf_msr_span", -1},                  // rounds follow the last frame's schedule across step changes (1), not (0), -1: on banded frames
        {"march_log", 0},                       // diagnostics: log {alive, steps, samples} of every iteration (sng_frame_buffer "march_log")
        {"nerf_onestep", 1},                    // trace_alt's one-step regime (n_alive > target / 2) ray-local and speculative (fused.hip)
        {"nerf_onestep_horizon", 2048},         // iterations one speculative segment of the regime spans
    };
    return d;
}

}  // namespace

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
    DevBuf rt_rec, rt_lc, rt_srec, rt_mask, rt_head, rt_count, rt_work;   // deferred-shadow raytracer queues
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

namespace {

void upload(DevBuf& b, const void* src, size_t n) {
    b.ensure(n);
    if (n) HIPCHK(hipMemcpy(b.p, src, n, hipMemcpyHostToDevice));
}

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

void build_occ_brick(sng_ctx* c, hipStream_t s);
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
            const uint32_t rounds = (uint32_t)std::max(0.0, c->p("nerf_spec_rounds"));
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
                    sa.in = rb[p]; sa.out = rb[p ^ 1]; sa.p = p;
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
                c->rt_count.ensure(16);
                q.rec = c->rt_rec.as<float4>(); q.lc = c->rt_lc.as<float4>(); q.srec = c->rt_srec.as<float4>(); q.mask = c->rt_mask.as<float>();
                q.head = c->rt_head.as<int>(); q.count = c->rt_count.as<uint32_t>(); q.cap = (uint32_t)cap;
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
// ================================================================================================
// Online training (BASELINE config 5): Testbed::train_nerf + training_prep_nerf on train.hip
// ================================================================================================
TrainImages train_images(sng_ctx* c) {
    auto& t = c->tr;
    return {t.pixels.as<uint32_t>(), t.xforms.as<float>(), t.xforms_ray.as<float>(), t.focal.as<float>(), t.pp.as<float>(),
            t.h_lens.empty() ? nullptr : t.lens.as<Lens>(), t.w, t.h, t.n_images};
}

// Testbed::reset_network's training state: fp32 master weights from the current model, zeroed
// optimizer moments, m_rng = pcg32(seed), density_grid_rng = pcg32(m_rng.next_uint()) (testbed.cu:3654-3667)
// a step generated ahead on s_gen (train_overlap_tail) is discarded: wait for its kernels, then the next step generates
// its own samples from the current state
static void train_drop_pregen(sng_ctx::Train& t) {
    if (t.pregen) { HIPCHK(hipStreamSynchronize(t.s_gen)); t.pregen = false; }
}

void train_reset(sng_ctx* c, uint64_t seed) {
    if (!c->has_model) throw SngError(SNG_ERR_STATE, "set or load a model before training");
    auto& t = c->tr;
    const uint64_t n = c->n_params;
    t.master.ensure(n * 4); t.grads.ensure(n * 4); t.m1.ensure(n * 4); t.m2.ensure(n * 4); t.steps.ensure(n * 4); t.ema.ensure(n * 4);
    t.p_train.ensure(n * 2); t.p_infer.ensure(n * 2);
    t.wfrag_train.ensure(20 * 512 * 2); t.wfrag_t.ensure(36 * 256 * 2);
    std::vector<uint16_t> h(n);
    HIPCHK(hipMemcpy(h.data(), c->d_params.p, n * 2, hipMemcpyDeviceToHost));
    std::vector<float> f(n);
    for (uint64_t i = 0; i < n; ++i) f[i] = h2f(h[i]);
    HIPCHK(hipMemcpy(t.master.p, f.data(), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.ema.p, f.data(), n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.p_train.p, h.data(), n * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t.p_infer.p, h.data(), n * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(t.m1.p, 0, n * 4)); HIPCHK(hipMemset(t.m2.p, 0, n * 4)); HIPCHK(hipMemset(t.steps.p, 0, n * 4));
    const uint32_t n_cells = GRID_CELLS * (c->max_cascade + 1);
    t.grid.ensure((size_t)n_cells * 4); t.grid_tmp.ensure((size_t)n_cells * 4);
    HIPCHK(hipMemset(t.grid.p, 0, (size_t)n_cells * 4));
    t.rng = Pcg32::seeded(seed);
    t.grid_rng = Pcg32::seeded(t.rng.next_uint());
    t.step = 0; t.grid_ema_step = 0; t.rays_per_batch = 1u << 12; t.measured = 0; t.measured_before = 0;
    t.sched.ensure(sizeof(TrainSched));
    t.sched_dirty = true;
    train_drop_pregen(t);   // a step generated ahead belongs to the old run
    t.target = (uint32_t)c->p("train_batch");
    const uint32_t target = t.target, max_samples = target * 16;
    t.ctrl.ensure(sizeof(TrainCtrl));
    const size_t max_rays = 1u << 18;   // rays_per_batch is capped at 2^18 (update_after_training)
    t.ray_indices.ensure(max_rays * 4); t.rays.ensure(max_rays * 32); t.numsteps.ensure(max_rays * 8);
    t.coords.ensure((size_t)max_samples * 28); t.mlp_out.ensure((size_t)max_samples * 8);
    t.coords_c.ensure((size_t)target * 28); t.dloss.ensure((size_t)target * 8); t.loss.ensure(max_rays * 4);
    t.acts.ensure((size_t)((target + 15) / 16) * TRAIN_FEATS * 16 * 2);
    t.partial.ensure((size_t)max_samples * 16); t.rayrec.ensure(max_rays * 48);
    t.cnt_i.ensure(max_rays * 4); t.cbase_i.ensure(max_rays * 4);
    t.tscr.ensure(max_rays * NERF_STEPS * 4);   // strided by the device's ray count, which the host does not wait for
    if (!t.h_sched) HIPCHK(hipHostMalloc((void**)&t.h_sched, 2 * sizeof(TrainSched), hipHostMallocDefault));
    for (hipEvent_t& e : t.sched_ev)
        if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // the bitfield the training marcher reads (density grid -> bitfield after every update)
    c->d_grid_f32.ensure((size_t)n_cells * 4);
    c->d_partial.ensure(1024 * sizeof(double));
    c->d_mean.ensure(sizeof(float));
    c->d_bitfield.ensure((size_t)GRID_CELLS / 8 * N_CASCADES);
    c->d_occ_linear.ensure((size_t)GRID_CELLS / 8 * N_CASCADES);   // every cascade (Volume::occ_lin_all)
    t.ready = true;
}

NetworkDev train_net(sng_ctx* c, const DevBuf& params, const DevBuf& wfrag) {
    NetworkDev n = c->net;
    n.wfrag = wfrag.p;
    n.grid = static_cast<uint16_t*>(params.p) + 3072 + 7168;
    return n;
}

// update_density_grid_nerf (testbed_nerf.cu:3121-3210) + update_density_grid_mean_and_bitfield
void train_density_update(sng_ctx* c, hipStream_t s) {
    auto& t = c->tr;
    const uint32_t n_casc = c->max_cascade + 1, n_cells = GRID_CELLS * n_casc;
    if (t.step == 0) {
        t.grid_ema_step = 0;
        launch_train_mark_untrained(n_cells, t.grid.as<float>(), train_images(c), 1, s);
    }
    const uint32_t n_uni = t.step < 256 ? n_cells : n_cells / 4, n_non = t.step < 256 ? 0 : n_cells / 4;
    const uint32_t n_tot = n_uni + n_non;
    t.grid_coords.ensure((size_t)n_tot * 28); t.grid_idx.ensure((size_t)n_tot * 4); t.grid_out.ensure((size_t)n_tot * 8);
    HIPCHK(hipMemsetAsync(t.grid_tmp.p, 0, (size_t)n_cells * 4, s));
    const int morton = c->p("train_grid_morton") != 0.0 ? 1 : 0;
    launch_train_grid_samples(n_uni, t.grid_rng, t.grid_ema_step, c->box, t.grid.as<float>(), t.grid_coords.as<float>(), t.grid_idx.as<uint32_t>(), n_casc, -0.01f,
                              morton, s);
    t.grid_rng.advance();
    launch_train_grid_samples(n_non, t.grid_rng, t.grid_ema_step, c->box, t.grid.as<float>(), t.grid_coords.as<float>() + (size_t)n_uni * 7,
                              t.grid_idx.as<uint32_t>() + n_uni, n_casc, NERF_MIN_OPTICAL_THICKNESS, morton, s);
    t.grid_rng.advance();
    // density of the training parameters (m_nerf_network->density, use_inference_params = false)
    launch_train_pack(t.p_train.as<uint16_t>(), t.wfrag_train.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), s);
    launch_network(train_net(c, t.p_train, t.wfrag_train), t.grid_coords.as<float>(), 7, n_tot, nullptr, t.grid_out.as<uint16_t>(),
                   c->p("train_grid_density_only") != 0.0 ? 2 : 1, 0, s);
    launch_train_grid_splat_ema(n_tot, t.grid_idx.as<uint32_t>(), t.grid_out.as<uint16_t>(), t.grid_tmp.as<float>(), n_cells, 0.95f, t.grid.as<float>(), s);
    ++t.grid_ema_step;
    HIPCHK(hipMemcpyAsync(c->d_grid_f32.p, t.grid.p, (size_t)n_cells * 4, hipMemcpyDeviceToDevice, s));
    launch_bitfield(nullptr, c->max_cascade, c->d_grid_f32.as<float>(), c->d_partial.as<double>(), c->d_mean.as<float>(), c->d_bitfield.as<uint8_t>(),
                    c->d_occ_linear.as<uint32_t>(), s);
    build_occ_brick(c, s);
    c->has_bitfield = true;
}

TrainStepArgs train_args(sng_ctx* c) {
    auto& t = c->tr;
    TrainStepArgs a{};
    a.vol = make_volume(c);
    a.sched = t.sched.as<TrainSched>();
    a.n_rays_grid = std::min(t.n_rays_est + t.n_rays_est / 4, 1u << 18);   // a lagged estimate plus room for its growth
    if (c->p("train_grid_est") > 0.0) a.n_rays_grid = (uint32_t)c->p("train_grid_est");   // tests: force the kernels' grid-stride trips
    a.target_batch = t.target;
    a.random_bg = c->p("train_random_bg") != 0.0 ? 1 : 0;
    a.background = mk(0.0f, 0.0f, 0.0f);
    a.loss_scale = 128.0f;   // default_loss_scale<__half>
    a.near_distance = 0.1f;
    a.debug = c->p("train_debug") != 0.0 ? 1 : 0;
    a.gen_bricks = c->p("train_gen_bricks") != 0.0 ? 1 : 0;
    a.gen_lanes = (int)c->p("train_gen_lanes");
    a.dw_pipe = c->p("train_dw_pipe") != 0.0 ? 1 : 0;
    a.dw_blocks_per_cu = std::max(1, (int)c->p("train_dw_blocks_per_cu"));
    a.grid_grad_f16 = c->p("train_grid_grad_f16") != 0.0 && c->net.F == 4 ? 1 : 0;
    return a;
}

TrainBatch train_batch(sng_ctx* c) {
    auto& t = c->tr;
    return {t.ctrl.as<TrainCtrl>(), t.ray_indices.as<uint32_t>(), t.rays.as<float4>(), t.numsteps.as<uint2>(), t.coords.as<float>(), t.mlp_out.as<uint16_t>(),
            t.coords_c.as<float>(), t.dloss.as<uint16_t>(), t.loss.as<float>(), t.acts.as<uint16_t>(), t.partial.as<float4>(), t.rayrec.as<float4>(),
            t.cnt_i.as<uint32_t>(), t.cbase_i.as<uint32_t>()};
}

// train_nerf_step (3532-3780) up to the gradients; stage > 0 stops early (parity hooks):
// 1 = samples generated, 2 = network outputs, 3 = loss / compaction, 4 = gradients
// ev (train_kernel_times): 8 events bracketing generate | network | loss | gradient clear | field | dW (the optimizer's
// event is recorded by train_steps)
void train_sched_push(sng_ctx* c, hipStream_t s) {
    auto& t = c->tr;
    if (t.sched_dirty) {   // host-set batch sizes (reset, snapshot load): train_args' max_inference from measured_before
        const uint32_t cap = t.target * 16;
        const TrainSched h{t.rays_per_batch,
                           t.measured_before == 0 ? cap : (std::min(t.measured_before, cap) + BATCH_SIZE_GRANULARITY - 1) / BATCH_SIZE_GRANULARITY * BATCH_SIZE_GRANULARITY,
                           t.measured, t.measured_before};
        HIPCHK(hipMemcpyAsync(t.sched.p, &h, sizeof(h), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));   // h is a stack value
        t.n_rays_est = t.rays_per_batch;
        t.sched_dirty = false;
    }
}

// the step's first stage: the per-ray buffers cleared, the samples generated (rng: the step's stream)
void train_generate_stage(sng_ctx* c, const Pcg32& rng, hipStream_t s) {
    auto& t = c->tr;
    const TrainStepArgs a = train_args(c);
    const TrainBatch b = train_batch(c);
    launch_train_clear(a, b, s);   // also zeroes the batch counters (TrainCtrl)
    launch_train_generate(a, train_images(c), b, rng, t.tscr.as<float>(), s);
}

// generated: the step's samples were queued ahead on the generator stream (train_steps); ev_loss: recorded after the
// loss stage (the next step's generate may start from there)
void train_forward_backward(sng_ctx* c, int stage, hipStream_t s, hipEvent_t* ev = nullptr, bool generated = false, hipEvent_t ev_loss = nullptr) {
    auto& t = c->tr;
    train_sched_push(c, s);
    const TrainStepArgs a = train_args(c);
    const TrainBatch b = train_batch(c);
    const TrainImages im = train_images(c);
    auto mark = [&](int k) { if (ev) HIPCHK(hipEventRecord(ev[k], s)); };
    if (!generated) {
        launch_train_clear(a, b, s);   // also zeroes the batch counters (TrainCtrl)
        mark(0);
        launch_train_generate(a, im, b, t.rng, t.tscr.as<float>(), s);
        mark(1);
    }
    if (stage == 1) return;
    // inference forward of every sample with the training params
    // with the network's count = min(numsteps_counter, max_samples): the generator drops rays beyond max_samples
    launch_train_pack(t.p_train.as<uint16_t>(), t.wfrag_train.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), s, &b.ctrl->numsteps_counter, a.sched,
                      t.ctrl.as<uint32_t>() + 3);
    const NetworkDev net = train_net(c, t.p_train, t.wfrag_train);
    launch_network(net, b.coords, 7, 0, t.ctrl.as<uint32_t>() + 3, b.mlp_out, 1, (t.target * 16 + 15) / 16, s);
    mark(2);
    if (stage == 2) return;
    launch_train_loss(a, im, b, t.rng, c->d_mean.as<float>(), stage == 0 ? t.sched.as<TrainSched>() : nullptr, s);
    if (ev_loss) HIPCHK(hipEventRecord(ev_loss, s));
    mark(3);
    if (stage == 3) return;
    const uint64_t n_mlp = 3072 + 7168;
    t.grads_h_used = a.grid_grad_f16 != 0;
    if (t.grads_h_used) {   // f32 MLP gradients + fp16 grid gradients (tcnn's grad_t)
        t.grads_h.ensure((c->n_params - n_mlp) * 2);
        HIPCHK(hipMemsetAsync(t.grads.p, 0, n_mlp * 4, s));
        HIPCHK(hipMemsetAsync(t.grads_h.p, 0, (c->n_params - n_mlp) * 2, s));
    } else {
        HIPCHK(hipMemsetAsync(t.grads.p, 0, c->n_params * 4, s));
    }
    mark(4);
    float* g = t.grads.as<float>();
    launch_train_field(a, b, net, t.wfrag_train.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), static_cast<uint16_t*>(net.grid), g + n_mlp,
                       t.grads_h_used ? t.grads_h.as<uint16_t>() : nullptr, s);
    mark(5);
    launch_train_dw(a, b.acts, g, (uint32_t)c->n_cus, s);
    mark(6);
}

void train_steps(sng_ctx* c, uint32_t n_steps, sng_train_stats* out) {
    if (!c->tr.ready) train_reset(c, 1337);
    auto& t = c->tr;
    if (t.n_images == 0) throw SngError(SNG_ERR_STATE, "no training images (sng_train_set_dataset)");
    hipStream_t s = c->s_nerf;
    HIPCHK(hipEventRecord(c->ev_start, s));
    double loss_acc = 0.0;
    // per-stage device times (param train_kernel_times): generate, network, loss, gradient clear, field, dW, optimizer
    const bool timed = c->p("train_kernel_times") != 0.0;
    while (timed && c->train_events.size() < 8) { hipEvent_t e; HIPCHK(hipEventCreate(&e)); c->train_events.push_back(e); }
    double stage_ms[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t timed_steps = 0;
    const bool overlap = !timed && c->p("train_overlap") != 0.0;
    if (overlap && !t.s_gen) {
        HIPCHK(hipStreamCreateWithFlags(&t.s_gen, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&t.ev_gen, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&t.ev_loss, hipEventDisableTiming));
    }
    // a step generated ahead (train_overlap_tail) is used as is, except under per-stage timing: its generate stage would
    // have no events, so it is generated again in the timed step (the same samples: same rng, grid and batch sizes)
    if (timed) train_drop_pregen(t);
    bool generated = t.pregen;
    t.pregen = false;
    train_sched_push(c, s);
    for (uint32_t k = 0; k < n_steps; ++k) {
        // Testbed::train: training_prep_nerf every clamp(step / 16, 1, 16) steps (testbed.cu:4081-4091)
        const uint32_t skip = std::min(16u, std::max(1u, t.step / 16u));
        if (t.step % skip == 0) train_density_update(c, s);   // never on a step generated ahead (below)
        if (generated) HIPCHK(hipStreamWaitEvent(s, t.ev_gen, 0));
        train_forward_backward(c, 0, s, timed ? c->train_events.data() : nullptr, generated, overlap ? t.ev_loss : nullptr);
        generated = false;
        // the next step's samples depend on this step's batch sizes (formed in the loss stage) and on the occupancy
        // grid, not on the parameters: unless a density-grid update comes first, they are generated on a second stream
        // while this step's gradients and optimizer run (train_overlap; not with per-stage timing)
        if (overlap && k + 1 < n_steps) {
            const uint32_t ns = t.step + 1, skip_n = std::min(16u, std::max(1u, ns / 16u));
            if (ns % skip_n != 0) {
                HIPCHK(hipStreamWaitEvent(t.s_gen, t.ev_loss, 0));
                Pcg32 r = t.rng;
                r.advance();
                train_generate_stage(c, r, t.s_gen);
                HIPCHK(hipEventRecord(t.ev_gen, t.s_gen));
                generated = true;
            }
        }
        // optimizer_step: Ema(ExponentialDecay(Adam)) (base.json)
        AdamArgs o{};
        const uint32_t decays = t.step >= 20000 ? (t.step - 20000) / 10000 + 1 : 0;
        o.lr = 1e-2f * std::pow(0.33f, (float)decays);
        o.beta1 = 0.9f; o.beta2 = 0.99f; o.epsilon = 1e-15f; o.l2_reg = 1e-6f; o.loss_scale = 128.0f; o.ema_decay = 0.95f; o.ema_step = t.step;
        o.deb_old = 1.0f - std::pow(o.ema_decay, (float)o.ema_step);
        o.deb_new = 1.0f - std::pow(o.ema_decay, (float)(o.ema_step + 1));
        // per-parameter step counts reach at most t.step + 1 after this update (a larger one forms the factor itself)
        if (t.adam_corr_n < t.step + 1) {
            const uint32_t need = t.step + 1;
            if (t.adam_corr.bytes < (size_t)(need + 1) * 4) {
                t.adam_corr.ensure(((size_t)need + 4096) / 4096 * 4096 * 4);
                t.adam_corr_n = 0;
            }
            // the table's whole capacity at once (one small launch per 4096 steps instead of one per step)
            const uint32_t to = (uint32_t)(t.adam_corr.bytes / 4) - 1;
            launch_train_adam_corr(t.adam_corr.as<float>(), t.adam_corr_n + 1, to, o.beta1, o.beta2, s);
            t.adam_corr_n = to;
        }
        o.corr = t.adam_corr.as<float>();
        o.corr_n = t.adam_corr_n;
        o.grads_h = t.grads_h_used ? t.grads_h.as<uint16_t>() : nullptr;
        launch_train_adam(o, c->n_params, 3072 + 7168, t.master.as<float>(), t.grads.as<float>(), t.m1.as<float>(), t.m2.as<float>(), t.steps.as<uint32_t>(),
                          t.ema.as<float>(), t.p_train.as<uint16_t>(), t.p_infer.as<uint16_t>(), s);
        if (timed) HIPCHK(hipEventRecord(c->train_events[7], s));
        t.rng.advance();
        ++t.step;
        // NerfCounters::update_after_training (3272-3296) ran on the device at the end of the loss stage (train_rollover_kernel):
        // the next step reads its batch sizes from there, so the host queues the steps without waiting for each (the
        // reference syncs on a readback every step)
        // the grid-size estimate follows the device's ray count through the readback slots (correctness never depends
        // on it: the kernels loop over the device count)
        if (t.step % 8 == 0) {
            const uint32_t q = t.sched_slot;
            if (t.sched_pending[q]) {   // issued 16 steps ago: waits only while the host is further ahead than that
                HIPCHK(hipEventSynchronize(t.sched_ev[q]));
                t.n_rays_est = std::max(t.h_sched[q].n_rays, 256u);
            }
            HIPCHK(hipMemcpyAsync(&t.h_sched[q], t.sched.p, sizeof(TrainSched), hipMemcpyDeviceToHost, s));
            HIPCHK(hipEventRecord(t.sched_ev[q], s));
            t.sched_pending[q] = true;
            t.sched_slot ^= 1u;
        }
        if (timed) {   // per-stage times need the step's events: one wait per step in this mode only
            HIPCHK(hipStreamSynchronize(s));
            for (int q = 0; q < 7; ++q) {
                float ms = 0.0f;
                HIPCHK(hipEventElapsedTime(&ms, c->train_events[q], c->train_events[q + 1]));
                stage_ms[q] += ms;
            }
            ++timed_steps;
        }
    }
    HIPCHK(hipEventRecord(c->ev_end, s));
    // inference params (EMA) -> the render path's weights and grid
    launch_train_pack(t.p_infer.as<uint16_t>(), c->d_wfrag.as<uint16_t>(), t.wfrag_t.as<uint16_t>(), s);
    HIPCHK(hipMemcpyAsync(c->d_grid.p, static_cast<uint16_t*>(t.p_infer.p) + 3072 + 7168, (c->n_params - 3072 - 7168) * 2, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d_params.p, t.p_infer.p, c->n_params * 2, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    if (n_steps) {   // the device's batch sizes and the last step's counters back to the host
        TrainSched h{};
        TrainCtrl hc{};
        HIPCHK(hipMemcpy(&h, t.sched.p, sizeof(h), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&hc, t.ctrl.p, sizeof(hc), hipMemcpyDeviceToHost));
        t.rays_per_batch = h.n_rays; t.measured = h.measured; t.measured_before = h.measured_before;
        t.n_rays_est = h.n_rays;
        t.sched_pending[0] = t.sched_pending[1] = false;
        if (out) {
            std::vector<float> l(std::max<uint32_t>(1, hc.ray_counter));
            const uint32_t nr = std::min<uint32_t>(hc.ray_counter, (uint32_t)(t.loss.bytes / 4));
            if (nr) HIPCHK(hipMemcpy(l.data(), t.loss.p, nr * 4, hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < nr; ++i) loss_acc += l[i];
            t.last_loss = (float)(loss_acc * (double)t.measured / (double)t.target);
        }
    }
    if (out) {
        std::memset(out, 0, sizeof(*out));
        out->step = t.step;
        out->loss = t.last_loss;
        out->rays_per_batch = t.rays_per_batch;
        out->measured_batch = t.measured;
        out->measured_batch_before_compaction = t.measured_before;
        HIPCHK(hipEventElapsedTime(&out->ms, c->ev_start, c->ev_end));
        out->timed_steps = timed_steps;
        float* dst[7] = {&out->ms_generate, &out->ms_network, &out->ms_loss, &out->ms_grad_clear, &out->ms_field, &out->ms_dw, &out->ms_optimizer};
        for (int q = 0; q < 7; ++q) *dst[q] = timed_steps ? (float)(stage_ms[q] / timed_steps) : 0.0f;
    }
    // tests (train_overlap_tail): the next step generated ahead as in the loop, for the parity hook to check; queued
    // after the counters above were read back (its generate stage clears the step's control words and losses)
    if (overlap && n_steps && c->p("train_overlap_tail") != 0.0) {
        const uint32_t skip_n = std::min(16u, std::max(1u, t.step / 16u));
        if (t.step % skip_n != 0) {
            HIPCHK(hipStreamWaitEvent(t.s_gen, t.ev_loss, 0));
            train_generate_stage(c, t.rng, t.s_gen);   // t.rng is the next step's stream already
            HIPCHK(hipEventRecord(t.ev_gen, t.s_gen));
            HIPCHK(hipStreamWaitEvent(s, t.ev_gen, 0));
            t.pregen = true;
        }
    }
}

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
                      &c->acc_depth, &c->final_rgba, &c->final_depth, &c->rt_rec, &c->rt_lc, &c->rt_srec, &c->rt_mask, &c->rt_head, &c->rt_plist, &c->rt_pcount, &c->rt_rval, &c->rt_count, &c->rt_work, &c->rt_tile_cost, &c->rt_tile_order, &c->fused_work, &c->rng_nerf, &c->rng_mesh, &c->rng_mesh_sp, &c->d_seq, &c->d_objs, &c->d_lights, &c->d_mats, &c->d_scene_blob,
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
struct ParsedSnapshot {
    sng_nerf_config cfg{};
    std::vector<uint16_t> params, grid;
    JValue root;
};
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
template <typename T>
std::vector<T> download(const DevBuf& b, size_t n) {
    std::vector<T> h(n);
    if (n) HIPCHK(hipMemcpy(h.data(), b.p, n * sizeof(T), hipMemcpyDeviceToHost));
    return h;
}
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

}  // namespace

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
