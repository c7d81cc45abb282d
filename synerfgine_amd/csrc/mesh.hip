// mesh.hip -- virtual objects: BVH traversal, path tracer, NeRF shadow pass, overlay, RNG.
//
// Replaces ray_intersect_nodes (triangle_bvh.cu:263-319), sng::depth_test_world /
// depth_test_nerf (synerfgine/common.cu:36-102), shade_with_shadow + shadow_for_px
// (testbed_nerf.cu:1614-1786), sng::init_rays_with_payload_kernel_nerf, shade_object,
// raytrace and overlay_nerf (synerfgine/raytracer.cu:6-258), and init_rand_state
// (synerfgine/common.cu:22-26, cuRAND XORWOW seeding restated).
//
// Arithmetic: this file is compiled with FMA contraction per expression (-ffp-contract=on, Makefile) and the triangle
// test's division is the hardware reciprocal -- the reference's --use_fast_math model (CMakeLists.txt:82: nvcc
// contracts a * b + c and turns x / y into rcp.approx), and the cascaded shadow marches' log / exp are __logf /
// __expf; other divisions and sqrt stay correctly rounded, so every kernel variant here computes the same bits
// (Makefile); the NeRF marcher and its schedule (nerf.hip, fused.hip) are IEEE without contraction.
// The overlay / tonemap, compared bit for bit with the oracle, live in overlay.hip (no contraction).
//
// BVH traversal keeps its 32-entry stack in LDS, interleaved by thread
// ([depth][thread]) so a wave's pushes/pops at equal depth hit 64 distinct
// banks.  Each pixel keeps its own XORWOW stream in SoA registers for the whole
// kernel (one coalesced load/store of 24 B per pixel per frame).
// The cone-stepping log / exp of this file's shadow marches (cascaded scenes) as __logf / __expf, the reference's
// fast-math forms (sng_math.h SNG_STEP_EXPF); A/B builds of the IEEE model define RT_IEEE_TRANSCENDENTALS
#ifndef RT_IEEE_TRANSCENDENTALS
#define SNG_FAST_TRANSCENDENTALS
#endif
#include <algorithm>
#include "sng_internal.h"
#include "sng_math.h"

namespace sng {

// Read-only scene tables (objects, lights) through the constant address space: written by the host before the launch and
// never by a kernel, so a wave-uniform index loads with scalar loads into SGPRs (the scalar cache) instead of a vector
// load and a vmcnt wait on every query -- the compiler cannot prove the global copies unclobbered by the kernels' stores.
template <class T>
__device__ __forceinline__ T const_load(const T* p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(4))) T*)p)[i];
#else
    return p[i];   // (the host pass of this device function: never executed)
#endif
}

constexpr int BVH_STACK = 32;
constexpr int TPB = 128;   // threads per block for the traversal kernels

struct Stack {
    int* base;   // LDS, [depth][thread]
    int stride;  // threads per block
    int n;
    __device__ __forceinline__ void push(int v) { base[n * stride] = v; ++n; }
    __device__ __forceinline__ int pop() { --n; return base[n * stride]; }
};
// The same LDS stack addressed by a moving LDS-typed pointer (no per-access depth x stride multiply,
// and always ds_read / ds_write, never a flat access).
typedef __attribute__((address_space(3))) int lds_int;
struct PStack {
    lds_int* base;
    lds_int* top;    // next free slot
    int stride;
    __device__ __forceinline__ void push(int v) { *top = v; top += stride; }
    __device__ __forceinline__ int pop() { top -= stride; return *top; }
    __device__ __forceinline__ bool empty() const { return top == base; }
};

// Where a traversal finds its stack and the BVH arrays.  LDS = true: every object's nodes and
// triangles were copied once per workgroup into LDS (scene blob, host_scene.cpp upload_scene) and the
// stack is only as deep as the deepest BVH needs (max depth + 2 <= 32, so the reference's
// FixedStack<32> overflow rule can never trigger differently).
// CNT = true (bench's counting frames only, sng_rt_counters): cnt -> this thread's {world queries,
// box tests, triangle tests}; the timed kernels are the CNT = false instantiations (no counting code).
template <bool LDS, bool CNT = false>
struct TraceCtx {
    int* stack;            // this thread's first stack slot
    int stride;
    const char* scene;     // LDS scene blob (LDS = true)
    int flat;              // near child in a register (bvh_walk_near)
    uint32_t* cnt = nullptr;
    int cnt_waves = 0;     // rt_count = 2: cnt[1], cnt[2] count wave iterations of the record / triangle loops instead
    __device__ __forceinline__ const BvhNode* nodes(const ObjectGpu& o) const {
        if constexpr (LDS) return reinterpret_cast<const BvhNode*>(scene + o.lds_nodes);
        else return o.nodes;
    }
    __device__ __forceinline__ const BvhWide* wide(const ObjectGpu& o) const {
        if constexpr (LDS) return reinterpret_cast<const BvhWide*>(scene + o.lds_wide);
        else return o.wide;
    }
    __device__ __forceinline__ const TriT* tris(const ObjectGpu& o) const {
        if constexpr (LDS) return reinterpret_cast<const TriT*>(scene + o.lds_trit);
        else return o.trit;
    }
};

// One BvhWide record: four 16-B loads (ds_read_b128 from the LDS scene blob).  d0, d1: the entry
// distances of its two child boxes, exactly as bvh_box_entry / aabb_entry_fast give them.
template <bool FAST>
__device__ __forceinline__ void wide_visit(const BvhWide* __restrict__ rec, f3 ro, f3 rd, f3 y, float& d0, float& d1, int& ref0, int& ref1) {
    const float4* r = reinterpret_cast<const float4*>(rec);
    const float4 a = r[0], b = r[1], c = r[2], e = r[3];
    if constexpr (FAST) {
        d0 = slab_entry_fast(pf2{a.x, a.y}, pf2{a.z, a.w}, pf2{b.x, b.y}, ro, y);
        d1 = slab_entry_fast(pf2{b.z, b.w}, pf2{c.x, c.y}, pf2{c.z, c.w}, ro, y);
    } else {
        d0 = bvh_box_entry(aabb{mk(a.x, a.z, b.x), mk(a.y, a.w, b.y)}, ro, y);
        d1 = bvh_box_entry(aabb{mk(b.z, c.x, c.z), mk(b.w, c.y, c.w)}, ro, y);
    }
    ref0 = __float_as_int(e.x);
    ref1 = __float_as_int(e.y);
}

// slot per lane with pred set, one atomic per wave
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred, int lane) {
    const unsigned long long mask = __ballot(pred);
    const uint32_t total = (uint32_t)__popcll(mask);
    uint32_t base = 0;
    const int leader = mask ? (int)(__ffsll((long long)mask) - 1) : 0;
    if (total && lane == leader) base = atomicAdd(counter, total);
    base = __shfl(base, leader, 64);
    return base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
}

// one slot per active lane from a device counter, one atomic per wave
__device__ __forceinline__ uint32_t wave_alloc(uint32_t* counter, int lane) {
    const unsigned long long mask = __ballot(1);
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(mask));
    base = __shfl(base, leader, 64);
    return base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
}

// counting frames: the wave's {queries, box tests, triangle tests} into dst[0..2] (one atomic each per wave)
__device__ __forceinline__ void flush_counts(unsigned long long* dst, const uint32_t (&c)[3], int lane) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        unsigned long long v = c[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
        if (lane == 0 && v) atomicAdd(dst + k, v);
    }
}

// Triangle::ray_intersect (triangle.cuh:45-59) fused with the caller's `t < mint` test: t is
// formed first and u, v only when t can win.  The accept set is unchanged: the reference replaces
// a rejected t by FLT_MAX, which never passes `t < mint` (mint <= MAX_DEPTH), and a NaN t fails
// both forms; u, v are evaluated with the reference's expressions and comparisons.
__device__ __forceinline__ bool tri_hit(const TriT* tp, f3 ro, f3 rd, float mint, float& t_out) {
    const float4* p4 = reinterpret_cast<const float4*>(tp);
    const float4 w0 = p4[0], w1 = p4[1], w2 = p4[2];
    const f3 v1v0 = mk(w0.w, w1.x, w1.y), v2v0 = mk(w1.z, w1.w, w2.x), n = mk(w2.y, w2.z, w2.w);
    const f3 rov0 = ro - mk(w0.x, w0.y, w0.z);
    // 1.0f / dot(rd, n) as the reference's --use_fast_math build evaluates it (CMakeLists.txt:82: a division becomes
    // rcp.approx), the hardware reciprocal v_rcp_f32 (1 ulp)
#ifdef RT_TRI_RCP_EXACT   // A/B builds of the IEEE model (Makefile: MESH_EXTRA=... -DRT_TRI_RCP_EXACT)
    const float d = 1.0f / dot(rd, n);
#else
    const float d = __builtin_amdgcn_rcpf(dot(rd, n));
#endif
    const float t = d * -dot(n, rov0);
    if (!(t >= 0.0f && t < mint)) return false;
    const f3 q = cross(rov0, rd);
    const float u = d * -dot(q, v2v0);
    const float v = d * dot(q, v1v0);
    if (u < 0.0f || u > 1.0f || v < 0.0f || (u + v) > 1.0f) return false;
    t_out = t;
    return true;
}

// ray_intersect_nodes_f<2> (triangle_bvh.cu:263-307); returns t, writes triangle index.
// Box tests: bvh_box_entry (sng_math.h), in its branch-free form (aabb_entry_fast) when the ray and
// the object keep every quotient finite; y = inv(rd) once per ray.
template <bool FAST>
__device__ __forceinline__ float bvh_walk(f3 ro, f3 rd, f3 y, const BvhNode* __restrict__ nodes, const TriT* __restrict__ tris, int* stack_lds,
                                          int stride, int& tri_out, float t_max, uint32_t* cnt = nullptr) {
    Stack st{stack_lds, stride, 0};
    st.push(0);
    float mint = t_max;
    int shortest = -1;
    while (st.n > 0) {
        const int idx = st.pop();
        const BvhNode node = nodes[idx];
        if (node.left < 0) {
            const int end = -node.right - 1;
            if (cnt) cnt[2] += (uint32_t)(end + node.left + 1);
            for (int i = -node.left - 1; i < end; ++i) {
                float t;
                if (tri_hit(tris + i, ro, rd, mint, t)) { mint = t; shortest = i; }
            }
        } else {
            const int c0 = node.left, c1 = node.left + 1;
            const BvhNode n0 = nodes[c0], n1 = nodes[c1];
            const aabb b0 = {mk(n0.lo[0], n0.lo[1], n0.lo[2]), mk(n0.hi[0], n0.hi[1], n0.hi[2])};
            const aabb b1 = {mk(n1.lo[0], n1.lo[1], n1.lo[2]), mk(n1.hi[0], n1.hi[1], n1.hi[2])};
            if (cnt) cnt[1] += 2u;
            float d0 = FAST ? aabb_entry_fast(b0, ro, y) : bvh_box_entry(b0, ro, y);
            float d1 = FAST ? aabb_entry_fast(b1, ro, y) : bvh_box_entry(b1, ro, y);
            // sorting_network<2>: descending, so the nearer child is pushed last
            int i0 = c0, i1 = c1;
            if (d0 < d1) { float td = d0; d0 = d1; d1 = td; i0 = c1; i1 = c0; }
            if (d0 < mint) { if (st.n >= BVH_STACK - 1) { /* FixedStack overflow: reference warns */ } else st.push(i0); }
            if (d1 < mint) { if (st.n >= BVH_STACK - 1) { } else st.push(i1); }
        }
    }
    tri_out = shortest;
    return mint;
}
// The same traversal over the BvhWide layout: identical box tests, push order, overflow rule and
// triangle order, so identical results; one record load per inner node, none per leaf.
template <bool FAST>
__device__ __forceinline__ float bvh_walk_wide(f3 ro, f3 rd, f3 y, const BvhWide* __restrict__ wide, const TriT* __restrict__ tris, int root_ref,
                                               int* stack_lds, int stride, int& tri_out, float t_max, uint32_t* cnt = nullptr) {
    Stack st{stack_lds, stride, 0};
    st.push(root_ref);
    float mint = t_max;
    int shortest = -1;
    while (st.n > 0) {
        const int ref = st.pop();
        if (ref < 0) {
            const uint32_t e = ~(uint32_t)ref;
            const int b = (int)(e & (WIDE_MAX_BEGIN - 1u)), end = b + (int)(e >> 24);
            if (cnt) cnt[2] += (uint32_t)(end - b);
            for (int i = b; i < end; ++i) {
                float t;
                if (tri_hit(tris + i, ro, rd, mint, t)) { mint = t; shortest = i; }
            }
        } else {
            if (cnt) cnt[1] += 2u;
            float d0, d1;
            int r0, r1;
            wide_visit<FAST>(wide + ref, ro, rd, y, d0, d1, r0, r1);
            int i0 = r0, i1 = r1;
            if (d0 < d1) { float td = d0; d0 = d1; d1 = td; i0 = r1; i1 = r0; }
            if (d0 < mint) { if (st.n >= BVH_STACK - 1) { } else st.push(i0); }
            if (d1 < mint) { if (st.n >= BVH_STACK - 1) { } else st.push(i1); }
        }
    }
    tri_out = shortest;
    return mint;
}
// The same traversal with the nearer child kept in a register instead of being pushed and popped
// straight away (push far, continue near): one LDS store + load less per inner visit that descends.
// The visiting sequence, `d < mint` culling at push time and triangle order are the reference's, so
// the result is identical.  (The reference's FixedStack<32> overflow rule cannot fire: the stack
// never holds more than max BVH depth + 2 <= 32 entries, host_scene.cpp upload_scene.)
template <bool FAST>
__device__ __forceinline__ float bvh_walk_near(f3 ro, f3 rd, f3 y, const BvhWide* __restrict__ wide, const TriT* __restrict__ tris, int root_ref,
                                               int* stack_lds, int stride, int& tri_out, float t_max, uint32_t* cnt = nullptr, bool cw = false) {
    PStack st{(lds_int*)stack_lds, (lds_int*)stack_lds, stride};
    float mint = t_max;
    int shortest = -1;
    int cur = root_ref;          // next stack entry to process
    while (true) {
        // inner records until this lane holds a leaf or has nothing left (WIDE_DONE)
        while (cur >= 0) {
            if (cnt) cnt[1] += cw ? (uint32_t)((int)__builtin_amdgcn_readfirstlane(__lane_id()) == (int)__lane_id()) : 2u;
            float d0, d1;
            int r0, r1;
            wide_visit<FAST>(wide + cur, ro, rd, y, d0, d1, r0, r1);
            int i0 = r0, i1 = r1;
            if (d0 < d1) { float td = d0; d0 = d1; d1 = td; i0 = r1; i1 = r0; }
            // reference: push(far) if d0 < mint, push(near) if d1 < mint, then pop
            const bool far_in = d0 < mint, near_in = d1 < mint;
            if (near_in) {
                if (far_in) st.push(i0);
                cur = i1;
            } else if (far_in) {
                cur = i0;
            } else {
                cur = st.empty() ? WIDE_DONE : st.pop();
            }
        }
        if (cur == WIDE_DONE) break;
        const uint32_t e = ~(uint32_t)cur;
        const int b = (int)(e & (WIDE_MAX_BEGIN - 1u)), end = b + (int)(e >> 24);
        if (cnt && !cw) cnt[2] += (uint32_t)(end - b);
        for (int i = b; i < end; ++i) {
            if (cnt && cw) cnt[2] += (uint32_t)((int)__builtin_amdgcn_readfirstlane(__lane_id()) == (int)__lane_id());
            float t;
            if (tri_hit(tris + i, ro, rd, mint, t)) { mint = t; shortest = i; }
        }
        if (st.empty()) break;
        cur = st.pop();
    }
    tri_out = shortest;
    return mint;
}

// t_max < MAX_DEPTH culls everything at or beyond t_max (the result is then min(closest, t_max));
// only the shadow kernel uses it, where any value >= full_dist yields the same mask.
template <bool LDS, bool CNT = false>
__device__ __forceinline__ float object_intersect(f3 ro, f3 rd, const ObjectGpu& o, const TraceCtx<LDS, CNT>& cx, int& tri, float t_max = MAX_DEPTH) {
    const f3 oro = mul(o.world_to_obj, ro - o.pos);
    const f3 ord = mul(o.world_to_obj, rd);
    const bool fast = o.fast_slab && slab_fast_ok(oro, ord);
    const f3 y = inv(ord);
    if (o.wide && cx.flat) {
        if (fast) return bvh_walk_near<true>(oro, ord, y, cx.wide(o), cx.tris(o), o.root_ref, cx.stack, cx.stride, tri, t_max, CNT ? cx.cnt : nullptr, CNT && cx.cnt_waves);
        return bvh_walk_near<false>(oro, ord, y, cx.wide(o), cx.tris(o), o.root_ref, cx.stack, cx.stride, tri, t_max, CNT ? cx.cnt : nullptr, CNT && cx.cnt_waves);
    }
    if (o.wide) {
        if (fast) return bvh_walk_wide<true>(oro, ord, y, cx.wide(o), cx.tris(o), o.root_ref, cx.stack, cx.stride, tri, t_max, CNT ? cx.cnt : nullptr);
        return bvh_walk_wide<false>(oro, ord, y, cx.wide(o), cx.tris(o), o.root_ref, cx.stack, cx.stride, tri, t_max, CNT ? cx.cnt : nullptr);
    }
    if (fast) return bvh_walk<true>(oro, ord, y, cx.nodes(o), cx.tris(o), cx.stack, cx.stride, tri, t_max, CNT ? cx.cnt : nullptr);
    return bvh_walk<false>(oro, ord, y, cx.nodes(o), cx.tris(o), cx.stack, cx.stride, tri, t_max, CNT ? cx.cnt : nullptr);
}

// sng::depth_test_world (common.cu:36-48)
template <bool LDS, bool CNT = false>
__device__ float depth_test_world(f3 origin, f3 dir, const ObjectGpu* __restrict__ objs, int n_objs, const TraceCtx<LDS, CNT>& cx, int& out_obj,
                                  float t_max = MAX_DEPTH) {
    float depth = MAX_DEPTH;
    const f3 off = origin + dir * MIN_DEPTH;
    if constexpr (CNT) cx.cnt[0] += 1u;
    for (int c = 0; c < n_objs; ++c) {
        int tri;
        const float t = object_intersect(off, dir, const_load(objs, c), cx, tri, t_max);
        if (t < depth && t > MIN_DEPTH) { out_obj = c; depth = t; }
    }
    return depth;
}

struct Hit {
    f3 pos, normal;
    m3 perturb;
    float t;
    int mat;
};
__device__ __forceinline__ f3 tri_normal(const Tri& t) { return normalize(cross(t.b - t.a, t.c - t.a)); }
// sng::depth_test_world(+HitRecord) (common.cu:50-67)
template <bool LDS, bool CNT = false>
__device__ int depth_test_world_hit(f3 origin, f3 dir, const ObjectGpu* __restrict__ objs, int n_objs, const TraceCtx<LDS, CNT>& cx, Hit& h) {
    const f3 off = origin + dir * MIN_DEPTH;
    if constexpr (CNT) cx.cnt[0] += 1u;
    // only the winner's (object, triangle, t) stay live across the objects' traversals; its record is formed once
    // after them, from the same values as the reference forms it at each improvement (common.cu:58-64)
    int out_obj = -1, out_tri = 0;
    float best = MAX_DEPTH;
    for (int c = 0; c < n_objs; ++c) {
        int tri;
        const float t = object_intersect(off, dir, const_load(objs, c), cx, tri);
        if (t < best && t > MIN_DEPTH) {
            out_obj = c;
            out_tri = tri;
            best = t;
        }
    }
    h.t = best;
    h.normal = splat(0.0f);
    h.mat = -1;
    h.perturb = {mk(1, 0, 0), mk(0, 1, 0), mk(0, 0, 1)};
    if (out_obj >= 0) {
        const ObjectGpu o = n_objs == 1 ? const_load(objs, 0) : objs[out_obj];   // (one object: a uniform index)
        h.mat = o.mat_id;
        const Tri tr = o.tris[out_tri];
        const f3 N = tri_normal(tr);
        h.normal = mul(o.rot, N);
        const f3 T = normalize((tr.a + tr.b + tr.c) / 3.0f - tr.a);   // Triangle::get_perturb_matrix (triangle.cuh:164-170)
        h.perturb = {T, cross(T, N), N};
    }
    h.pos = origin + h.t * dir;
    return out_obj;
}

// sng::depth_test_nerf (common.cu:69-83), with two exact early exits.  The march's distance s never
// decreases, and once s >= full_d at the start of a trip the result is full_d (the next sample or
// exit trip clamps to it, DDA trips in between change nothing), so it returns full_d there.  And a
// caller that only uses min(result, cap) with cap <= full_d lets the walk stop once s >= cap: both
// results are then >= cap.
__device__ float depth_test_nerf(float full_d, uint32_t n_steps, const Volume& vol, f3 src, f3 L, f3 invL, uint32_t min_mip, uint32_t max_mip,
                                 float cap) {
    float s = 0.0f;
    if (vol.linear && vol.bitfield && min_mip == 0 && max_mip == 0 && vol.cone <= 1e-5f) {
        // the same march flattened into one loop (one DDA step or one sample per trip), see generate_kernel
        const f3 hs = half_sign(L);
        uint32_t j = 0;
        while (j < n_steps) {
#ifndef SHADOW_MARCH_NO_EARLY_EXIT   // A/B builds (tools/frame_dump.py): the early exits must not change a bit
            if (s >= cap) return s;
            if (s >= full_d) return full_d;
#endif
            const f3 pos = src + L * s;
            const bool out = s >= MAX_DEPTH || !aabb_contains(vol.render_aabb, to_local(vol, pos));
            if (out || occupied_linear(pos, vol.occ_linear)) {
                if (out) s = MAX_DEPTH;
                if (s >= full_d) { s = full_d; break; }
                s += calc_dt(s, 0.0f);
                ++j;
            } else {
                s = dda_step_linear(s, pos, invL, hs);
            }
        }
        return s;
    }
    // general path, flattened the same way (occ_step: one DDA step or one sample per trip)
    uint32_t j = 0;
    while (j < n_steps) {
#ifndef SHADOW_MARCH_NO_EARLY_EXIT   // A/B builds (tools/frame_dump.py): the early exits must not change a bit
        if (s >= cap) return s;
        if (s >= full_d) return full_d;
#endif
        if (occ_step(s, vol.ss, src, L, invL, min_mip, max_mip, vol)) {
            if (s >= full_d) { s = full_d; break; }
            s += calc_dt(s, vol.ss);
            ++j;
        }
    }
    return s;
}

__device__ __forceinline__ Xorwow load_rng(const uint32_t* __restrict__ st, size_t n, size_t i) {
    return {st[i], st[n + i], st[2 * n + i], st[3 * n + i], st[4 * n + i], st[5 * n + i]};
}
__device__ __forceinline__ void store_rng(uint32_t* __restrict__ st, size_t n, size_t i, const Xorwow& s) {
    st[i] = s.v0; st[n + i] = s.v1; st[2 * n + i] = s.v2; st[3 * n + i] = s.v3; st[4 * n + i] = s.v4; st[5 * n + i] = s.d;
}
// pow(x, n) with the exponents of the render path (the Phong exponent of every reference material, the
// shadow intensities, all small integers): an integer n in [0, 4096] by binary exponentiation (exact for
// n = 0, 1, 2, a few ulps above; the reference's build, --use_fast_math, evaluates __powf =
// exp2(n * log2(x)), which is coarser), otherwise powf.  Every kernel computing the same quantity calls
// it, so the path-tracer variants stay bit-identical to each other.
__device__ __forceinline__ float pow_small_int(float x, float n) {
    if (floorf(n) == n && n >= 0.0f && n <= 4096.0f) {
        uint32_t e = (uint32_t)n;
        float r = 1.0f, b = x;
        while (e) {
            if (e & 1u) r *= b;
            b *= b;
            e >>= 1;
        }
        return r;
    }
    return powf(x, n);
}
// Light::sample(rand_state) (light.cuh:71-77)
__device__ __forceinline__ f3 light_sample(const LightGpu& l, Xorwow& r) {
    const float x = fractf_(curand_uniform(r)), y = fractf_(curand_uniform(r)), z = fractf_(curand_uniform(r));
    return l.pos + mk(x, y, z) * l.size * 1.0f;
}

__device__ __forceinline__ void xorwow_skip(Xorwow& r, uint32_t n) {
#pragma unroll 1
    for (uint32_t j = 0; j < n; ++j) (void)xorwow_next(r);
}

// ---------------------------------------------------------------------------
// shade_with_shadow (testbed_nerf.cu:1702-1786) / shadow_for_px (1614-1700)
// ---------------------------------------------------------------------------
// One neighbour's term of shade_with_shadow: shadow_for_px at (pos, nrm); the k-th point light's sample
// (Light::sample, 3 draws from the pixel's XORWOW state) is lp[k * lp_stride], drawn beforehand in the
// reference's order by shadow_draw_kernel.
template <bool LDS>
__device__ __forceinline__ float shadow_term(const ShadowArgs& a, const TraceCtx<LDS, false>& cx, f3 pos, f3 nrm, const float4* __restrict__ lp,
                                             size_t lp_stride) {
    float overall = 1.0f;
    int k = 0;
    for (int li = 0; li < a.n_lights; ++li) {
        const LightGpu L = const_load(a.lights, li);
        if (L.type == 0) {
            const float4 l4 = lp[(size_t)k++ * lp_stride];
            const f3 lpos = mk(l4.x, l4.y, l4.z);
            const f3 l = normalize(lpos - pos);
            const float full_d = length(lpos - pos);
            int hit = -1;
            // with a non-negative intensity a depth >= full_d gives pow(>= 1) >= 1 = no change to `overall`, so the
            // query is culled at full_d (the closest hit nearer than that is found as before; none: full_d)
            const float syn_depth = depth_test_world(pos, l, a.objs, a.n_objs, cx, hit, a.intensity >= 0.0f ? full_d : MAX_DEPTH);
            overall = fminf(overall, pow_small_int(syn_depth / full_d, a.intensity));
            const f3 fract_offset = full_d * a.threshold * lpos;
            const f3 src = pos + fract_offset;
            const float fd = length(lpos - src);
            const f3 Ld = normalize(lpos - src);
            const float k1 = 1.0f - fminf(L.intensity, 0.0f);
            const double k2 = (double)full_d * (1.0 - (double)a.threshold);
            // the march matters only while its mask stays below `overall`: the mask is non-decreasing in the march
            // distance, so the walk may stop at the smallest c with mask(c) >= overall (depth_test_nerf's cap; the
            // march distance never decreases, so a walk past c ends at a result >= c and leaves `overall` as it is)
            // Any cap c with mask(c) >= overall is exact; c = overall k2 / k1 (1 + 2^-20) is one: mask(c) rounds c k1 to
            // float and divides by k2, relative errors below 2^-23 in all, so mask(c) >= overall (1 + 2^-20)(1 - 2^-23).
            // No division is needed (k1 >= 1: a multiply by 1 / k1 in double is within 2^-52 of the quotient).
            float cap = full_d <= fd ? full_d : __builtin_huge_valf();
            if (k1 > 0.0f && k2 > 0.0 && overall >= 0.0f) {
                const float c = (float)((double)overall * k2 * (1.0 / (double)k1) * (1.0 + 0x1p-20));
                cap = fminf(cap, c);
            }
            const float nd = fminf(full_d, depth_test_nerf(fd, MAX_STEPS_BETWEEN_COMPACTION, a.vol, src, Ld, inv(Ld), 0, a.vol.max_mip, cap));
            const double mask = (double)(nd * k1) / k2;
            overall = (float)fmin((double)overall, mask);
        } else {
            const f3 l = normalize(L.pos - pos);
            const double v = (double)overall + fmin(0.0, (double)dot(l, nrm)) * (double)L.intensity;
            overall = (float)fmin(1.0, v);
        }
    }
    return overall;
}
__device__ __forceinline__ f3 load_f3(const float* __restrict__ p, size_t i) { return mk(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }

// shade_with_shadow (testbed_nerf.cu:1702-1786) in three passes, so that the (2r+1)^2 neighbour terms of a
// pixel -- independent once their light samples are drawn -- run on separate lanes (a thin band of rows
// then still fills the GPU):
//   shadow_draw_kernel    one lane per pixel: the pixel's XORWOW stream drawn in the reference's order
//                         (neighbour slots row-major, lights in order, 3 draws per point light), the light
//                         samples stored per (slot, point light), the state stored back;
//   shadow_term_kernel    one lane per (slot, pixel): the slot's term (the mesh and NeRF depth tests);
//   shadow_finish_kernel  one lane per pixel: the terms summed in slot order, / blend, ^ intensity, applied.
// The same float operations in the same order as one lane looping over the neighbours, so the same bits.
__device__ __forceinline__ bool shadow_slot(const ShadowArgs& a, uint32_t p, uint32_t slot, int& fx, int& fy) {
    const int w = 2 * a.radius + 1;
    const int x = (int)(p % (uint32_t)a.W), y = a.row0 + (int)(p / (uint32_t)a.W);
    fx = x + (int)slot / w - a.radius;
    fy = y + (int)slot % w - a.radius;
    return fx >= 0 && fy >= 0 && fx < a.W && fy < a.H;
}
__global__ __launch_bounds__(256) void shadow_draw_kernel(ShadowArgs a, uint32_t n, uint32_t* __restrict__ rng, uint32_t n_rng, float4* __restrict__ lp) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const size_t idx = (size_t)(p % (uint32_t)a.W) + (size_t)a.W * (a.row0 + (int)(p / (uint32_t)a.W));
    Xorwow r = load_rng(rng, n_rng, idx);
    const uint32_t slots = (uint32_t)((2 * a.radius + 1) * (2 * a.radius + 1));
    for (uint32_t sl = 0; sl < slots; ++sl) {
        int fx, fy;
        if (!shadow_slot(a, p, sl, fx, fy)) continue;
        int k = 0;
        for (int li = 0; li < a.n_lights; ++li) {
            const LightGpu L = const_load(a.lights, li);
            if (L.type != 0) continue;
            const f3 q = light_sample(L, r);
            lp[((size_t)sl * a.n_point + k++) * n + p] = make_float4(q.x, q.y, q.z, 0.0f);
        }
    }
    store_rng(rng, n_rng, idx, r);
}
// persistent grid; with LDS the objects' BVH records and triangles are staged in LDS per workgroup (as the
// raytracer's traversal kernels do), the stacks follow them.  64-item chunks (one slot, 64 consecutive pixels)
// are handed out by SHADOW_NCTR counters in separate memory channels (see shadow_rays_kernel).
template <bool LDS>
__global__ __launch_bounds__(1024) void shadow_term_kernel(ShadowArgs a, uint32_t n, const float* __restrict__ positions, const float* __restrict__ normals,
                                                           const float4* __restrict__ lp, float* __restrict__ terms, uint32_t* __restrict__ work) {
    extern __shared__ float4 smem4[];
    if constexpr (LDS) {
        for (uint32_t k = threadIdx.x; k < a.scene_f4; k += blockDim.x) smem4[k] = a.scene_blob[k];
        __syncthreads();
    }
    int* stack = reinterpret_cast<int*>(smem4 + (LDS ? a.scene_f4 : 0u));
    const TraceCtx<LDS, false> cx{stack + threadIdx.x, (int)blockDim.x, reinterpret_cast<const char*>(smem4), a.bvh_flat};
    const int lane = threadIdx.x & 63;
    const uint32_t slots = (uint32_t)((2 * a.radius + 1) * (2 * a.radius + 1));
    const uint32_t cps = (n + 63u) / 64u, n_chunks = slots * cps;
    uint32_t x = blockIdx.x % SHADOW_NCTR, tried = 0;
    while (tried < SHADOW_NCTR) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(work + x * SHADOW_CTR_STRIDE, 1u);
        k = __shfl(k, 0, 64);
        const uint32_t c = k * SHADOW_NCTR + x;
        if (c >= n_chunks) {
            x = (x + 1u) % SHADOW_NCTR;
            ++tried;
            continue;
        }
        const uint32_t sl = c / cps, p = (c - sl * cps) * 64u + (uint32_t)lane;
        int fx, fy;
        if (p >= n || !shadow_slot(a, p, sl, fx, fy)) continue;
        const size_t tid = (size_t)fy * a.W + fx;
        terms[(size_t)sl * n + p] = shadow_term(a, cx, load_f3(positions, tid), load_f3(normals, tid), lp + (size_t)sl * a.n_point * n + p, n);
    }
}
__global__ __launch_bounds__(256) void shadow_finish_kernel(ShadowArgs a, uint32_t n, const float* __restrict__ terms, float4* __restrict__ rgba) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t slots = (uint32_t)((2 * a.radius + 1) * (2 * a.radius + 1));
    float sum = 0.0f;
    int blend = 0;
    for (uint32_t sl = 0; sl < slots; ++sl) {
        int fx, fy;
        if (!shadow_slot(a, p, sl, fx, fy)) continue;
        sum += terms[(size_t)sl * n + p];
        ++blend;
    }
    sum /= (float)blend;
    sum = pow_small_int(sum, a.intensity);
    const size_t idx = (size_t)(p % (uint32_t)a.W) + (size_t)a.W * (a.row0 + (int)(p / (uint32_t)a.W));
    float4 c = rgba[idx];
    c.x = srgb_to_linear(c.x) * sum;
    c.y = srgb_to_linear(c.y) * sum;
    c.z = srgb_to_linear(c.z) * sum;
    rgba[idx] = c;
}

// ---------------------------------------------------------------------------
// mesh-layer camera rays (raytracer.cu:59-99) -- uv without the half-pixel offset
// ---------------------------------------------------------------------------
__global__ void mesh_rays_kernel(int W, int H, int row0, int row1, CamDev cam, f2 focal, f2 sc, float4* __restrict__ origin_out,
                                 float4* __restrict__ dir_out, float4* __restrict__ acc_rgba, float* __restrict__ acc_depth) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = (uint32_t)(row1 - row0) * (uint32_t)W;
    if (t >= n) return;
    const int x = (int)(t % (uint32_t)W), y = row0 + (int)(t / (uint32_t)W);
    const size_t idx = (size_t)x + (size_t)W * y;
    const f2 uv = {(float)x / (float)W, (float)y / (float)H};
    f3 d = mk((uv.x - sc.x) * (float)W / focal.x, (uv.y - sc.y) * (float)H / focal.y, 1.0f);
    d = mul(m3{cam.c0, cam.c1, cam.c2}, d);
    d = normalize(d);
    origin_out[idx] = make_float4(cam.c3.x, cam.c3.y, cam.c3.z, 0.0f);
    dir_out[idx] = make_float4(d.x, d.y, d.z, 0.0f);
    acc_rgba[idx] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    acc_depth[idx] = MAX_DEPTH;
}

// ---------------------------------------------------------------------------
// sng::raytrace (raytracer.cu:101-218), Final buffer
// ---------------------------------------------------------------------------
// The reference builds with --use_fast_math (CMakeLists.txt:82), so its sinf/cosf here are the
// hardware approximations; __sincosf is the same class (v_sin/v_cos on the angle in revolutions).
__device__ __forceinline__ f3 cone_random_up(f3 orig, f3 up, float longi, float latid) {   // common.cuh:37-48
    const f3 N = normalize(orig);
    const f3 B = normalize(cross(N, up));
    const f3 T = cross(B, N);
    float sl, cl, sp, cp;
    __sincosf(longi, &sl, &cl);
    __sincosf(latid, &sp, &cp);
    const f3 off = mk(sl * cp, sl * sp, cl);
    return orig + mul(m3{T, B, N}, off);
}
__device__ __forceinline__ f3 cone_random_frame(f3 orig, const m3& frame, float longi, float latid) {   // common.cuh:33-36
    float sl, cl, sp, cp;
    __sincosf(longi, &sl, &cl);
    __sincosf(latid, &sp, &cp);
    const f3 off = mk(cl * sp, sl * sp, cl);
    return orig + mul(frame, off);
}
//
// DEFER = false: the whole path per pixel in one kernel (reference structure).
// DEFER = true : the same path and RNG sequence, but every point-light shadow test is written to
//                a shadow-ray queue and the light colours to a hit record; shadow_rays_kernel
//                traces the queue with every lane busy, and rt_accumulate_kernel replays the
//                colour sums in the original order.  Bit-identical to DEFER = false.
// Dynamic LDS of the traversal kernels: [scene blob (LDS = true)][stack: stack_depth x blockDim ints].
// Workgroups are persistent (grid-stride), so each copies the scene blob once.
template <bool LDS, bool CNT = false>
__device__ __forceinline__ TraceCtx<LDS, CNT> trace_ctx_setup(const RaytraceArgs& a, uint32_t* cnt = nullptr) {
    extern __shared__ float4 smem4[];
    if constexpr (LDS) {
        for (uint32_t k = threadIdx.x; k < a.scene_f4; k += blockDim.x) smem4[k] = a.scene_blob[k];
        __syncthreads();
    }
    int* stack = reinterpret_cast<int*>(smem4 + (LDS ? a.scene_f4 : 0u));
    return TraceCtx<LDS, CNT>{stack + threadIdx.x, (int)blockDim.x, reinterpret_cast<const char*>(smem4), a.bvh_flat, cnt, a.count_waves};
}

// shade_object's light loop of one hit (raytracer.cu:16-50) in deferred form: per (light, shadow
// iteration) jl the light colour {lc, 0} -> q.lc_at(k, jl); per point-light sample jp the shadow ray
// {L, full_dist} -> q.shadow_ray(k, jp) (its origin, the hit position, is in the record header).
// One 16-B store each, sample-major (RtQueue): the lanes' consecutive records make each store one
// contiguous run.
__device__ __forceinline__ void write_light_samples(const RaytraceArgs& a, const RtQueue& q, uint32_t k, f3 pos, f3 normal, f3 rd,
                                                    const MaterialGpu& m, Xorwow& r) {
    const f3 V = normalize(-rd);
    uint32_t jl = 0, jp = 0;
    for (int l = 0; l < a.n_lights; ++l) {
        const LightGpu L = const_load(a.lights, l);
        for (uint32_t s = 0; s < a.shadow_iters; ++s, ++jl) {
            const f3 lpos = light_sample(L, r);
            f3 Lv = lpos - pos;
            const float full_dist = length(Lv);
            Lv = normalize(Lv);
            const f3 R = reflect(Lv, normal);
            const f3 lc = fmaxf(0.0f, dot(Lv, normal)) * m.kd * L.intensity + pow_small_int(fmaxf(0.0f, dot(R, V)), m.n) * m.ks;
            *q.lc_at(k, jl) = make_float4(lc.x, lc.y, lc.z, 0.0f);
            if (L.type == 0) *q.shadow_ray(k, jp++) = make_float4(Lv.x, Lv.y, Lv.z, full_dist);
        }
    }
}
template <bool LDS, bool CNT>
__device__ __forceinline__ float trace_shadow_ray(const RaytraceArgs& a, const RtQueue& q, const TraceCtx<LDS, CNT>& cx, uint32_t kr, uint32_t jp);

// Fused shadow queue of a banded frame (rt_fused_shadow; every wave of the path kernel has at most one tile): each
// record allocation of a path wave is published in its workgroup's LDS queue once its records are written, and the
// workgroup's waves without a tile (or past theirs) trace those records' shadow rays while the costly tiles' chains still
// run -- the hand-off stays inside one workgroup (workgroup-scope release / acquire, one CU's L1).  LDS words: [0] entries
// published, [1] entries claimed, [2] waves past their tiles, [3] pad, then RT_FQ_CAP entries {first record, count}.
template <bool LDS, bool CNT>
__device__ __forceinline__ void fq_publish(uint32_t* fq, const RaytraceArgs& a, const RtQueue& q, const TraceCtx<LDS, CNT>& cx, uint32_t k, int lane) {
    const unsigned long long m = __ballot(1);
    const int leader = __ffsll((long long)m) - 1;
    const uint32_t k0 = __shfl(k, leader, 64);   // wave_alloc: the lowest active lane holds the allocation's first record
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the records' global stores before the entry
    uint32_t slot = 0;
    if (lane == leader) slot = __hip_atomic_fetch_add(&fq[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    slot = __shfl(slot, leader, 64);
    if (slot < RT_FQ_CAP) {
        if (lane == leader) {
            __hip_atomic_store(&fq[4 + 2 * slot], k0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(&fq[5 + 2 * slot], (uint32_t)__popcll(m), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else {   // queue full (not reached when every wave has at most one tile): the lanes trace their own record's rays
        for (uint32_t jp = 0; jp < q.nps; ++jp) q.mask[q.mask_at(k, jp)] = trace_shadow_ray(a, q, cx, k, jp);
    }
}
// the consumer side, after the wave's tile loop: claim entries in order until every wave of the workgroup is past its
// tiles and every published entry is claimed.  A claimed entry that is not yet written belongs to a wave between its
// slot claim and its two stores, so every wait ends.
template <bool LDS, bool CNT>
__device__ __forceinline__ void fq_consume(uint32_t* fq, const RaytraceArgs& a, const RtQueue& q, const TraceCtx<LDS, CNT>& cx, int lane) {
    const uint32_t n_waves = blockDim.x >> 6;
    __builtin_amdgcn_s_setprio(0);
    if (lane == 0) __hip_atomic_fetch_add(&fq[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (true) {
        uint32_t h = 0;
        if (lane == 0) h = __hip_atomic_fetch_add(&fq[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        h = __builtin_amdgcn_readfirstlane(__shfl(h, 0, 64));
        uint32_t n = 0, k0 = 0;
        while (true) {
            if (h < RT_FQ_CAP) n = __hip_atomic_load(&fq[5 + 2 * h], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            n = __builtin_amdgcn_readfirstlane(n);
            if (n) break;
            const uint32_t done = __hip_atomic_load(&fq[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t tail = __hip_atomic_load(&fq[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (__builtin_amdgcn_readfirstlane(done) == n_waves && h >= min(__builtin_amdgcn_readfirstlane(tail), RT_FQ_CAP)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (!n) break;
        k0 = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&fq[4 + 2 * h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t total = n * q.nps;
        for (uint32_t j = (uint32_t)lane; j < total; j += 64u) {
            const uint32_t kr = k0 + j / q.nps, jp = j % q.nps;
            q.mask[q.mask_at(kr, jp)] = trace_shadow_ray(a, q, cx, kr, jp);
        }
    }
}

// record header: {next, spp, mat, pos.z} {pdf, att, pos.x, pos.y}
__device__ __forceinline__ void write_record_header(float4* rk, int next, uint32_t spp, int mat, f3 pos, float pdf, float att) {
    rk[0] = make_float4(__int_as_float(next), __uint_as_float(spp), __int_as_float(mat), pos.z);
    rk[1] = make_float4(pdf, att, pos.x, pos.y);
}

// shade_object + Material::scatter of one hit, deferred form (raytracer.cu:6-57, material.cuh:112-123):
// the hit record (linked after prev_rec, or as the pixel's head), its light colours and point-light
// shadow rays go to q; rp / rd / pdf / att become the scattered ray's.
template <bool LDS, bool CNT>
__device__ __forceinline__ void defer_hit(const RaytraceArgs& a, const RtQueue& q, const TraceCtx<LDS, CNT>& cx, uint32_t* fq, int lane, size_t i, uint32_t t,
                                          uint32_t spp, const Hit& h, int& prev_rec, uint32_t& n_hits, Xorwow& r, f3& rp, f3& rd, float& pdf, float& att
#ifdef RT_CHAIN_PROBE
                                          , uint64_t* al_acc = nullptr
#endif
                                          ) {
    const MaterialGpu m = a.mats[h.mat];
#ifdef RT_CHAIN_PROBE
    const uint64_t pa = (uint64_t)wall_clock64();
    const uint32_t k = wave_alloc(q.count, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the atomic's return (and the stores still in flight)
    if (al_acc) *al_acc += (uint64_t)wall_clock64() - pa;
#else
    const uint32_t k = wave_alloc(q.count, lane);
#endif
    if (q.plist) q.plist[(size_t)t * q.max_hits + n_hits] = (int)k;
    ++n_hits;
    float4* rk = q.rec + (size_t)k * q.rec_stride;
    write_record_header(rk, -1, spp, h.mat, h.pos, pdf, att);
    if (prev_rec < 0) q.head[i] = (int)k;
    else reinterpret_cast<int*>(q.rec + (size_t)prev_rec * q.rec_stride)[0] = (int)k;
    prev_rec = (int)k;
    write_light_samples(a, q, k, h.pos, h.normal, rd, m, r);
    if (fq) fq_publish(fq, a, q, cx, k, lane);
    const float spec = m.type == 0 ? PI_F / 2 : m.spec_angle;
    const float lo = curand_uniform(r) * spec;
    const float la = (float)((double)curand_uniform(r) * 2.0 * (double)PI_F);
    const f3 ndir = cone_random_frame(h.normal, h.perturb, lo, la);
    rp = h.pos;
    rd = ndir;
    pdf = 1.0f / fmaxf(1.0f, spec * 2.0f);
    att = 1.0f * m.rg;
}

#ifdef RT_CHAIN_PROBE
// timing-only build (make BUILD=_build_probe EXTRA=-DRT_CHAIN_PROBE, tools/chain_probe.py): s_memrealtime ticks of a
// pixel's phases -- [0] world queries, [1] deferred shading (record allocation included), [2] the allocation's atomic
// alone, [3] queries made -- written after the frame's per-tile costs (rt_tile_cost[n_tiles + 8 tile + j], lane 0)
struct ChainProbe { uint64_t q, sh, al; uint32_t nq; };
#define PROBE_T() ((uint64_t)wall_clock64())
#endif
template <bool DEFER, bool LDS, bool CNT = false>
__device__ __forceinline__ uint32_t raytrace_pixel(const RaytraceArgs& a, const RtQueue& q, const TraceCtx<LDS, CNT>& cx, uint32_t t,
                                               const float4* __restrict__ origins, const float4* __restrict__ dirs, uint32_t* __restrict__ rng,
                                               uint32_t n_rng, float4* __restrict__ acc_rgba, float* __restrict__ acc_depth, uint32_t* fq = nullptr
#ifdef RT_CHAIN_PROBE
                                               , ChainProbe* pr = nullptr
#endif
                                               ) {
    const size_t i = (size_t)a.row0 * a.W + t;
    const int lane = threadIdx.x & 63;
    Xorwow r = load_rng(rng, n_rng, i);
    const float4 o4 = origins[i], d4 = dirs[i];
    const f3 src_p = mk(o4.x, o4.y, o4.z), src_d = mk(d4.x, d4.y, d4.z);
    f3 shade = splat(0.0f), next_pos = splat(0.0f);
    // the ImgBufferType views' sums (raytracer.cu:134-143; one-kernel path only, DEFER requires Final)
    const int buf = DEFER ? 0 : a.buffer_type;
    f3 normal = splat(0.0f), view_pos = splat(0.0f), view_dir = splat(0.0f), next_dir = splat(0.0f);
    float nerf_shadow = 1.0f;
    int prev_rec = -1;
    uint32_t n_hits = 0;
    if (DEFER) q.head[i] = -1;
    for (uint32_t spp = 0; spp < a.samples; ++spp) {
        const float longi = curand_uniform(r) * a.lens;
        const float latid = a.lens != 0.0f ? 0.0f : (float)((double)curand_uniform(r) * 2.0 * (double)PI_F);
        f3 rp = src_p, rd = cone_random_up(src_d, a.up, longi, latid);
        float pdf = 1.0f / (float)a.bounces, att = 1.0f;
        f3 shade_s = splat(0.0f);
        for (uint32_t bounce = 0; bounce < a.bounces; ++bounce) {
            Hit h;
#ifdef RT_CHAIN_PROBE
            const uint64_t pt0 = PROBE_T();
#endif
            const int hit_obj = depth_test_world_hit(rp, rd, a.objs, a.n_objs, cx, h);
#ifdef RT_CHAIN_PROBE
            if (pr) { pr->q += PROBE_T() - pt0; pr->nq += 1; }
#endif
            if (!bounce) {
                next_pos = next_pos + h.pos;
                if (buf != 0) { normal = normal + h.normal; view_pos = view_pos + rp; view_dir = view_dir + rd; }
            }
            if (hit_obj < 0) break;
            if (DEFER) {
#ifdef RT_CHAIN_PROBE
                const uint64_t pt1 = PROBE_T();
#endif
#ifdef RT_CHAIN_PROBE
                defer_hit(a, q, cx, fq, lane, i, t, spp, h, prev_rec, n_hits, r, rp, rd, pdf, att, pr ? &pr->al : nullptr);
#else
                defer_hit(a, q, cx, fq, lane, i, t, spp, h, prev_rec, n_hits, r, rp, rd, pdf, att);
#endif
#ifdef RT_CHAIN_PROBE
                if (pr) pr->sh += PROBE_T() - pt1;
#endif
                continue;
            }
            // shade_object (raytracer.cu:6-57)
            const MaterialGpu m = a.mats[h.mat];
            f3 color = splat(0.0f);
            for (int l = 0; l < a.n_lights; ++l) {
                const LightGpu L = const_load(a.lights, l);
                for (uint32_t s = 0; s < a.shadow_iters; ++s) {
                    const f3 lpos = light_sample(L, r);
                    f3 Lv = lpos - h.pos;
                    const float full_dist = length(Lv);
                    Lv = normalize(Lv);
                    const f3 R = reflect(Lv, h.normal);
                    const f3 V = normalize(-rd);
                    const f3 lc = fmaxf(0.0f, dot(Lv, h.normal)) * m.kd * L.intensity + pow_small_int(fmaxf(0.0f, dot(R, V)), m.n) * m.ks;
                    if (L.type == 0) {
                        const f3 invL = inv(Lv);
                        int oh = -1;
                        const float syn = a.show_nerf_shadow ? depth_test_world(h.pos, Lv, a.objs, a.n_objs, cx, oh) : 1.0f;
                        // the NerfShadow view needs the march's own value, not only min(it, syn, full_dist): no cap then
                        const float nerf = a.show_nerf_shadow
                                               ? depth_test_nerf((float)((double)syn + 1.0), a.shadow_steps, a.vol, h.pos, Lv, invL, 0, a.vol.max_mip,
                                                                 buf == 7 ? 3.0e38f : fminf(syn, full_dist))
                                               : 1.0f;
                        nerf_shadow = fminf(nerf / full_dist, nerf_shadow);   // out_nerf_shadow (raytracer.cu:32)
                        const float sh = fminf(fminf(nerf, syn), full_dist);
                        const float mask = pow_small_int(smoothstep(sh / full_dist), a.syn_shadow_factor);
                        color = color + lc * mask;
                    } else {
                        color = color + lc;
                    }
                }
            }
            color = color / (float)a.shadow_iters;
            color = color + m.ka;
            // Material::scatter (material.cuh:112-123)
            const float spec = m.type == 0 ? PI_F / 2 : m.spec_angle;
            const float lo = curand_uniform(r) * spec;
            const float la = (float)((double)curand_uniform(r) * 2.0 * (double)PI_F);
            const f3 ndir = cone_random_frame(h.normal, h.perturb, lo, la);
            shade_s = shade_s + color * pdf * att;
            if (!bounce) next_dir = next_dir + ndir;
            rp = h.pos;
            rd = ndir;
            pdf = 1.0f / fmaxf(1.0f, spec * 2.0f);
            att = 1.0f * m.rg;
        }
        if (!DEFER) shade = shade + shade_s;
    }
    const float weight = (float)a.samples;
    next_pos = next_pos / weight;
    const float depth = dot(src_d, next_pos - src_p);
    acc_depth[i] = depth;
    if (!DEFER) {
        shade = shade / weight;
        float4 cur = acc_rgba[i];
        const f3 curr = mk(cur.x, cur.y, cur.z);
        if (buf == 0) {
            if (dot(curr, curr) > 0.001f) shade = shade * 0.5f + curr * 0.5f;
        } else {   // raytracer.cu:189-209, vec3_to_col (common.cu:300-302) = v * 0.5 + 0.5
            view_pos = view_pos / weight; view_dir = view_dir / weight; next_dir = next_dir / weight; normal = normal / weight;
            auto col = [](f3 v) { return v * 0.5f + splat(0.5f); };
            switch (buf) {
            case 1: shade = length(next_pos - view_pos) + MIN_DEPTH > MAX_DEPTH ? splat(0.0f) : col(normalize(next_pos)); break;   // NextOrigin
            case 2: shade = col(normalize(view_pos)); break;   // SrcOrigin
            case 3: shade = col(next_dir); break;              // NextDirection
            case 4: shade = col(view_dir); break;              // SrcDirection
            case 5: shade = col(normal); break;                // Normal
            case 6: shade = splat(depth); break;               // Depth
            default: shade = splat(nerf_shadow); break;        // NerfShadow
            }
        }
        acc_rgba[i] = make_float4(shade.x, shade.y, shade.z, cur.w);
    }
    if (DEFER && q.pcount) q.pcount[t] = (uint8_t)n_hits;
    store_rng(rng, n_rng, i, r);
    return n_hits;
}

__global__ void rt_wait_started_kernel(const uint32_t* __restrict__ started, uint32_t seq, uint64_t timeout_ticks) {
    const uint64_t t0 = wall_clock64();   // s_memrealtime, 100 MHz
    while (__hip_atomic_load(started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != seq && wall_clock64() - t0 < timeout_ticks)
        __builtin_amdgcn_s_sleep(8);
}
void launch_rt_wait_started(const uint32_t* started, uint32_t seq, uint32_t timeout_us, hipStream_t s) {
    hipLaunchKernelGGL(rt_wait_started_kernel, dim3(1), dim3(64), 0, s, started, seq, (uint64_t)timeout_us * 100u);
}

// Persistent workgroups; each wave takes T x T pixel tiles (T = 8, or 4 for thin bands: a tile is a
// serial chain of 8 samples x 2 bounces whose divergent traversals cost the union of its lanes' paths,
// so fewer pixels per wave shorten the chain when there are too few tiles to fill the GPU anyway)
// from a device counter (dynamic balance:
// only ~15 % of the pixels hit an object and those cost ~100x the others).  Square tiles keep a
// wave's primary rays coherent (fewer hit/miss-divergent waves than 64-pixel row segments).
// FQ: the fused shadow queue compiled in (banded frames only: the shadow-ray code raises the register pressure)
template <bool DEFER, bool LDS, bool CNT = false, bool FQ = false>
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 4
#endif
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU))) void raytrace_kernel(RaytraceArgs a, RtQueue q, uint32_t* __restrict__ work, const float4* __restrict__ origins,
                                                        const float4* __restrict__ dirs, uint32_t* __restrict__ rng, uint32_t n_rng,
                                                        float4* __restrict__ acc_rgba, float* __restrict__ acc_depth) {
    uint32_t counts[3] = {0u, 0u, 0u};
    if (a.started && threadIdx.x == 0) __hip_atomic_store(a.started, a.started_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the fused shadow queue sits after the blob and the stacks in the dynamic LDS
    uint32_t* fq = nullptr;
    if (DEFER && FQ && a.fused_shadow) {
        extern __shared__ float4 smem4[];
        fq = reinterpret_cast<uint32_t*>(smem4 + (LDS ? a.scene_f4 : 0u)) + (size_t)a.stack_depth * blockDim.x;
        for (uint32_t w = threadIdx.x; w < RT_FQ_WORDS; w += blockDim.x) fq[w] = 0u;
        __syncthreads();
    }
    const TraceCtx<LDS, CNT> cx = trace_ctx_setup<LDS, CNT>(a, counts);
    const int lane = threadIdx.x & 63;
    const uint32_t rows = (uint32_t)(a.row1 - a.row0);
    const uint32_t T = (uint32_t)a.tile, TH = (uint32_t)a.tile_h, tiles_x = ((uint32_t)a.W + T - 1) / T, n_tiles = tiles_x * ((rows + TH - 1) / TH);
    // rt_spread: the first round of tiles is dealt rank r -> workgroup r % grid, wave r / grid, so the costliest tiles of the
    // order start one per CU (and per SIMD) instead of sixteen to the first workgroup to claim; later tiles are claimed
    const uint32_t n_first = a.spread ? gridDim.x * (blockDim.x >> 6) : 0u;
    bool first = a.spread != 0;
    while (true) {
        uint32_t k = 0;
        if (first) {
            k = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
            first = false;
        } else {
            if (lane == 0) k = atomicAdd(work, 1u);
            k = __shfl(k, 0, 64) + n_first;
        }
        if (k >= n_tiles) break;
        // tiles in descending cost of the previous frame (tile_sort_kernel), so the few expensive
        // object tiles start first instead of being the latency tail of the launch
        const uint32_t tile = a.tile_order ? a.tile_order[k] : k;
        // the costliest tiles of the last frame (the first prio_tiles of the order) issue ahead of the other waves
        // of their SIMD: the launch lasts as long as its slowest tile's chain, and the others have slack.  prio_tiles
        // and prio2_tiles are both cumulative bounds of the order (level 3 below the first, level 2 below the second)
        if (a.prio_tiles || a.prio2_tiles) {
            const uint32_t ks = __builtin_amdgcn_readfirstlane(k);
            if (ks < a.prio_tiles) __builtin_amdgcn_s_setprio(3);
            else if (ks < a.prio2_tiles) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
        }
        const uint64_t t0 = wall_clock64();
        const uint32_t x = (tile % tiles_x) * T + (uint32_t)lane % T, y = (tile / tiles_x) * TH + (uint32_t)lane / T;
#ifdef RT_CHAIN_PROBE
        ChainProbe pr{0, 0, 0, 0};
        const uint32_t c0 = counts[0], c1 = counts[1], c2 = counts[2];   // counting frames (rt_count): this tile's share
        if ((uint32_t)lane < T * TH && x < (uint32_t)a.W && y < rows) raytrace_pixel<DEFER>(a, q, cx, y * (uint32_t)a.W + x, origins, dirs, rng, n_rng, acc_rgba, acc_depth, FQ ? fq : nullptr, &pr);
        if (a.tile_cost && lane == 0) {
            uint32_t* pp = a.tile_cost + n_tiles + 8u * tile;
            pp[0] = (uint32_t)pr.q; pp[1] = (uint32_t)pr.sh; pp[2] = (uint32_t)pr.al; pp[3] = pr.nq;
            pp[4] = counts[0] - c0; pp[5] = counts[1] - c1; pp[6] = counts[2] - c2;
        }
#else
        if ((uint32_t)lane < T * TH && x < (uint32_t)a.W && y < rows) raytrace_pixel<DEFER>(a, q, cx, y * (uint32_t)a.W + x, origins, dirs, rng, n_rng, acc_rgba, acc_depth, FQ ? fq : nullptr);
#endif
        if (a.tile_cost && lane == 0) a.tile_cost[tile] = (uint32_t)min<uint64_t>(wall_clock64() - t0, 0xFFFFFFFFull);
    }
    if constexpr (DEFER && FQ) {
        if (fq) fq_consume(fq, a, q, cx, lane);
    }
    if constexpr (CNT) flush_counts(a.counts, counts, lane);
}

// ---------------------------------------------------------------------------------------------
// rt_rng = 1: a measurement mode, off by default and NOT the reference's RNG order.  Each (pixel,
// light sample) draws from its own XORWOW subsequence, curand_init(1999, pixel * S + s, 0) (the same seeding, another
// subsequence per sample), so the S samples of a pixel are independent and trace on S adjacent lanes at once: a wave
// holds 64 / S pixels, and the dependent chain of a unit is one sample's bounces instead of a pixel's S samples in
// turn.  Everything after the path kernel is unchanged: the records carry their sample index, each pixel's record
// list is written in (sample, bounce) order, so shadow_rays_kernel, rt_record_colour_kernel and rt_accumulate_kernel
// sum the same terms as for a serial pixel; the bounce-0 positions (the depth) are summed in sample order.  The frame
// agrees with the reference's in distribution, not bit for bit (tests/test_gpu_rt_rng.py).
// ---------------------------------------------------------------------------------------------
template <bool LDS>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(RT_WAVES_PER_EU))) void raytrace_sp_kernel(
    RaytraceArgs a, RtQueue q, uint32_t* __restrict__ work, const float4* __restrict__ origins, const float4* __restrict__ dirs,
    uint32_t* __restrict__ rng, uint32_t n_rng, float* __restrict__ acc_depth) {
    if (a.started && threadIdx.x == 0) __hip_atomic_store(a.started, a.started_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const TraceCtx<LDS, false> cx = trace_ctx_setup<LDS, false>(a);
    const int lane = threadIdx.x & 63;
    const uint32_t S = a.samples, ppw = 64u / S;                     // pixels per wave (1 <= S <= 64)
    const uint32_t n_px = (uint32_t)(a.row1 - a.row0) * (uint32_t)a.W, n_units = (n_px + ppw - 1u) / ppw;
    const uint32_t sub = (uint32_t)lane / S, s = (uint32_t)lane % S, g0 = sub * S;   // lane -> (pixel of the unit, sample)
    // units claimed a_sp_chunk at a time (host_render.cpp: ~8 claims per wave, 1 for thin bands) -- a full frame has ~2.6e5 units,
    // whose claims on one counter would serialise like the shadow kernel's once did
    const uint32_t chunk = max(1u, a.sp_chunk);
    uint32_t k = 0, k_end = 0;
    while (true) {
        if (k >= k_end) {
            uint32_t c = 0;
            if (lane == 0) c = atomicAdd(work, 1u);
            k = __shfl(c, 0, 64) * chunk;
            if (k >= n_units) break;
            k_end = min(k + chunk, n_units);
        }
        const uint32_t t = k * ppw + sub;
        ++k;
        const bool active = sub < ppw && t < n_px;
        const size_t i = (size_t)a.row0 * a.W + (active ? t : 0u);
        f3 p0 = splat(0.0f), src_p = splat(0.0f), src_d = splat(0.0f);
        uint32_t nh = 0;
        int recs[RT_SP_MAX_BOUNCES];
        if (active) {
            Xorwow r = load_rng(rng, n_rng, i * S + s);
            const float4 o4 = origins[i], d4 = dirs[i];
            src_p = mk(o4.x, o4.y, o4.z);
            src_d = mk(d4.x, d4.y, d4.z);
            // raytrace_pixel's sample loop body for sample s (raytracer.cu:101-218), deferred shading
            const float longi = curand_uniform(r) * a.lens;
            const float latid = a.lens != 0.0f ? 0.0f : (float)((double)curand_uniform(r) * 2.0 * (double)PI_F);
            f3 rp = src_p, rd = cone_random_up(src_d, a.up, longi, latid);
            float pdf = 1.0f / (float)a.bounces, att = 1.0f;
            for (uint32_t bounce = 0; bounce < a.bounces; ++bounce) {
                Hit h;
                const int hit_obj = depth_test_world_hit(rp, rd, a.objs, a.n_objs, cx, h);
                if (!bounce) p0 = h.pos;
                if (hit_obj < 0) break;
                const MaterialGpu m = a.mats[h.mat];
                const uint32_t kr = wave_alloc(q.count, lane);
                recs[nh < RT_SP_MAX_BOUNCES ? nh : 0] = (int)kr;
                ++nh;
                write_record_header(q.rec + (size_t)kr * q.rec_stride, -1, s, h.mat, h.pos, pdf, att);
                write_light_samples(a, q, kr, h.pos, h.normal, rd, m, r);
                const float spec = m.type == 0 ? PI_F / 2 : m.spec_angle;
                const float lo = curand_uniform(r) * spec;
                const float la = (float)((double)curand_uniform(r) * 2.0 * (double)PI_F);
                rd = cone_random_frame(h.normal, h.perturb, lo, la);
                rp = h.pos;
                pdf = 1.0f / fmaxf(1.0f, spec * 2.0f);
                att = 1.0f * m.rg;
            }
            store_rng(rng, n_rng, i * S + s, r);
        }
        // the pixel's list in (sample, bounce) order: an exclusive prefix of the hit counts over its S lanes
        uint32_t off = 0, total = 0;
        f3 next_pos = splat(0.0f);
        for (uint32_t j = 0; j < S; ++j) {
            const uint32_t c = __shfl(nh, (int)(g0 + j), 64);
            const f3 pj = mk(__shfl(p0.x, (int)(g0 + j), 64), __shfl(p0.y, (int)(g0 + j), 64), __shfl(p0.z, (int)(g0 + j), 64));
            if (j < s) off += c;
            total += c;
            next_pos = next_pos + pj;   // raytrace_pixel's sum over the samples, in sample order
        }
        if (active) {
            int* L = q.plist + (size_t)t * q.max_hits;
            for (uint32_t b = 0; b < nh && b < RT_SP_MAX_BOUNCES; ++b) L[off + b] = recs[b];
            if (s == 0) {
                q.pcount[t] = (uint8_t)total;
                next_pos = next_pos / (float)S;
                acc_depth[i] = dot(src_d, next_pos - src_p);
            }
        }
    }
}

// One shadow ray of the deferred raytracer: shade_object's depth_test_world + depth_test_nerf +
// mask (raytracer.cu:30-50).  The BVH query is culled at full_dist: any syn >= full_dist gives
// the same mask (sh = min(nerf, syn, full_dist) and the NeRF march below full_dist does not
// depend on its cap syn + 1 >= full_dist), so the result is bit-identical.
template <bool LDS, bool CNT>
__device__ __forceinline__ float trace_shadow_ray(const RaytraceArgs& a, const RtQueue& q, const TraceCtx<LDS, CNT>& cx, uint32_t kr, uint32_t jp) {
    const float4 s1 = *q.shadow_ray(kr, jp);
    const float4* rk = q.rec + (size_t)kr * q.rec_stride;   // the origin: the record's hit position (header)
    const float4 h0 = rk[0], h1 = rk[1];
    const f3 pos = mk(h1.z, h1.w, h0.w), Lv = mk(s1.x, s1.y, s1.z);
    const float full_dist = s1.w;
    int oh = -1;
    const float syn = depth_test_world(pos, Lv, a.objs, a.n_objs, cx, oh, full_dist);
    const float nerf = depth_test_nerf((float)((double)syn + 1.0), a.shadow_steps, a.vol, pos, Lv, inv(Lv), 0, a.vol.max_mip, fminf(syn, full_dist));
    const float sh = fminf(fminf(nerf, syn), full_dist);
    return pow_small_int(smoothstep(sh / full_dist), a.syn_shadow_factor);
}

// The shadow-ray pass after the path kernel.  (Tracing each tile's shadow rays in the wave that traced its paths
// measured 30 % slower: the shadow work, ~5,000 wave-ms per C3 frame, about equals the path work, and it lands on
// the costliest tiles, which bound the launch.)
template <bool LDS, bool CNT = false>
__global__ __launch_bounds__(1024) void shadow_rays_kernel(RaytraceArgs a, RtQueue q, uint32_t* __restrict__ work) {
    uint32_t counts[3] = {0u, 0u, 0u};
    const TraceCtx<LDS, CNT> cx = trace_ctx_setup<LDS, CNT>(a, counts);
    const uint32_t n_rec = *q.count, total = n_rec * q.nps;
    const int lane = threadIdx.x & 63;
    // 64-ray chunks handed out by SHADOW_NCTR counters in separate memory channels: chunk c belongs to
    // counter c % NCTR, a wave starts on the counter of its workgroup's XCD slot and moves on when that
    // one runs dry.  One shared counter serialised ~200 K same-address atomics per frame (2.0 ms on
    // their own, measured with the tracing removed); static round-robin dealing has no atomics but
    // unbalances the waves (2.8 ms), because the expensive rays cluster in the queue.
    const uint32_t n_chunks = (total + 63u) / 64u;
    uint32_t x = blockIdx.x % SHADOW_NCTR, tried = 0;
    while (tried < SHADOW_NCTR) {
        uint32_t k = 0;
        if (lane == 0) k = atomicAdd(work + x * SHADOW_CTR_STRIDE, 1u);
        k = __shfl(k, 0, 64);
        const uint32_t c = k * SHADOW_NCTR + x;
        if (c >= n_chunks) {
            x = (x + 1u) % SHADOW_NCTR;
            ++tried;
            continue;
        }
        const uint32_t j = c * 64u + (uint32_t)lane;
        if (j >= total) continue;
        const uint32_t kr = j / q.nps, jp = j - kr * q.nps;   // record, shadow sample (RtQueue::shadow_ray)
        q.mask[q.mask_at(kr, jp)] = trace_shadow_ray(a, q, cx, kr, jp);
    }
    if constexpr (CNT) flush_counts(a.counts + 3, counts, lane);
}

// One hit record's term of the colour replay: shade_object's colour (raytracer.cu:6-57) times pdf * att,
// evaluated exactly as rt_accumulate_kernel's chain walk does; .w = the record's sample index.  A wave
// stages its 64 consecutive records and their masks in LDS with coalesced 16-B loads, then each lane
// sums its own record.  Dynamic LDS: waves per block x 64 x (rec_stride float4 + nps floats).
__global__ __launch_bounds__(256) void rt_record_colour_kernel(RaytraceArgs a, RtQueue q) {
    extern __shared__ float4 rc_lds[];
    const uint32_t n = min(*q.count, q.cap);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t rs = q.rec_stride, wave_f4 = 64u * rs + (64u * q.nps + 3u) / 4u;
    float4* recs = rc_lds + wave * wave_f4;
    float* masks = reinterpret_cast<float*>(recs + 64u * rs);
    for (uint32_t k0 = (blockIdx.x * (blockDim.x >> 6) + wave) * 64u; k0 < n; k0 += gridDim.x * blockDim.x) {
        const uint32_t nk = min(64u, n - k0);
        const float4* src = q.rec + (size_t)k0 * rs;
        for (uint32_t e = lane; e < nk * rs; e += 64u) recs[e] = src[e];
        const float* msrc = q.mask + q.mask_at(k0, 0);
        for (uint32_t e = lane; e < nk * q.nps; e += 64u) masks[e] = msrc[e];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < nk) {
            const float4* rk = recs + lane * rs;
            const float4 h0 = rk[0], h1 = rk[1];
            const float* mk_ = masks + lane * q.nps;
            f3 color = splat(0.0f);
            uint32_t jl = 0, jp = 0;
            for (int l = 0; l < a.n_lights; ++l) {
                const bool point = const_load(a.lights, l).type == 0;
                for (uint32_t s = 0; s < a.shadow_iters; ++s, ++jl) {
                    const float4 l4 = *q.lc_at(k0 + lane, jl);
                    const f3 c = mk(l4.x, l4.y, l4.z);
                    if (point) color = color + c * mk_[jp++];
                    else color = color + c;
                }
            }
            color = color / (float)a.shadow_iters;
            color = color + a.mats[__float_as_int(h0.z)].ka;
            const f3 v = color * h1.x * h1.y;
            q.rval[k0 + lane] = make_float4(v.x, v.y, v.z, h0.y);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// Colour replay of the deferred raytracer, in raytrace_kernel's exact float order.
__global__ __launch_bounds__(256) void rt_accumulate_kernel(RaytraceArgs a, RtQueue q, float4* __restrict__ acc_rgba, const float4* __restrict__ next_pos,
                                                            const float4* __restrict__ origins, const float4* __restrict__ dirs, float* __restrict__ acc_depth) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = (uint32_t)(a.row1 - a.row0) * (uint32_t)a.W;
    if (t >= n) return;
    const size_t i = (size_t)a.row0 * a.W + t;
    f3 shade = splat(0.0f);
    if (q.plist) {
        // list mode: the pixel's records in allocation order, their terms from rt_record_colour_kernel; the
        // first 16 are loaded up front (independent loads), so the sum waits for memory once, not per record
        constexpr uint32_t PRE = 16;
        const uint32_t cnt = q.pcount[t];
        const int* L = q.plist + (size_t)t * q.max_hits;
        // unconditional loads within the pixel's list (slots past the count re-read its last record and are discarded by the
        // select): a conditional load per slot compiled into a branch and a wait per record, i.e. 16 serial round trips
        float4 v[PRE];
        if (cnt) {   // (a pixel without hits -- most of them -- loads nothing)
            int idx[PRE];
#pragma unroll
            for (uint32_t h = 0; h < PRE; ++h) idx[h] = L[min(h, cnt - 1u)];
#pragma unroll
            for (uint32_t h = 0; h < PRE; ++h) {
                const float4 x = q.rval[idx[h]];
                v[h] = h < cnt ? x : make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0xFFFFFFFFu));
            }
        }
        uint32_t h = 0;
        for (uint32_t spp = 0; spp < a.samples; ++spp) {
            f3 shade_s = splat(0.0f);
            while (h < cnt) {
                float4 w;
                if (h < PRE) {
#pragma unroll
                    for (uint32_t u = 0; u < PRE; ++u) if (u == h) w = v[u];
                } else {
                    w = q.rval[L[h]];
                }
                if (__float_as_uint(w.w) != spp) break;
                shade_s = shade_s + mk(w.x, w.y, w.z);
                ++h;
            }
            shade = shade + shade_s;
        }
    } else {
    int k = q.head[i];
    for (uint32_t spp = 0; spp < a.samples; ++spp) {
        f3 shade_s = splat(0.0f);
        while (k >= 0) {
            const float4* rk = q.rec + (size_t)k * q.rec_stride;
            const float4 h0 = rk[0], h1 = rk[1];
            if (__float_as_uint(h0.y) != spp) break;
            f3 color = splat(0.0f);
            uint32_t jl = 0, jp = 0;
            for (int l = 0; l < a.n_lights; ++l) {
                const bool point = const_load(a.lights, l).type == 0;
                for (uint32_t s = 0; s < a.shadow_iters; ++s, ++jl) {
                    const float4 l4 = *q.lc_at((uint32_t)k, jl);
                    const f3 c = mk(l4.x, l4.y, l4.z);
                    if (point) color = color + c * q.mask[q.mask_at((uint32_t)k, jp++)];
                    else color = color + c;
                }
            }
            color = color / (float)a.shadow_iters;
            color = color + a.mats[__float_as_int(h0.z)].ka;
            shade_s = shade_s + color * h1.x * h1.y;
            k = __float_as_int(h0.x);
        }
        shade = shade + shade_s;
    }
    }
    shade = shade / (float)a.samples;
    if (next_pos) {   // staged mode: raytrace_pixel's depth from the summed first hits
        const float4 np = next_pos[i], o4 = origins[i], d4 = dirs[i];
        const f3 npv = mk(np.x, np.y, np.z) / (float)a.samples;
        acc_depth[i] = dot(mk(d4.x, d4.y, d4.z), npv - mk(o4.x, o4.y, o4.z));
    }
    float4 cur = acc_rgba[i];
    const f3 curr = mk(cur.x, cur.y, cur.z);
    if (dot(curr, curr) > 0.001f) shade = shade * 0.5f + curr * 0.5f;
    acc_rgba[i] = make_float4(shade.x, shade.y, shade.z, cur.w);
}

// ---------------------------------------------------------------------------
// curand_init(PT_SEED, idx, 0): v <- (M^(2^67))^idx v via precomputed powers
// ---------------------------------------------------------------------------
__global__ void xorwow_init_kernel(uint32_t n, uint32_t seed_lo, uint32_t seed_hi, const uint32_t* __restrict__ seq_pow /* 32 x 160 x 5 */,
                                   uint32_t* __restrict__ st) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t s0 = seed_lo ^ 0xaad26b49u, s1 = seed_hi ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0, t1 = 2591861531u * s1;
    uint32_t v[5] = {123456789u + t0, 362436069u ^ t0, 521288629u + t1, 88675123u ^ t1, 5783321u + t0};
    const uint32_t d = 6615241u + t1 + t0;
    for (int k = 0; k < 32; ++k) {
        if (!((i >> k) & 1u)) continue;
        const uint32_t* m = seq_pow + (size_t)k * 160 * 5;
        uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
        for (int j = 0; j < 160; ++j) {
            const uint32_t w = (j < 32) ? v[0] : (j < 64) ? v[1] : (j < 96) ? v[2] : (j < 128) ? v[3] : v[4];
            if ((w >> (j & 31)) & 1u) {
                const uint32_t* c = m + j * 5;
                r0 ^= c[0]; r1 ^= c[1]; r2 ^= c[2]; r3 ^= c[3]; r4 ^= c[4];
            }
        }
        v[0] = r0; v[1] = r1; v[2] = r2; v[3] = r3; v[4] = r4;
    }
    st[i] = v[0]; st[n + i] = v[1]; st[2 * (size_t)n + i] = v[2]; st[3 * (size_t)n + i] = v[3]; st[4 * (size_t)n + i] = v[4];
    st[5 * (size_t)n + i] = d;
}

// ---------------------------------------------------------------------------
void launch_mesh_rays(int W, int H, int row0, int row1, const CamDev& cam, f2 focal, f2 sc, float4* o, float4* d, float4* acc, float* accd,
                      hipStream_t s) {
    const uint32_t n = (uint32_t)(row1 - row0) * (uint32_t)W;
    if (!n) return;
    hipLaunchKernelGGL(mesh_rays_kernel, dim3((n + 255) / 256), dim3(256), 0, s, W, H, row0, row1, cam, focal, sc, o, d, acc, accd);
}
// Order tiles by descending previous-frame cost: 32 log2 buckets, one workgroup (n_tiles <= 2^20).
// Tile order for the next path-kernel launch: tiles binned by log2(cost), descending (any order is exact --
// it only schedules).  Two wide passes instead of one workgroup: per-block LDS histograms summed into 32
// global bins, then each block takes its bins' ranges with one atomic per bin and scatters.
// aux: [0, 32) bin counts, [32, 64) bin cursors (zeroed by the launcher).
__device__ __forceinline__ uint32_t tile_bin(uint32_t cost) { return 31u - min(31u, 31u - (uint32_t)__clz(cost | 1u)); }
__global__ __launch_bounds__(256) void tile_hist_kernel(const uint32_t* __restrict__ cost, uint32_t n, uint32_t* __restrict__ aux) {
    __shared__ uint32_t h[32];
    if (threadIdx.x < 32) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) atomicAdd(&h[tile_bin(cost[i])], 1u);
    __syncthreads();
    if (threadIdx.x < 32 && h[threadIdx.x]) atomicAdd(&aux[threadIdx.x], h[threadIdx.x]);
}
__global__ __launch_bounds__(256) void tile_scatter_kernel(const uint32_t* __restrict__ cost, uint32_t n, uint32_t* __restrict__ aux,
                                                           uint32_t* __restrict__ order) {
    __shared__ uint32_t h[32], base[32];
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x, i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    if (threadIdx.x < 32) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = i0 + threadIdx.x; i < i1; i += 256) atomicAdd(&h[tile_bin(cost[i])], 1u);
    __syncthreads();
    if (threadIdx.x < 32) {
        uint32_t pre = 0;
        for (uint32_t b = 0; b < threadIdx.x; ++b) pre += aux[b];
        base[threadIdx.x] = h[threadIdx.x] ? pre + atomicAdd(&aux[32 + threadIdx.x], h[threadIdx.x]) : 0u;
    }
    __syncthreads();
    for (uint32_t i = i0 + threadIdx.x; i < i1; i += 256) order[atomicAdd(&base[tile_bin(cost[i])], 1u)] = i;
}
void launch_tile_sort(const uint32_t* cost, uint32_t n, uint32_t* order, uint32_t* aux, hipStream_t s) {
    (void)hipMemsetAsync(aux, 0, 64 * sizeof(uint32_t), s);
    const uint32_t blocks = std::max(1u, std::min(256u, (n + 1023) / 1024));
    hipLaunchKernelGGL(tile_hist_kernel, dim3(blocks), dim3(256), 0, s, cost, n, aux);
    hipLaunchKernelGGL(tile_scatter_kernel, dim3(blocks), dim3(256), 0, s, cost, n, aux, order);
}

static size_t trace_lds_bytes(const RaytraceArgs& a, bool lds, uint32_t tpb) {
    return (lds ? (size_t)a.scene_f4 * 16 : 0) + (size_t)a.stack_depth * tpb * 4;
}
template <typename K>
static void allow_lds(K kernel, size_t bytes) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
void launch_raytrace(const RaytraceArgs& a, const float4* o, const float4* d, uint32_t* rng, uint32_t n_rng, float4* acc, float* accd,
                     hipStream_t s) {
    const uint32_t n = (uint32_t)(a.row1 - a.row0) * (uint32_t)a.W;
    if (!n) return;
    const uint32_t tpb = 256, blocks = std::min((n + tpb - 1) / tpb, a.persistent_blocks * 3);
    const size_t lds = trace_lds_bytes(a, false, tpb);
    (void)hipMemsetAsync(a.work, 0, RT_WORK_WORDS * sizeof(uint32_t), s);
    allow_lds(raytrace_kernel<false, false>, lds);
    hipLaunchKernelGGL((raytrace_kernel<false, false>), dim3(blocks), dim3(tpb), lds, s, a, RtQueue{}, a.work, o, d, rng, n_rng, acc, accd);
}
void launch_raytrace_wavefront(const RaytraceArgs& a, const RtQueue& q, const float4* o, const float4* d, uint32_t* rng, uint32_t n_rng, float4* acc,
                               float* accd, uint32_t shadow_blocks, hipStream_t s) {
    const uint32_t n = (uint32_t)(a.row1 - a.row0) * (uint32_t)a.W;
    if (!n) return;
    // the work counters, the record counter among them (q.count = work + RT_REC_COUNT, host_render.cpp): one clear
    // (errors surface through hipGetLastError in the caller)
    if (q.count < a.work || q.count >= a.work + RT_WORK_WORDS) (void)hipMemsetAsync(q.count, 0, sizeof(uint32_t), s);
    (void)hipMemsetAsync(a.work, 0, RT_WORK_WORDS * sizeof(uint32_t), s);
    // path kernel: capped at 128 VGPRs (amdgpu_waves_per_eu(4), a few spills) -> 4 waves/SIMD = 2 x 512-thread workgroups;
    // measured faster than 3 waves/SIMD without spills
    // shadow kernel: ~100 VGPRs -> 5 waves/SIMD; LDS-bound at 16 waves per CU (2 x 512 or 1 x 1024 threads, lds_tpb)
    const bool lds = a.scene_in_lds != 0;
    const uint32_t tp = lds ? a.lds_tpb : 512u, ts = tp, per_cu = 1024u / tp;   // 16 waves per CU either way
    const size_t lp = trace_lds_bytes(a, lds, tp) + (a.fused_shadow ? RT_FQ_WORDS * 4u : 0u), ls = trace_lds_bytes(a, lds, ts);
    const uint32_t n_tiles = (((uint32_t)a.W + a.tile - 1) / a.tile) * (((uint32_t)(a.row1 - a.row0) + a.tile_h - 1) / a.tile_h);
    // rt_spread: every CU gets a workgroup (a thin band's tiles then spread over the whole GPU, one wave each)
    const uint32_t bp = (a.spread || a.sample_par) ? a.persistent_blocks * per_cu : std::min((n_tiles + tp / 64 - 1) / (tp / 64), a.persistent_blocks * per_cu);
    const uint32_t sb = shadow_blocks ? shadow_blocks : a.persistent_blocks * per_cu;
    if (a.sample_par) {   // rt_rng = 1 (host_render.cpp: list mode, no counters, no fused queue): the sample-parallel path kernel
        RaytraceArgs b = a;   // ~8 claims per wave of the grid (a band's few units: one per claim)
        const uint32_t ppw = 64u / std::max(1u, a.samples), units = (n + ppw - 1) / ppw, waves = bp * (tp / 64u);
        b.sp_chunk = std::max(1u, units / (waves * 8u));
        if (lds) {
            allow_lds(raytrace_sp_kernel<true>, lp);
            allow_lds(shadow_rays_kernel<true>, ls);
            hipLaunchKernelGGL((raytrace_sp_kernel<true>), dim3(bp), dim3(tp), lp, s, b, q, a.work, o, d, rng, n_rng, accd);
            hipLaunchKernelGGL(shadow_rays_kernel<true>, dim3(sb), dim3(ts), ls, s, a, q, a.work + SHADOW_CTR0);
        } else {
            allow_lds(raytrace_sp_kernel<false>, lp);
            allow_lds(shadow_rays_kernel<false>, ls);
            hipLaunchKernelGGL((raytrace_sp_kernel<false>), dim3(bp), dim3(tp), lp, s, b, q, a.work, o, d, rng, n_rng, accd);
            hipLaunchKernelGGL(shadow_rays_kernel<false>, dim3(sb), dim3(ts), ls, s, a, q, a.work + SHADOW_CTR0);
        }
    } else if (lds && a.counts) {   // counting frame (rt_count): the same kernels with the traversal counters compiled in
        allow_lds(raytrace_kernel<true, true, true>, lp);
        allow_lds(shadow_rays_kernel<true, true>, ls);
        hipLaunchKernelGGL((raytrace_kernel<true, true, true>), dim3(bp), dim3(tp), lp, s, a, q, a.work, o, d, rng, n_rng, acc, accd);
            hipLaunchKernelGGL((shadow_rays_kernel<true, true>), dim3(sb), dim3(ts), ls, s, a, q, a.work + SHADOW_CTR0);
    } else if (lds) {
        if (a.fused_shadow) {
            allow_lds(raytrace_kernel<true, true, false, true>, lp);
            hipLaunchKernelGGL((raytrace_kernel<true, true, false, true>), dim3(bp), dim3(tp), lp, s, a, q, a.work, o, d, rng, n_rng, acc, accd);
        } else {
            allow_lds(raytrace_kernel<true, true>, lp);
            allow_lds(shadow_rays_kernel<true>, ls);
            hipLaunchKernelGGL((raytrace_kernel<true, true>), dim3(bp), dim3(tp), lp, s, a, q, a.work, o, d, rng, n_rng, acc, accd);
            hipLaunchKernelGGL(shadow_rays_kernel<true>, dim3(sb), dim3(ts), ls, s, a, q, a.work + SHADOW_CTR0);
        }
    } else {
        allow_lds(raytrace_kernel<true, false>, lp);
        allow_lds(shadow_rays_kernel<false>, ls);
        if (a.fused_shadow) {
            allow_lds(raytrace_kernel<true, false, false, true>, lp);
            hipLaunchKernelGGL((raytrace_kernel<true, false, false, true>), dim3(bp), dim3(tp), lp, s, a, q, a.work, o, d, rng, n_rng, acc, accd);
        } else {
            hipLaunchKernelGGL((raytrace_kernel<true, false>), dim3(bp), dim3(tp), lp, s, a, q, a.work, o, d, rng, n_rng, acc, accd);
            hipLaunchKernelGGL(shadow_rays_kernel<false>, dim3(sb), dim3(ts), ls, s, a, q, a.work + SHADOW_CTR0);
        }
    }
    if (q.plist) {   // host_render.cpp enables the lists only when one wave's staging fits 64 KB
        const size_t per_wave = 16u * (64u * q.rec_stride + (64u * q.nps + 3u) / 4u);
        const uint32_t waves = (uint32_t)std::max<size_t>(1, std::min<size_t>(4, (160u * 1024u) / per_wave));
        allow_lds(rt_record_colour_kernel, waves * per_wave);
        hipLaunchKernelGGL(rt_record_colour_kernel, dim3(a.persistent_blocks * 16 / waves), dim3(64 * waves), waves * per_wave, s, a, q);
    }
    hipLaunchKernelGGL(rt_accumulate_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, q, acc, (const float4*)nullptr, o, d, accd);
}

void launch_xorwow_init(uint32_t n, uint64_t seed, const uint32_t* seq_pow, uint32_t* st, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(xorwow_init_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, (uint32_t)seed, (uint32_t)(seed >> 32), seq_pow, st);
}

constexpr size_t SHADOW_WORK_BYTES = SHADOW_NCTR * SHADOW_CTR_STRIDE * sizeof(uint32_t);
size_t shadow_scratch_bytes(const ShadowArgs& a) {
    const size_t n = (size_t)(a.row1 - a.row0) * (size_t)a.W, slots = (size_t)(2 * a.radius + 1) * (size_t)(2 * a.radius + 1);
    return SHADOW_WORK_BYTES + slots * n * ((size_t)a.n_point * sizeof(float4) + sizeof(float));
}
void launch_shadows(const ShadowArgs& a, float4* rgba, const float* pos, const float* nrm, uint32_t* rng, uint32_t n_rng, void* scratch, hipStream_t s) {
    const uint32_t n = (uint32_t)(a.row1 - a.row0) * (uint32_t)a.W;
    if (!n) return;
    const size_t slots = (size_t)(2 * a.radius + 1) * (size_t)(2 * a.radius + 1);
    uint32_t* work = static_cast<uint32_t*>(scratch);
    float4* lp = reinterpret_cast<float4*>(static_cast<char*>(scratch) + SHADOW_WORK_BYTES);
    float* terms = reinterpret_cast<float*>(lp + slots * (size_t)a.n_point * n);
    (void)hipMemsetAsync(work, 0, SHADOW_WORK_BYTES, s);   // errors surface through hipGetLastError in the caller
    hipLaunchKernelGGL(shadow_draw_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, n, rng, n_rng, lp);
    const size_t lds = (a.scene_in_lds ? (size_t)a.scene_f4 * 16 : 0) + (size_t)a.stack_depth * a.tpb * 4;
    if (a.scene_in_lds) {
        allow_lds(shadow_term_kernel<true>, lds);
        hipLaunchKernelGGL(shadow_term_kernel<true>, dim3(a.blocks), dim3(a.tpb), lds, s, a, n, pos, nrm, lp, terms, work);
    } else {
        allow_lds(shadow_term_kernel<false>, lds);
        hipLaunchKernelGGL(shadow_term_kernel<false>, dim3(a.blocks), dim3(a.tpb), lds, s, a, n, pos, nrm, lp, terms, work);
    }
    hipLaunchKernelGGL(shadow_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, n, terms, rgba);
}

}  // namespace sng
