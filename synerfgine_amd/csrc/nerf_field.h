// nerf_field.h -- device functions of the fused NeRF field (hash grid + SH + MLPs on MFMA),
// shared by the standalone network kernel (network.hip) and the fused marcher (fused.hip).
// See network.hip for the lane/fragment mapping.  [tcnn semantics restated -- DESIGN.md]
#pragma once
#include <type_traits>
#include "sng_math.h"
#include "sng_internal.h"

namespace sng {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma16(h8 a, h8 b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

// ReLU + round two accumulator blocks into one 32-deep B fragment (slots 0-3 from lo, 4-7 from hi)
__device__ __forceinline__ h8 pack_relu(f4v lo, f4v hi) {
    h8 r;
    r[0] = (_Float16)fmaxf(lo[0], 0.0f); r[1] = (_Float16)fmaxf(lo[1], 0.0f);
    r[2] = (_Float16)fmaxf(lo[2], 0.0f); r[3] = (_Float16)fmaxf(lo[3], 0.0f);
    r[4] = (_Float16)fmaxf(hi[0], 0.0f); r[5] = (_Float16)fmaxf(hi[1], 0.0f);
    r[6] = (_Float16)fmaxf(hi[2], 0.0f); r[7] = (_Float16)fmaxf(hi[3], 0.0f);
    return r;
}

// tcnn grid_index: the dense or hashed index modulo the level size.  FAST_MOD: for a dense level
// res^3 <= size, so a corner inside the grid (x, y, z <= res) has idx <= res + res^2 + res^3 < 2 * size
// and the modulo is one conditional subtraction; the full `%` runs only for corners outside (same value).
// (The network kernel keeps the plain form: 2 more VGPRs would cost it a wave per SIMD.)
template <bool FAST_MOD = false>
__device__ __forceinline__ uint32_t grid_index(const LevelInfo& L, uint32_t x, uint32_t y, uint32_t z) {
    uint32_t idx = L.dense ? (x + y * L.res + z * L.res2) : ((x * 1u) ^ (y * 2654435761u) ^ (z * 805459861u));
    if (L.pow2_mask) return idx & L.pow2_mask;
    if (FAST_MOD && L.dense && idx < 2u * L.size) return idx >= L.size ? idx - L.size : idx;
    return idx % L.size;
}

// Interpolate one level for one sample: tcnn kernel_grid N-linear path,
// result = fma((half)weight, corner, result) over corners idx = 0..7.
template <int F>
__device__ __forceinline__ void encode_level(const LevelInfo& L, const _Float16* __restrict__ grid, float x0, float x1, float x2,
                                             _Float16* out) {
    float p0 = fmaf(L.scale, x0, 0.5f), p1 = fmaf(L.scale, x1, 0.5f), p2 = fmaf(L.scale, x2, 0.5f);
    float q0 = floorf(p0), q1 = floorf(p1), q2 = floorf(p2);
    uint32_t g0 = (uint32_t)(int)q0, g1 = (uint32_t)(int)q1, g2 = (uint32_t)(int)q2;
    float f0 = p0 - q0, f1 = p1 - q1, f2 = p2 - q2;
    const _Float16* tbl = grid + (size_t)L.offset * F;
    // issue all 8 gathers first
    uint32_t idx[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) idx[c] = grid_index(L, g0 + (c & 1), g1 + ((c >> 1) & 1), g2 + ((c >> 2) & 1)) * F;
    if constexpr (F == 4) {
        uint2 v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = *reinterpret_cast<const uint2*>(tbl + idx[c]);
        h2 r01 = {(_Float16)0.0f, (_Float16)0.0f}, r23 = r01;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float w = 1.0f;
            w *= (c & 1) ? f0 : 1.0f - f0;
            w *= (c & 2) ? f1 : 1.0f - f1;
            w *= (c & 4) ? f2 : 1.0f - f2;
            asm volatile("" : "+v"(w));   // keep the f32 product rounded before the f16 cast (no v_fma_mix fusion): tcnn (T)weight
            _Float16 wh = (_Float16)w;
            h2 w2 = {wh, wh};
            h2 a = __builtin_bit_cast(h2, v[c].x), b = __builtin_bit_cast(h2, v[c].y);
            r01 = __builtin_elementwise_fma(w2, a, r01);
            r23 = __builtin_elementwise_fma(w2, b, r23);
        }
        out[0] = r01[0]; out[1] = r01[1]; out[2] = r23[0]; out[3] = r23[1];
    } else {
        uint32_t v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = *reinterpret_cast<const uint32_t*>(tbl + idx[c]);
        h2 r = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float w = 1.0f;
            w *= (c & 1) ? f0 : 1.0f - f0;
            w *= (c & 2) ? f1 : 1.0f - f1;
            w *= (c & 4) ? f2 : 1.0f - f2;
            asm volatile("" : "+v"(w));   // keep the f32 product rounded before the f16 cast (no v_fma_mix fusion): tcnn (T)weight
            _Float16 wh = (_Float16)w;
            h2 w2 = {wh, wh};
            r = __builtin_elementwise_fma(w2, __builtin_bit_cast(h2, v[c]), r);
        }
        out[0] = r[0]; out[1] = r[1];
    }
}

// The lane's 8 features: levels [lpl*g, lpl*g + lpl) (lpl = 8/F levels per lane), one level at a time
// (the standalone network kernel: 72 VGPRs and 7 waves per SIMD hide the gathers best this way).
template <int F>
__device__ __forceinline__ h8 encode_lane(const LevelInfo* __restrict__ levels, const _Float16* __restrict__ grid, int g, float x0,
                                          float x1, float x2) {
    constexpr int LPL = 8 / F;
    _Float16 e[8];
#pragma unroll
    for (int l = 0; l < LPL; ++l) {
        LevelInfo L = levels[g * LPL + l];
        encode_level<F>(L, grid, x0, x1, x2, e + l * F);
    }
    h8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = e[j];
    return r;
}
// The same features with the gathers of ALL the lane's levels issued before any corner is blended, so
// a sample waits for memory once instead of once per level (encode_level's arithmetic; the fused tail,
// whose waves each walk their own samples: 0.85 -> 0.75 ms in C3; the network kernel lost occupancy
// with the 8 extra VGPRs and ran 12 % slower, so it keeps encode_lane).
template <int F>
__device__ __forceinline__ h8 encode_lane_all(const LevelInfo* __restrict__ levels, const _Float16* __restrict__ grid, int g, float x0,
                                              float x1, float x2) {
    constexpr int LPL = 8 / F;
    typedef typename std::conditional<F == 4, uint2, uint32_t>::type V;
    V v[LPL][8];
    float fr[LPL][3];
#pragma unroll
    for (int l = 0; l < LPL; ++l) {
        const LevelInfo L = levels[g * LPL + l];
        const float p0 = fmaf(L.scale, x0, 0.5f), p1 = fmaf(L.scale, x1, 0.5f), p2 = fmaf(L.scale, x2, 0.5f);
        const float q0 = floorf(p0), q1 = floorf(p1), q2 = floorf(p2);
        const uint32_t g0 = (uint32_t)(int)q0, g1 = (uint32_t)(int)q1, g2 = (uint32_t)(int)q2;
        fr[l][0] = p0 - q0; fr[l][1] = p1 - q1; fr[l][2] = p2 - q2;
        const _Float16* tbl = grid + (size_t)L.offset * F;
#pragma unroll
        for (int c = 0; c < 8; ++c)
            v[l][c] = *reinterpret_cast<const V*>(tbl + grid_index<true>(L, g0 + (c & 1), g1 + ((c >> 1) & 1), g2 + ((c >> 2) & 1)) * F);
    }
    h8 r;
#pragma unroll
    for (int l = 0; l < LPL; ++l) {
        const float f0 = fr[l][0], f1 = fr[l][1], f2 = fr[l][2];
        if constexpr (F == 4) {
            h2 r01 = {(_Float16)0.0f, (_Float16)0.0f}, r23 = r01;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                float w = 1.0f;
                w *= (c & 1) ? f0 : 1.0f - f0;
                w *= (c & 2) ? f1 : 1.0f - f1;
                w *= (c & 4) ? f2 : 1.0f - f2;
                asm volatile("" : "+v"(w));   // keep the f32 product rounded before the f16 cast (no v_fma_mix fusion): tcnn (T)weight
                const _Float16 wh = (_Float16)w;
                const h2 w2 = {wh, wh};
                r01 = __builtin_elementwise_fma(w2, __builtin_bit_cast(h2, v[l][c].x), r01);
                r23 = __builtin_elementwise_fma(w2, __builtin_bit_cast(h2, v[l][c].y), r23);
            }
            r[l * 4 + 0] = r01[0]; r[l * 4 + 1] = r01[1]; r[l * 4 + 2] = r23[0]; r[l * 4 + 3] = r23[1];
        } else {
            h2 acc = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                float w = 1.0f;
                w *= (c & 1) ? f0 : 1.0f - f0;
                w *= (c & 2) ? f1 : 1.0f - f1;
                w *= (c & 4) ? f2 : 1.0f - f2;
                asm volatile("" : "+v"(w));   // keep the f32 product rounded before the f16 cast (no v_fma_mix fusion): tcnn (T)weight
                const _Float16 wh = (_Float16)w;
                const h2 w2 = {wh, wh};
                acc = __builtin_elementwise_fma(w2, __builtin_bit_cast(h2, v[l][c]), acc);
            }
            r[l * 2 + 0] = acc[0]; r[l * 2 + 1] = acc[1];
        }
    }
    return r;
}

// SH degree 4 (tcnn sh_enc), coefficients 4g..4g+3 for this lane group
__device__ __forceinline__ void sh_lane(int g, float dx, float dy, float dz, float o[4]) {
    float x = dx * 2.f - 1.f, y = dy * 2.f - 1.f, z = dz * 2.f - 1.f;
    float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    float s0, s1, s2, s3;
    if (g == 0) {
        s0 = 0.28209479177387814f; s1 = -0.48860251190291987f * y; s2 = 0.48860251190291987f * z; s3 = -0.48860251190291987f * x;
    } else if (g == 1) {
        s0 = 1.0925484305920792f * xy; s1 = -1.0925484305920792f * yz; s2 = 0.94617469575755997f * z2 - 0.31539156525251999f;
        s3 = -1.0925484305920792f * xz;
    } else if (g == 2) {
        s0 = 0.54627421529603959f * x2 - 0.54627421529603959f * y2; s1 = 0.59004358992664352f * y * (-3.0f * x2 + y2);
        s2 = 2.8906114426405538f * xy * z; s3 = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
    } else {
        s0 = 0.3731763325901154f * z * (5.0f * z2 - 3.0f); s1 = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
        s2 = 1.4453057213202769f * z * (x2 - y2); s3 = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
    }
    o[0] = s0; o[1] = s1; o[2] = s2; o[3] = s3;
}

// One 16-sample tile: lane (g = lane>>4, col = lane&15) holds sample `col`'s coordinates; returns
// the rgb accumulator rows 4g..4g+3 (o) and density rows 4g..4g+3 (dens) of that sample.
// Weights in LDS instead of VGPRs: W[f] reads this lane's 16-B slice of fragment f (20 KiB per
// workgroup, conflict-free ds_read_b128), freeing 80 VGPRs per lane (nerf_network_kernel)
struct LdsWeights {
    const h8* base;   // LDS, [20][64]
    int lane;
    __device__ __forceinline__ h8 operator[](int f) const { return base[f * 64 + lane]; }
};

// DENS_ONLY: the density MLP alone (NerfNetwork::density, the density-grid update): o = 0, no SH, no rgb MLP
template <int F, bool GATHER_ALL = false, typename WT = const h8*, bool DENS_ONLY = false>
__device__ __forceinline__ void field_tile(WT W, const LevelInfo* __restrict__ levels, const _Float16* __restrict__ grid, int g, float x0,
                                           float x1, float x2, float d0, float d1, float d2, f4v& o, f4v& dens) {
    const f4v zero = {0.0f, 0.0f, 0.0f, 0.0f};
    // ---- hash grid encoding -> B fragment of layer 0
    h8 enc = GATHER_ALL ? encode_lane_all<F>(levels, grid, g, x0, x1, x2) : encode_lane<F>(levels, grid, g, x0, x1, x2);
    // ---- density MLP: H^T = relu(W0 E^T) (64 rows = 4 blocks), O^T = W1 H^T (16 rows)
    f4v a0 = mfma16(W[0], enc, zero), a1 = mfma16(W[1], enc, zero), a2 = mfma16(W[2], enc, zero), a3 = mfma16(W[3], enc, zero);
    dens = mfma16(W[4], pack_relu(a0, a1), zero);
    dens = mfma16(W[5], pack_relu(a2, a3), dens);
    if constexpr (DENS_ONLY) {
        o = zero;
        return;
    }
    // ---- rgb MLP input: slots 0-3 = density_out rows 4g..4g+3 (fp16), 4-7 = SH 4g..4g+3
    float sh[4];
    sh_lane(g, d0, d1, d2, sh);
    h8 rin;
    rin[0] = (_Float16)dens[0]; rin[1] = (_Float16)dens[1]; rin[2] = (_Float16)dens[2]; rin[3] = (_Float16)dens[3];
    rin[4] = (_Float16)sh[0]; rin[5] = (_Float16)sh[1]; rin[6] = (_Float16)sh[2]; rin[7] = (_Float16)sh[3];
    f4v b0 = mfma16(W[6], rin, zero), b1 = mfma16(W[7], rin, zero), b2 = mfma16(W[8], rin, zero), b3 = mfma16(W[9], rin, zero);
    h8 k0 = pack_relu(b0, b1), k1 = pack_relu(b2, b3);
    f4v c0 = mfma16(W[10], k0, zero); c0 = mfma16(W[11], k1, c0);
    f4v c1 = mfma16(W[12], k0, zero); c1 = mfma16(W[13], k1, c1);
    f4v c2 = mfma16(W[14], k0, zero); c2 = mfma16(W[15], k1, c2);
    f4v c3 = mfma16(W[16], k0, zero); c3 = mfma16(W[17], k1, c3);
    o = mfma16(W[18], pack_relu(c0, c1), zero);
    o = mfma16(W[19], pack_relu(c2, c3), o);
}

}  // namespace sng
