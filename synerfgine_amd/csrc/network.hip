// network.hip -- fused NeRF field evaluation for gfx950 (CDNA4).
//
// Replaces NerfNetwork<__half>::inference_mixed_precision (nerf_network.h:105-139):
//   tcnn GridEncoding (hash grid, L levels x F features, CoherentPrime hash)
//   -> density FullyFusedMLP 32 -> 64 -> 16 (ReLU hidden, no bias)
//   -> SH degree 4 of the direction (tcnn SphericalHarmonics)
//   -> rgb FullyFusedMLP 32 -> 64 -> 64 -> 16 on [density_out(16) | SH(16)]
//   -> extract_density (row 3 <- density output 0).
// [tcnn semantics restated; tcnn is an unvendored submodule -- DESIGN.md]
//
// One wave evaluates 16 samples per step.  Each lane owns one sample (lane&15)
// and two (F=4) or four (F=2) grid levels (lane>>4), so the 8 fp16 features it
// interpolates ARE its B fragment of v_mfma_f32_16x16x32_f16 (B[k][col]:
// k = 8*(lane>>4)+j, col = lane&15).  Every layer computes OUT^T = W * IN^T so
// samples stay on the MFMA column; the f32 accumulator of one layer becomes the
// next layer's B operand in registers (no LDS): accumulator rows 4*(lane>>4)+i
// of two adjacent 16-row blocks give the 8 k-slots of one 32-deep k step, and
// the host stores each weight matrix's columns in that permuted k order.
// The 20 weight fragments (20 KiB) are staged once per workgroup in LDS and read per layer with
// conflict-free ds_read_b128 (72 VGPRs, 7 waves/SIMD); keeping them resident in 80 VGPRs per wave instead
// (149 VGPRs, 3 waves/SIMD) measured 1.5-2 % slower per launch.
#include <hip/hip_ext.h>

#include "nerf_field.h"

namespace sng {

// OUT_LAYOUT 0: tcnn RM [16][n]; 1: AoS [n][4] (r,g,b,density)
#ifndef NET_WAVES_PER_EU
#define NET_WAVES_PER_EU 3
#endif
template <int F, int OUT_LAYOUT, bool DENS_ONLY = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NET_WAVES_PER_EU))) void nerf_network_kernel(const float* __restrict__ coords, uint32_t stride, uint32_t n_static,
                                                           const uint32_t* __restrict__ n_dev, const h8* __restrict__ wfrag,
                                                           const _Float16* __restrict__ grid, const LevelInfo* __restrict__ levels,
                                                           uint16_t* __restrict__ out, uint32_t out_rows_stride, uint32_t* __restrict__ n_rec) {
    const uint32_t n = n_dev ? *n_dev : n_static;
    if (n_rec && blockIdx.x == 0 && threadIdx.x == 0) *n_rec = n;   // the launch's sample count (per-launch roofline)
    const uint32_t n_tiles = (n + 15) >> 4;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
    const int g = lane >> 4, col = lane & 15;

    __shared__ h8 sW[20 * 64];
    for (int k = threadIdx.x; k < 20 * 64; k += blockDim.x) sW[k] = wfrag[k];
    __syncthreads();
    const LdsWeights W{sW, lane};
    // workgroup slot x = blockIdx % 8 (one XCD under round-robin dispatch: affinity only) walks one
    // contiguous eighth of the tiles, so neighbouring rays' mid-level cells meet in the same L2
    // (measured 1.5 % shorter launches than the grid-wide interleave over all waves)
    uint32_t t_begin = wave, t_end = n_tiles, t_step = n_waves;
    if ((gridDim.x & 7u) == 0) {
        const uint32_t wpb = blockDim.x >> 6, x = blockIdx.x & 7u;
        const uint32_t per = (n_tiles + 7u) >> 3;
        t_begin = x * per + (blockIdx.x >> 3) * wpb + (threadIdx.x >> 6);
        t_end = min(n_tiles, (x + 1u) * per);
        t_step = (gridDim.x >> 3) * wpb;
    }
    for (uint32_t tile = t_begin; tile < t_end; tile += t_step) {
        const uint32_t s = tile * 16 + col;
        const bool valid = s < n;
        const float* c = coords + (size_t)(valid ? s : n - 1) * stride;
        const float x0 = c[0], x1 = c[1], x2 = c[2];
        const float d0 = c[4], d1 = c[5], d2 = c[6];

        f4v o, dens;
        field_tile<F, false, LdsWeights, DENS_ONLY>(W, levels, grid, g, x0, x1, x2, d0, d1, d2, o, dens);

        if (!valid) continue;
        if constexpr (OUT_LAYOUT == 1) {
            if (g == 0) {
                h4 r;
                r[0] = (_Float16)o[0]; r[1] = (_Float16)o[1]; r[2] = (_Float16)o[2]; r[3] = (_Float16)dens[0];
                *reinterpret_cast<h4*>(out + (size_t)s * 4) = r;
            }
        } else {
            // rows 4g+i of the padded rgb output; row 3 <- density (extract_density)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v = (g == 0 && i == 3) ? (float)(_Float16)dens[0] : o[i];
                _Float16 h = (_Float16)v;
                out[(size_t)(4 * g + i) * out_rows_stride + s] = __builtin_bit_cast(uint16_t, h);
            }
        }
    }
}

// Standalone encoding (parity hook): out [n][L*F]
template <int F>
__global__ __launch_bounds__(256) void hashgrid_encode_kernel(const float* __restrict__ coords, uint32_t stride, uint32_t n,
                                                              const _Float16* __restrict__ grid, const LevelInfo* __restrict__ levels,
                                                              uint16_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t s = t >> 2;
    const int g = t & 3;
    if (s >= n) return;
    const float* c = coords + (size_t)s * stride;
    h8 e = encode_lane<F>(levels, grid, g, c[0], c[1], c[2]);
    *reinterpret_cast<h8*>(out + (size_t)s * 32 + g * 8) = e;   // 16-B store of the lane's 8 features
}

// Standalone direction encoding (parity hook): out [n][16] fp16, the SH degree-4 rows the network
// feeds its rgb MLP (sh_lane, one lane per 4 coefficients as in field_tile)
__global__ __launch_bounds__(256) void sh_encode_kernel(const float* __restrict__ coords, uint32_t stride, uint32_t dir_offset, uint32_t n,
                                                        uint16_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t s = t >> 2;
    const int g = t & 3;
    if (s >= n) return;
    const float* d = coords + (size_t)s * stride + dir_offset;
    float sh[4];
    sh_lane(g, d[0], d[1], d[2], sh);
    _Float16 h[4] = {(_Float16)sh[0], (_Float16)sh[1], (_Float16)sh[2], (_Float16)sh[3]};
    *reinterpret_cast<uint2*>(out + (size_t)s * 16 + g * 4) = *reinterpret_cast<const uint2*>(h);   // 8-B store
}

void launch_sh_encode(const float* coords, uint32_t stride, uint32_t dir_offset, uint32_t n, uint16_t* out, hipStream_t stream) {
    if (n == 0) return;
    hipLaunchKernelGGL(sh_encode_kernel, dim3((uint32_t)(((uint64_t)n * 4 + 255) / 256)), dim3(256), 0, stream, coords, stride, dir_offset, n, out);
}

int launch_network(const NetworkDev& net, const float* coords, uint32_t stride, uint32_t n_static, const uint32_t* n_dev,
                   uint16_t* out, int layout, uint32_t max_tiles_hint, hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1, uint32_t* n_rec) {
    uint32_t tiles = n_dev ? max_tiles_hint : (n_static + 15) / 16;
    if (tiles == 0) return 0;
    // persistent-style grid: one occupancy's worth of waves (7/SIMD), never more than the tiles
    uint32_t max_waves = (uint32_t)net.n_cus * 28u;
    uint32_t waves = tiles < max_waves ? tiles : max_waves;
    uint32_t blocks = (waves + 3) / 4;
    blocks = (blocks + 7u) & ~7u;   // whole XCD slots
    const h8* w = reinterpret_cast<const h8*>(net.wfrag);
    const _Float16* gr = reinterpret_cast<const _Float16*>(net.grid);
    auto go = [&](auto kernel) {
        if (ev0 || ev1)
            hipExtLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, stream, ev0, ev1, 0u, coords, stride, n_static, n_dev, w, gr, net.levels, out, n_static, n_rec);
        else
            hipLaunchKernelGGL(kernel, dim3(blocks), dim3(256), 0, stream, coords, stride, n_static, n_dev, w, gr, net.levels, out, n_static, n_rec);
    };
    // layout 2: [n][4] with the density only (rgb 0; NerfNetwork::density for the density-grid update)
    if (net.F == 4) {
        if (layout == 2) go(nerf_network_kernel<4, 1, true>);
        else if (layout == 1) go(nerf_network_kernel<4, 1>);
        else go(nerf_network_kernel<4, 0>);
    } else {
        if (layout == 2) go(nerf_network_kernel<2, 1, true>);
        else if (layout == 1) go(nerf_network_kernel<2, 1>);
        else go(nerf_network_kernel<2, 0>);
    }
    return 0;
}

// ---------------------------------------------------------------------------------------------
// Testbed::render_nerf's extra network passes (testbed_nerf.cu:2363-2366).  tcnn is called with the
// network input matrix as its own output, so the samples' NerfCoordinates are rewritten in place and
// composite_kernel_nerf then reads the result as "warped_pos" (and dt):
//   Normals     (2): NerfNetwork::input_gradient(dim 3): rows 0-2 = d(raw density)/d(warped position)
//                    (density MLP backward -> GridEncoding input gradient, kernel_grid's dy_dx with
//                    linear interpolation), rows 4-6 = 0 (the direction feeds only rgb), row 3 untouched;
//   EncodingVis (10): visualize_activation(layer, dim) (tcnn extract_dimension_pos_neg_kernel over a
//                    7-row output): (max(-v, 0), max(v, 0), 0, 1, 1, 1, 1), v = activation `dim` of
//                    NerfNetwork layer `layer` (0 encoding, 1 density hidden, 2 rgb-network input,
//                    3-4 rgb hidden).
// One thread per sample with plain f32 arithmetic (the oracle's dense() accumulation order) (tcnn backpropagates in fp16 with a 128 loss scale;
// after normalize() the direction differs by O(1e-3)); activations are the fp16 values tcnn keeps.
// Not a hot path: only these two render modes run it.
template <int F>
__global__ __launch_bounds__(128) void field_probe_kernel(float* __restrict__ coords, const uint32_t* __restrict__ n_dev,
                                                          const uint16_t* __restrict__ mlp, const _Float16* __restrict__ grid,
                                                          const LevelInfo* __restrict__ levels, int n_levels, int mode, int layer, int dim) {
    const uint32_t n = *n_dev;
    const _Float16* W = reinterpret_cast<const _Float16*>(mlp);
    const _Float16* dW0 = W;                 // density [64][32]
    const _Float16* dW1 = W + 64 * 32;       // density [16][64]
    const _Float16* cW0 = dW1 + 16 * 64;     // rgb [64][32]
    const _Float16* cW1 = cW0 + 64 * 32;     // rgb [64][64]
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n; s += gridDim.x * blockDim.x) {
        float* c = coords + (size_t)s * 7;
        const float x0 = c[0], x1 = c[1], x2 = c[2];
        _Float16 enc[32];
        for (int l = 0; l < n_levels; ++l) encode_level<F>(levels[l], grid, x0, x1, x2, enc + l * F);
        _Float16 hid[64];
        float gh[64];
        for (int j = 0; j < 64; ++j) {
            float a = 0.0f;
            for (int i = 0; i < 32; ++i) a += (float)dW0[j * 32 + i] * (float)enc[i];
            hid[j] = (_Float16)fmaxf(a, 0.0f);
        }
        if (mode == 2) {
            // d(raw density) / d(hidden) = W1[0][j] where the ReLU passed, then / d(encoding) = W0^T
            for (int j = 0; j < 64; ++j) gh[j] = (float)hid[j] > 0.0f ? (float)dW1[j] : 0.0f;
            float g[3] = {0.0f, 0.0f, 0.0f};
            for (int l = 0; l < n_levels; ++l) {
                float ge[F];
                for (int f = 0; f < F; ++f) {
                    float a = 0.0f;
                    for (int j = 0; j < 64; ++j) a = fmaf((float)dW0[j * 32 + l * F + f], gh[j], a);
                    ge[f] = a;
                }
                const LevelInfo L = levels[l];
                const float xs[3] = {x0, x1, x2};
                float fr[3];
                uint32_t gi[3];
                for (int d = 0; d < 3; ++d) {
                    const float p = fmaf(L.scale, xs[d], 0.5f);
                    const float q = floorf(p);
                    gi[d] = (uint32_t)(int)q;
                    fr[d] = p - q;
                }
                const _Float16* tbl = grid + (size_t)L.offset * F;
                // kernel_grid dy_dx: for each axis, the 4 edges along it weighted by the other two axes
                for (int gd = 0; gd < 3; ++gd) {
                    const int da = gd == 0 ? 1 : 0, db = gd == 2 ? 1 : 2;
                    for (int e = 0; e < 4; ++e) {
                        float w = L.scale;
                        uint32_t cc[3];
                        cc[da] = gi[da] + (e & 1); w *= (e & 1) ? fr[da] : 1.0f - fr[da];
                        cc[db] = gi[db] + ((e >> 1) & 1); w *= (e & 2) ? fr[db] : 1.0f - fr[db];
                        cc[gd] = gi[gd];
                        const uint32_t il = grid_index(L, cc[0], cc[1], cc[2]) * F;
                        cc[gd] = gi[gd] + 1;
                        const uint32_t ir = grid_index(L, cc[0], cc[1], cc[2]) * F;
                        for (int f = 0; f < F; ++f) g[gd] += ge[f] * (w * ((float)tbl[ir + f] - (float)tbl[il + f]));
                    }
                }
            }
            c[0] = g[0]; c[1] = g[1]; c[2] = g[2];
            c[4] = 0.0f; c[5] = 0.0f; c[6] = 0.0f;
        } else {
            float v = 0.0f;
            if (layer == 0) {
                v = (float)enc[dim];
            } else if (layer == 1) {
                v = (float)hid[dim];
            } else {
                // rgb-network input: the density MLP's 16 outputs (no output activation), then SH degree 4
                _Float16 rin[32];
                for (int k = 0; k < 16; ++k) {
                    float a = 0.0f;
                    for (int j = 0; j < 64; ++j) a += (float)dW1[k * 64 + j] * (float)hid[j];
                    rin[k] = (_Float16)a;
                }
                for (int g4 = 0; g4 < 4; ++g4) {
                    float o[4];
                    sh_lane(g4, c[4], c[5], c[6], o);
                    for (int q = 0; q < 4; ++q) rin[16 + 4 * g4 + q] = (_Float16)o[q];
                }
                if (layer == 2) {
                    v = (float)rin[dim];
                } else {
                    _Float16 h1[64];
                    for (int j = 0; j < 64; ++j) {
                        float a = 0.0f;
                        for (int i = 0; i < 32; ++i) a += (float)cW0[j * 32 + i] * (float)rin[i];
                        h1[j] = (_Float16)fmaxf(a, 0.0f);
                    }
                    if (layer == 3) {
                        v = (float)h1[dim];
                    } else {
                        float a = 0.0f;
                        for (int i = 0; i < 64; ++i) a += (float)cW1[dim * 64 + i] * (float)h1[i];
                        v = (float)(_Float16)fmaxf(a, 0.0f);
                    }
                }
            }
            c[0] = fmaxf(-v, 0.0f); c[1] = fmaxf(v, 0.0f); c[2] = 0.0f;
            c[3] = 1.0f; c[4] = 1.0f; c[5] = 1.0f; c[6] = 1.0f;
        }
    }
}

void launch_field_probe(const NetworkDev& net, const uint16_t* mlp_params, float* coords, const uint32_t* n_dev, int mode, int layer, int dim,
                        hipStream_t stream) {
    const uint32_t blocks = (uint32_t)net.n_cus * 8;
    const _Float16* gr = reinterpret_cast<const _Float16*>(net.grid);
    if (net.F == 4) hipLaunchKernelGGL((field_probe_kernel<4>), dim3(blocks), dim3(128), 0, stream, coords, n_dev, mlp_params, gr, net.levels, net.L, mode, layer, dim);
    else hipLaunchKernelGGL((field_probe_kernel<2>), dim3(blocks), dim3(128), 0, stream, coords, n_dev, mlp_params, gr, net.levels, net.L, mode, layer, dim);
}

int launch_encode(const NetworkDev& net, const float* coords, uint32_t stride, uint32_t n, uint16_t* out, hipStream_t stream) {
    if (n == 0) return 0;
    uint32_t blocks = (n * 4 + 255) / 256;
    const _Float16* gr = reinterpret_cast<const _Float16*>(net.grid);
    if (net.F == 4) hipLaunchKernelGGL((hashgrid_encode_kernel<4>), dim3(blocks), dim3(256), 0, stream, coords, stride, n, gr, net.levels, out);
    else hipLaunchKernelGGL((hashgrid_encode_kernel<2>), dim3(blocks), dim3(256), 0, stream, coords, stride, n, gr, net.levels, out);
    return 0;
}

}  // namespace sng
