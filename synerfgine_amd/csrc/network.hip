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
// conflict-free ds_read_b128 (72 VGPRs, 7 waves/SIMD); -DNET_W_REGS keeps them resident in 80 VGPRs
// per wave instead (149 VGPRs, 3 waves/SIMD), measured 1.5-2 % slower per launch.
#include "nerf_field.h"

namespace sng {

// OUT_LAYOUT 0: tcnn RM [16][n]; 1: AoS [n][4] (r,g,b,density)
#ifndef NET_WAVES_PER_EU
#define NET_WAVES_PER_EU 3
#endif
template <int F, int OUT_LAYOUT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NET_WAVES_PER_EU))) void nerf_network_kernel(const float* __restrict__ coords, uint32_t stride, uint32_t n_static,
                                                           const uint32_t* __restrict__ n_dev, const h8* __restrict__ wfrag,
                                                           const _Float16* __restrict__ grid, const LevelInfo* __restrict__ levels,
                                                           uint16_t* __restrict__ out, uint32_t out_rows_stride) {
    const uint32_t n = n_dev ? *n_dev : n_static;
    const uint32_t n_tiles = (n + 15) >> 4;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
#ifdef NET_W_REGS
    if (wave >= n_tiles) return;
#endif
    const int g = lane >> 4, col = lane & 15;

#ifndef NET_W_REGS
    __shared__ h8 sW[20 * 64];
    for (int k = threadIdx.x; k < 20 * 64; k += blockDim.x) sW[k] = wfrag[k];
    __syncthreads();
    const LdsWeights W{sW, lane};
#else
    h8 W[20];
#pragma unroll
    for (int f = 0; f < 20; ++f) W[f] = wfrag[f * 64 + lane];
#endif
#ifndef NET_XCD_INTERLEAVED
    // workgroup slot x = blockIdx % 8 (one XCD under round-robin dispatch: affinity only) walks one
    // contiguous eighth of the tiles, so neighbouring rays' mid-level cells meet in the same L2
    // (measured 1.5 % shorter launches than the grid-wide interleave)
    uint32_t t_begin = wave, t_end = n_tiles, t_step = n_waves;
    if ((gridDim.x & 7u) == 0) {
        const uint32_t wpb = blockDim.x >> 6, x = blockIdx.x & 7u;
        const uint32_t per = (n_tiles + 7u) >> 3;
        t_begin = x * per + (blockIdx.x >> 3) * wpb + (threadIdx.x >> 6);
        t_end = min(n_tiles, (x + 1u) * per);
        t_step = (gridDim.x >> 3) * wpb;
    }
    for (uint32_t tile = t_begin; tile < t_end; tile += t_step) {
#else
    for (uint32_t tile = wave; tile < n_tiles; tile += n_waves) {
#endif
        const uint32_t s = tile * 16 + col;
        const bool valid = s < n;
        const float* c = coords + (size_t)(valid ? s : n - 1) * stride;
        const float x0 = c[0], x1 = c[1], x2 = c[2];
        const float d0 = c[4], d1 = c[5], d2 = c[6];

        f4v o, dens;
        field_tile<F>(W, levels, grid, g, x0, x1, x2, d0, d1, d2, o, dens);

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

int launch_network(const NetworkDev& net, const float* coords, uint32_t stride, uint32_t n_static, const uint32_t* n_dev,
                   uint16_t* out, int layout, uint32_t max_tiles_hint, hipStream_t stream) {
    uint32_t tiles = n_dev ? max_tiles_hint : (n_static + 15) / 16;
    if (tiles == 0) return 0;
    // persistent-style grid: one occupancy's worth of waves (3/SIMD with register weights, 7/SIMD with
    // LDS weights), never more than the tiles
#ifndef NET_GRID_WAVES_PER_CU
#ifdef NET_W_REGS
#define NET_GRID_WAVES_PER_CU 12u
#else
#define NET_GRID_WAVES_PER_CU 28u
#endif
#endif
    uint32_t max_waves = (uint32_t)net.n_cus * NET_GRID_WAVES_PER_CU;
    uint32_t waves = tiles < max_waves ? tiles : max_waves;
    uint32_t blocks = (waves + 3) / 4;
#ifndef NET_XCD_INTERLEAVED
    blocks = (blocks + 7u) & ~7u;   // whole XCD slots
#endif
    const h8* w = reinterpret_cast<const h8*>(net.wfrag);
    const _Float16* gr = reinterpret_cast<const _Float16*>(net.grid);
    if (net.F == 4) {
        if (layout == 1) hipLaunchKernelGGL((nerf_network_kernel<4, 1>), dim3(blocks), dim3(256), 0, stream, coords, stride, n_static, n_dev, w, gr, net.levels, out, n_static);
        else hipLaunchKernelGGL((nerf_network_kernel<4, 0>), dim3(blocks), dim3(256), 0, stream, coords, stride, n_static, n_dev, w, gr, net.levels, out, n_static);
    } else {
        if (layout == 1) hipLaunchKernelGGL((nerf_network_kernel<2, 1>), dim3(blocks), dim3(256), 0, stream, coords, stride, n_static, n_dev, w, gr, net.levels, out, n_static);
        else hipLaunchKernelGGL((nerf_network_kernel<2, 0>), dim3(blocks), dim3(256), 0, stream, coords, stride, n_static, n_dev, w, gr, net.levels, out, n_static);
    }
    return 0;
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
