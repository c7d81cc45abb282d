// overlay.hip -- the depth composite of the two layers and the tonemap curve (overlay_nerf, raytracer.cu:220-258;
// sng_tonemap, synerfgine/common.cu:186-243).  Its own translation unit: mesh.hip is built with FMA contraction (the
// reference's --use_fast_math arithmetic), this one without, so the composite and the curves stay bit-exact against the
// oracle's restatement (tests/test_gpu_literal.py test_tonemap_curve_matches_oracle).
#include "sng_internal.h"
#include "sng_math.h"

namespace sng {

// ---------------------------------------------------------------------------
// overlay_nerf (raytracer.cu:220-258) with sng_tonemap (synerfgine/common.cu:186-243)
// ---------------------------------------------------------------------------
// ETonemapCurve (common.h:113): 0 Identity, 1 ACES, 2 Hable, 3 Reinhard.  The rational curves' constants are the
// reference's float expressions (folded at compile time); the per-pixel division is IEEE (-fno-fast-math).
__device__ __forceinline__ f3 sng_tonemap(f3 x, int curve) {
    if (curve == 0) return x;
    x = mk(fmaxf(x.x, 0.0f), fmaxf(x.y, 0.0f), fmaxf(x.z, 0.0f));
    float k0, k1, k2, k3, k4, k5;
    if (curve == 1) {
        k0 = 0.6f * 0.6f * 2.51f;
        k1 = 0.6f * 0.03f;
        k2 = 0.0f;
        k3 = 0.6f * 0.6f * 2.43f;
        k4 = 0.6f * 0.59f;
        k5 = 0.14f;
    } else if (curve == 2) {
        constexpr float A = 0.15f, B = 0.50f, C = 0.10f, D = 0.20f, E = 0.02f, F = 0.30f;
        constexpr float h0 = A * F - A * E, h1 = C * B * F - B * E, h2 = 0.0f, h3 = A * F, h4 = B * F, h5 = D * F * F;
        constexpr float W = 11.2f;
        constexpr float nom = h0 * (W * W) + h1 * W + h2;
        constexpr float denom = h3 * (W * W) + h4 * W + h5;
        constexpr float white_scale = denom / nom;
        k0 = 4.0f * h0 * white_scale;
        k1 = 2.0f * h1 * white_scale;
        k2 = h2 * white_scale;
        k3 = 4.0f * h3;
        k4 = 2.0f * h4;
        k5 = h5;
    } else {
        const float Y = 0.2126f * x.x + 0.7152f * x.y + 0.0722f * x.z;
        return x * (1.f / (Y + 1.0f));
    }
    const f3 sq = x * x;
    const f3 nom = sq * k0 + x * k1 + k2;
    const f3 den = sq * k3 + x * k4 + k5;
    return mk(nom.x / den.x, nom.y / den.y, nom.z / den.z);
}

__global__ void overlay_kernel(int W, int row0, int row1, int scale, int nerf_w, int n_nerf, int show_nerf, float depth_offset, float exposure_mul, int srgb,
                               int tonemap, const float4* __restrict__ syn_rgba, const float* __restrict__ syn_depth, const float4* __restrict__ nerf_rgba,
                               const float* __restrict__ nerf_depth, float4* __restrict__ final_rgba, float* __restrict__ final_depth) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = (uint32_t)(row1 - row0) * (uint32_t)W;
    if (t >= n) return;
    const int x = (int)(t % (uint32_t)W), y = row0 + (int)(t / (uint32_t)W);
    const int sid = x + y * W;
    // nerf_res = syn_res / syn_px_scale as in the reference (raytracer.cu:242-246); an index past the NeRF buffer
    // (a window not divisible by the scale: the reference reads out of bounds) is clamped for memory safety
    const int nid = min((x / scale) + (y / scale) * nerf_w, n_nerf - 1);
    const float sdepth = syn_depth[sid];
    const float4 use = (!show_nerf || sdepth - depth_offset < nerf_depth[nid]) ? syn_rgba[sid] : nerf_rgba[nid];
    f3 c = sng_tonemap(mk(use.x * exposure_mul, use.y * exposure_mul, use.z * exposure_mul), tonemap);
    if (srgb) c = mk(linear_to_srgb(c.x), linear_to_srgb(c.y), linear_to_srgb(c.z));
    final_rgba[sid] = make_float4(c.x, c.y, c.z, use.w);
    final_depth[sid] = sdepth;
}

void launch_overlay(int W, int row0, int row1, int scale, int nerf_w, int n_nerf, int show_nerf, float depth_offset, float exposure_mul, int srgb,
                    int tonemap, const float4* syn, const float* synd, const float4* nerf, const float* nerfd, float4* fin, float* find, hipStream_t s) {
    const uint32_t n = (uint32_t)(row1 - row0) * (uint32_t)W;
    if (!n) return;
    hipLaunchKernelGGL(overlay_kernel, dim3((n + 255) / 256), dim3(256), 0, s, W, row0, row1, scale, nerf_w, n_nerf, show_nerf, depth_offset, exposure_mul,
                       srgb, tonemap, syn, synd, nerf, nerfd, fin, find);
}

}  // namespace sng
