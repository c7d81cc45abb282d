// display.hip -- headless display stage: what Display::present draws into the
// window from the final frame (display.cu:153-303, scripts/virtual_desc/main.frag:24-117) and what
// Display::save_image reads back (display.cu:305-322), as one HIP kernel per frame:
//
//   * main.frag: tex_coords = unwarp((UV.x, 1 - UV.y)) -- the foveation warp is the identity without
//     foveated rendering (the only mode on this path) -- then fxaa(syn_rgba, tex_coords, full_res)
//     (FXAA 3.11 "mobile": 4 diagonal luma taps, REDUCE_MIN 1/128, REDUCE_MUL 1/8, SPAN_MAX 8) with
//     GL_LINEAR / GL_REPEAT sampling of the RGBA32F texture (display.cu:242-247);
//   * blending GL_ONE / GL_ONE_MINUS_SRC_ALPHA over the clear colour (display.cu:269-281);
//   * glReadPixels(GL_RGB, GL_UNSIGNED_BYTE): unorm8 = round(clamp(c, 0, 1) * 255).
// Output rows are top-down (the readback is flipped on write, stbi_flip_vertically_on_write).
#include "sng_internal.h"
#include "sng_math.h"

namespace sng {

// GL_LINEAR + GL_REPEAT texture() on an RGBA32F image (exact bilinear; GL hardware quantises the
// sub-texel weights, so a GL implementation differs by at most ~1 unorm8 step)
__device__ __forceinline__ float4 tex_linear(const float4* __restrict__ img, int W, int H, float u, float v, int ox = 0, int oy = 0) {
    const float x = u * (float)W - 0.5f + (float)ox, y = v * (float)H - 0.5f + (float)oy;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const float ax = x - fx0, ay = y - fy0;
    int x0 = (int)fx0 % W, y0 = (int)fy0 % H;
    if (x0 < 0) x0 += W;
    if (y0 < 0) y0 += H;
    const int x1 = x0 + 1 == W ? 0 : x0 + 1, y1 = y0 + 1 == H ? 0 : y0 + 1;
    const float4 a = img[(size_t)y0 * W + x0], b = img[(size_t)y0 * W + x1], c = img[(size_t)y1 * W + x0], d = img[(size_t)y1 * W + x1];
    const float w00 = (1.0f - ax) * (1.0f - ay), w10 = ax * (1.0f - ay), w01 = (1.0f - ax) * ay, w11 = ax * ay;
    return make_float4(a.x * w00 + b.x * w10 + c.x * w01 + d.x * w11, a.y * w00 + b.y * w10 + c.y * w01 + d.y * w11,
                       a.z * w00 + b.z * w10 + c.z * w01 + d.z * w11, a.w * w00 + b.w * w10 + c.w * w01 + d.w * w11);
}
// textureProjOffset(tex, vec4(uv, 1, 1), ivec2(ox, oy)): the offset is added in texel space
__device__ __forceinline__ float4 tex_offset(const float4* __restrict__ img, int W, int H, float u, float v, int ox, int oy) {
    return tex_linear(img, W, H, u, v, ox, oy);
}
__device__ __forceinline__ float luma(float4 c) { return c.x * 0.299f + c.y * 0.587f + c.z * 0.114f; }

// img: the syn_rgba texture (W x H, the final frame at mesh resolution); output: the window (OW x OH,
// full_resolution) as RGB8, top-down
__global__ __launch_bounds__(256) void display_kernel(const float4* __restrict__ img, int W, int H, int OW, int OH, f3 clear, uint8_t* __restrict__ out) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), row = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= OW || row >= OH) return;
    const int ygl = OH - 1 - row;   // window row from the bottom
    const float u = ((float)x + 0.5f) / (float)OW;
    const float v = 1.0f - ((float)ygl + 0.5f) / (float)OH;   // tex_coords.y = 1.0 - UVs.y
    // fxaa (main.frag:50-97); inverseVP from full_resolution
    const float ivx = 1.0f / (float)OW, ivy = 1.0f / (float)OH;
    const float4 nw = tex_offset(img, W, H, u, v, -1, 1), ne = tex_offset(img, W, H, u, v, 1, 1);
    const float4 sw = tex_offset(img, W, H, u, v, -1, -1), se = tex_offset(img, W, H, u, v, 1, -1);
    const float4 tc = tex_linear(img, W, H, u, v);
    const float lNW = luma(nw), lNE = luma(ne), lSW = luma(sw), lSE = luma(se), lM = luma(tc);
    const float lmin = fminf(lM, fminf(fminf(lNW, lNE), fminf(lSW, lSE)));
    const float lmax = fmaxf(lM, fmaxf(fmaxf(lNW, lNE), fmaxf(lSW, lSE)));
    float dx = -((lNW + lNE) - (lSW + lSE));
    float dy = ((lNW + lSW) - (lNE + lSE));
    const float reduce = fmaxf((lNW + lNE + lSW + lSE) * (0.25f * (1.0f / 8.0f)), 1.0f / 128.0f);
    const float rcp_min = 1.0f / (fminf(fabsf(dx), fabsf(dy)) + reduce);
    dx = fminf(8.0f, fmaxf(-8.0f, dx * rcp_min)) * ivx;
    dy = fminf(8.0f, fmaxf(-8.0f, dy * rcp_min)) * ivy;
    const float k1 = 1.0f / 3.0f - 0.5f, k2 = 2.0f / 3.0f - 0.5f;
    const float4 a1 = tex_linear(img, W, H, u + dx * k1, v + dy * k1), a2 = tex_linear(img, W, H, u + dx * k2, v + dy * k2);
    const f3 rgbA = mk(0.5f * (a1.x + a2.x), 0.5f * (a1.y + a2.y), 0.5f * (a1.z + a2.z));
    const float4 b1 = tex_linear(img, W, H, u + dx * -0.5f, v + dy * -0.5f), b2 = tex_linear(img, W, H, u + dx * 0.5f, v + dy * 0.5f);
    const f3 rgbB = mk(rgbA.x * 0.5f + 0.25f * (b1.x + b2.x), rgbA.y * 0.5f + 0.25f * (b1.y + b2.y), rgbA.z * 0.5f + 0.25f * (b1.z + b2.z));
    const float lB = rgbB.x * 0.299f + rgbB.y * 0.587f + rgbB.z * 0.114f;
    const f3 c = (lB < lmin || lB > lmax) ? rgbA : rgbB;
    // blend GL_ONE, GL_ONE_MINUS_SRC_ALPHA over the clear colour, then unorm8
    const float ia = 1.0f - tc.w;
    const float r = c.x + clear.x * ia, g = c.y + clear.y * ia, b = c.z + clear.z * ia;
    auto u8 = [](float f) { f = fminf(fmaxf(f, 0.0f), 1.0f); return (uint8_t)(int)(f * 255.0f + 0.5f); };
    uint8_t* o = out + 3 * ((size_t)row * OW + x);
    o[0] = u8(r); o[1] = u8(g); o[2] = u8(b);
}

void launch_display(const float4* img, int W, int H, int OW, int OH, f3 clear, uint8_t* out, hipStream_t s) {
    if (W <= 0 || H <= 0 || OW <= 0 || OH <= 0) return;
    hipLaunchKernelGGL(display_kernel, dim3((OW + 15) / 16, (OH + 15) / 16), dim3(256), 0, s, img, W, H, OW, OH, clear, out);
}

// Band composition for multi-GPU frames: the final RGBA32F rows [r0, r1) of the
// frame quantised to RGBA8 (unorm8 = round(clamp(c, 0, 1) * 255), the readback rule above) into a
// contiguous tile, so the RCCL gather moves 4 B/px instead of 16.  One 16-B load, one 4-B store per px.
__global__ __launch_bounds__(256) void rgba8_band_kernel(const float4* __restrict__ img, uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 c = img[i];
    auto u8 = [](float f) { f = fminf(fmaxf(f, 0.0f), 1.0f); return (uint32_t)(int)(f * 255.0f + 0.5f); };
    out[i] = u8(c.x) | (u8(c.y) << 8) | (u8(c.z) << 16) | (u8(c.w) << 24);
}

void launch_rgba8_band(const float4* img, uint32_t n, uint32_t* out, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(rgba8_band_kernel, dim3((n + 255) / 256), dim3(256), 0, s, img, n, out);
}

}  // namespace sng
