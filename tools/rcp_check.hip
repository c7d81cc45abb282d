// Exhaustive check (every float bit pattern) of the reciprocal forms the triangle test could use,
// against IEEE 1.0f / x as the library compiles it (-fno-fast-math: correctly rounded):
//   form 0: y = v_rcp_f32(x); e = fma(-x, y, 1); y + e*y (fma)
// Prints mismatches per biased exponent of x.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//   -fno-fast-math tools/rcp_check.hip -o rcp_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float rcp_fix(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, y, 1.0f);
    return fmaf(e, y, y);
}

__global__ void check(uint32_t hi, unsigned long long* bad, uint32_t* example) {
    const uint32_t lo = blockIdx.x * blockDim.x + threadIdx.x;   // 2^16 per launch slice
    const uint32_t u = (hi << 16) | lo;
    float x;
    memcpy(&x, &u, 4);
    const float a = 1.0f / x, b = rcp_fix(x);
    uint32_t ua, ub;
    memcpy(&ua, &a, 4);
    memcpy(&ub, &b, 4);
    const bool nan_both = (a != a) && (b != b);
    if (ua != ub && !nan_both) {
        const uint32_t ex = (u >> 23) & 0xFFu;
        atomicAdd(bad + ex, 1ull);
        example[ex] = u;
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* ex;
    hipMalloc(&bad, 256 * sizeof(unsigned long long));
    hipMalloc(&ex, 256 * sizeof(uint32_t));
    hipMemset(bad, 0, 256 * sizeof(unsigned long long));
    hipMemset(ex, 0, 256 * sizeof(uint32_t));
    for (uint32_t hi = 0; hi < 65536; ++hi) hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, 0, hi, bad, ex);
    unsigned long long h[256];
    uint32_t he[256];
    hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(he, ex, sizeof(he), hipMemcpyDeviceToHost);
    unsigned long long tot = 0;
    for (int e = 0; e < 256; ++e) {
        tot += h[e];
        if (h[e]) {
            float x;
            memcpy(&x, &he[e], 4);
            printf("exp %3d (2^%d): %llu mismatches, e.g. %08x = %g\n", e, e - 127, h[e], he[e], x);
        }
    }
    printf("total mismatches %llu over 2^32 inputs\n", tot);
    return 0;
}
