// Latency probe: shader cycles per instruction for one wave alone on a SIMD (dependent f32 FMA chain,
// independent chains, a divergent loop with a data-dependent branch, an LDS read chain, a global store
// per iteration).  Calibrates the per-trip cost of the marchers' dependent loops.
// build: hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o /tmp/lat_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(float* out, unsigned long long* cyc, int n, const unsigned* lds_init) {
    __shared__ unsigned lds[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) lds[k] = lds_init[k];
    __syncthreads();
    const int lane = threadIdx.x;
    float a = 1.0f + lane * 1e-7f, b = 0.999999f;
    // 1: dependent FMA chain
    unsigned long long t0 = clock64();
    for (int i = 0; i < n; ++i) { a = fmaf(a, b, 1e-7f); }
    unsigned long long t1 = clock64();
    // 2: four independent chains
    float c0 = a, c1 = a + 1, c2 = a + 2, c3 = a + 3;
    for (int i = 0; i < n; ++i) { c0 = fmaf(c0, b, 1e-7f); c1 = fmaf(c1, b, 1e-7f); c2 = fmaf(c2, b, 1e-7f); c3 = fmaf(c3, b, 1e-7f); }
    unsigned long long t2 = clock64();
    // 3: divergent data-dependent loop (each trip: branch on a per-lane bit, ~10 VALU per side)
    float t = a;
    unsigned k = lane * 2654435761u;
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
        k = k * 1664525u + 1013904223u;
        if (k & 0x100u) { t = t * 1.0001f + 0.5f; t = floorf(t * 0.5f) + t * 0.25f; }
        else { t = t * 0.9999f - 0.25f; t = ceilf(t * 0.25f) - t * 0.125f; }
    }
    unsigned long long t3 = clock64();
    // 4: dependent LDS read chain
    unsigned idx = lane;
#pragma unroll 1
    for (int i = 0; i < n; ++i) idx = lds[idx & 1023];
    unsigned long long t4 = clock64();
    // 5: uniform loop with a global store per trip (fire and forget)
#pragma unroll 1
    for (int i = 0; i < n; ++i) { a = fmaf(a, b, 1e-7f); out[(size_t)i * 64 + lane] = a; }
    unsigned long long t5 = clock64();
    out[(size_t)n * 64 + lane] = a + c0 + c1 + c2 + c3 + t + (float)idx;
    if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4; }
}

int main() {
    const int n = 4096;
    float* out;
    unsigned long long* cyc;
    unsigned* li;
    hipMalloc(&out, (size_t)(n + 1) * 64 * 4);
    hipMalloc(&cyc, 5 * 8);
    unsigned h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = (i * 37 + 11) & 1023;
    hipMalloc(&li, sizeof(h));
    hipMemcpy(li, h, sizeof(h), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, cyc, n, li);
        hipDeviceSynchronize();
    }
    unsigned long long c[5];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, cyc, n, li);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long tot = c[0] + c[1] + c[2] + c[3] + c[4];
    std::printf("{\"n\": %d, \"dep_fma_cyc\": %.2f, \"indep4_fma_cyc_per_iter\": %.2f, \"divergent_trip_cyc\": %.2f, \"lds_chain_cyc\": %.2f, "
                "\"store_trip_cyc\": %.2f, \"kernel_ms\": %.4f, \"clock_ghz_est\": %.3f}\n",
                n, (double)c[0] / n, (double)c[1] / n, (double)c[2] / n, (double)c[3] / n, (double)c[4] / n, ms, tot / (ms * 1e6));
    return 0;
}
