// Streaming-read ceiling on this GPU for the access shapes the engine uses (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int UNROLL>
__global__ void rd(const uint4 *__restrict__ p, uint64_t n16, uint32_t *out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[u] = p[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

// per-lane contiguous ranges (the small-kernel shape)
__global__ void rd_lane(const uint4 *__restrict__ p, uint64_t n16, uint64_t per_lane, uint32_t *out) {
    uint32_t acc = 0;
    const uint64_t first = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * per_lane;
    for (uint64_t i = first; i < first + per_lane && i < n16; i++) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t bytes = 50331648ull + 16777216ull;   // codes + indices at C3
    const uint64_t n16 = bytes / 16;
    uint4 *p; uint32_t *o;
    hipMalloc(&p, bytes); hipMalloc(&o, 4);
    hipMemset(p, 1, bytes);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 3; w++) launch();
        hipEventRecord(a);
        for (int r = 0; r < 20; r++) launch();
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-40s %8.1f us  %7.0f GB/s\n", name, ms * 1000 / 20, bytes / (ms / 20 * 1e-3) / 1e9);
    };
    run("grid 256x1024 unroll1", [&] { hipLaunchKernelGGL(rd<1>, dim3(256), dim3(1024), 0, 0, p, n16, o); });
    run("grid 256x1024 unroll4", [&] { hipLaunchKernelGGL(rd<4>, dim3(256), dim3(1024), 0, 0, p, n16, o); });
    run("grid 1024x1024 unroll4", [&] { hipLaunchKernelGGL(rd<4>, dim3(1024), dim3(1024), 0, 0, p, n16, o); });
    run("grid 2048x256 unroll4", [&] { hipLaunchKernelGGL(rd<4>, dim3(2048), dim3(256), 0, 0, p, n16, o); });
    run("grid 8192x256 unroll4", [&] { hipLaunchKernelGGL(rd<4>, dim3(8192), dim3(256), 0, 0, p, n16, o); });
    run("grid n16/256 x256 unroll1", [&] { hipLaunchKernelGGL(rd<1>, dim3((n16 + 255) / 256), dim3(256), 0, 0, p, n16, o); });
    run("lane ranges 256x1024 (16 per lane)", [&] { hipLaunchKernelGGL(rd_lane, dim3(256), dim3(1024), 0, 0, p, n16, (n16 + 262143) / 262144, o); });
    return 0;
}
