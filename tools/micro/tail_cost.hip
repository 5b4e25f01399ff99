// Durations of small dependent kernels after a large writer (diagnostic; read the numbers
// from a rocprofv3 kernel trace): what a per-level tail launch costs on its own.
//   hipcc --offload-arch=gfx950 -O3 tail_cost.hip -o tail_cost
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void writer(uint64_t *p, uint64_t n, unsigned *cnt) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = i;
    if (threadIdx.x == 0) atomicAdd(cnt, 1u);
}
// reads the counter and exits (the no-ties kd_resolve / no-flags recheck case)
__global__ void read_exit_a(const unsigned *cnt, unsigned *out) {
    if (*cnt == 12345u && threadIdx.x == 0) out[blockIdx.x] = 1;
}
__global__ void read_exit_b(const unsigned *cnt, unsigned *out) {
    if (*cnt == 12345u && threadIdx.x == 0) out[blockIdx.x] = 1;
}
__global__ void empty_a() {}
__global__ void empty_b() {}
// 16 loads per thread from the written buffer, block-reduce, one store (the reduce shape)
__global__ void gather16(const uint64_t *p, uint64_t stride, uint64_t *out) {
    uint64_t v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = p[(uint64_t)u * stride + blockIdx.x * 64 + (threadIdx.x & 63)];
    uint64_t s = 0;
#pragma unroll
    for (int u = 0; u < 16; u++) s += v[u];
    if (s == 42) out[threadIdx.x] = s;
}
// one store to mapped host memory after a system fence (the ready publication)
__global__ void publish(volatile uint64_t *host, uint64_t seq) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        *host = seq;
    }
}
// atomic ticket, the last block stores (the finalize's last-block pattern)
__global__ void ticket(unsigned *done, uint64_t *out) {
    __shared__ bool last;
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
        *done = 0;
        out[0] = 1;
    }
}

int main() {
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const uint64_t n = 25ull << 20 >> 3;   // 25 MB
    uint64_t *p, *out;
    unsigned *cnt, *done;
    hipMalloc(&p, n * 8);
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cnt, 4);
    hipMalloc(&done, 4);
    hipMemset(cnt, 0, 4);
    hipMemset(done, 0, 4);
    uint64_t *h;
    hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
    uint64_t *dh;
    hipHostGetDevicePointer((void **)&dh, h, 0);
    for (int rep = 0; rep < 20; rep++) {
        // A: writer then empty x2
        hipLaunchKernelGGL(writer, dim3(256), dim3(1024), 0, st, p, n, cnt);
        hipLaunchKernelGGL(empty_a, dim3(1), dim3(64), 0, st);
        hipLaunchKernelGGL(empty_b, dim3(1), dim3(64), 0, st);
        // B: writer then read_exit 16x1024, then read_exit 1x64
        hipLaunchKernelGGL(writer, dim3(256), dim3(1024), 0, st, p, n, cnt);
        hipLaunchKernelGGL(read_exit_a, dim3(16), dim3(1024), 0, st, cnt, (unsigned *)out);
        hipLaunchKernelGGL(read_exit_b, dim3(1), dim3(64), 0, st, cnt, (unsigned *)out);
        // C: writer then gather16 (1 block and 208 blocks)
        hipLaunchKernelGGL(writer, dim3(256), dim3(1024), 0, st, p, n, cnt);
        hipLaunchKernelGGL(gather16, dim3(1), dim3(1024), 0, st, p, (uint64_t)24 * 1024, out);
        hipLaunchKernelGGL(gather16, dim3(208), dim3(1024), 0, st, p, (uint64_t)13 * 1024 * 8, out);
        // D: publish and ticket
        hipLaunchKernelGGL(publish, dim3(1), dim3(64), 0, st, (volatile uint64_t *)dh, (uint64_t)rep);
        hipLaunchKernelGGL(ticket, dim3(128), dim3(256), 0, st, done, out);
        hipLaunchKernelGGL(ticket, dim3(1), dim3(256), 0, st, done, out);
    }
    hipStreamSynchronize(st);
    printf("done %llu\n", (unsigned long long)*h);
    return 0;
}
