// Durations of early-exit kernels by grid, block and LDS size, each after a large writer (read
// them from a rocprofv3 kernel trace): what the per-level tail launches cost on their own.
//   hipcc --offload-arch=gfx950 -O3 launch_grid.hip -o launch_grid
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void writer(uint64_t *p, uint64_t n, unsigned *cnt) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = i;
    if (threadIdx.x == 0) atomicAdd(cnt, 1u);
}
template <int TAG>
__global__ void exit_k(const unsigned *cnt, unsigned *out) {
    extern __shared__ unsigned sm[];
    if (*cnt == 12345u && threadIdx.x == 0) { sm[0] = 1; out[blockIdx.x] = sm[0]; }
}
template <int TAG>
__global__ void sysfence_k(const unsigned *cnt, unsigned *out, volatile uint64_t *host) {
    if (threadIdx.x == 0) {
        out[blockIdx.x] = *cnt;
        __threadfence_system();
        *host = 1;
    }
}
int main() {
    uint64_t n = 1ull << 24;
    uint64_t *p; unsigned *cnt, *out; uint64_t *h;
    hipMalloc(&p, n * 8); hipMalloc(&cnt, 4); hipMalloc(&out, 4096 * 4);
    hipHostMalloc(&h, 64, hipHostMallocMapped);
    hipStream_t st; hipStreamCreate(&st);
    for (int rep = 0; rep < 20; rep++) {
#define W hipLaunchKernelGGL(writer, dim3(256), dim3(1024), 0, st, p, n, cnt)
        W; hipLaunchKernelGGL(exit_k<1>, dim3(1), dim3(64), 0, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<2>, dim3(1), dim3(1024), 0, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<3>, dim3(16), dim3(1024), 0, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<4>, dim3(65), dim3(1024), 0, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<5>, dim3(256), dim3(1024), 0, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<6>, dim3(65), dim3(1024), 64 * 1024, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<7>, dim3(256), dim3(1024), 100 * 1024, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<8>, dim3(8), dim3(1024), 64 * 1024, st, cnt, out);
        W; hipLaunchKernelGGL(exit_k<9>, dim3(2), dim3(256), 0, st, cnt, out);
        W; hipLaunchKernelGGL(sysfence_k<1>, dim3(1), dim3(64), 0, st, cnt, out, h);
        W; hipLaunchKernelGGL(sysfence_k<2>, dim3(1), dim3(256), 0, st, cnt, out, h);
        hipLaunchKernelGGL(exit_k<10>, dim3(1), dim3(64), 0, st, cnt, out);   // back to back, no writer
        hipLaunchKernelGGL(exit_k<11>, dim3(1), dim3(64), 0, st, cnt, out);
    }
    hipStreamSynchronize(st);
    printf("done\n");
    return 0;
}
