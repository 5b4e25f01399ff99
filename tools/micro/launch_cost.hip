// Launch cost of back-to-back kernels on one stream (diagnostic): empty kernels of several
// shapes, and a kernel that reads one global counter and exits, timed with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void empty_kernel() {}
__global__ void read_exit(const unsigned *cnt, unsigned *out) {
    if (*cnt == 12345u && threadIdx.x == 0) out[blockIdx.x] = 1;
}
extern "C" __global__ void lds_kernel(const unsigned *cnt, unsigned *out) {
    extern __shared__ unsigned s[];
    if (*cnt == 12345u) { s[threadIdx.x] = 1; __syncthreads(); out[blockIdx.x] = s[0]; }
}

int main() {
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    unsigned *cnt, *out;
    hipMalloc(&cnt, 4);
    hipMalloc(&out, 4096 * 4);
    hipMemset(cnt, 0, 4);
    hipFuncSetAttribute((const void *)lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int R = 200;
    struct Cfg { const char *name; int kind, grid, block; size_t lds; };
    Cfg cfgs[] = {{"empty 1x64", 0, 1, 64, 0},          {"empty 256x1024", 0, 256, 1024, 0},
                  {"read 1x64", 1, 1, 64, 0},           {"read 16x1024", 1, 16, 1024, 0},
                  {"read 256x256", 1, 256, 256, 0},     {"read 256x1024", 1, 256, 1024, 0},
                  {"lds160K 16x1024", 2, 16, 1024, 160 * 1024}, {"lds160K 256x1024", 2, 256, 1024, 160 * 1024}};
    for (const Cfg &c : cfgs) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a, st);
            for (int i = 0; i < R; i++) {
                if (c.kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(c.grid), dim3(c.block), 0, st);
                else if (c.kind == 1) hipLaunchKernelGGL(read_exit, dim3(c.grid), dim3(c.block), 0, st, cnt, out);
                else hipLaunchKernelGGL(lds_kernel, dim3(c.grid), dim3(c.block), c.lds, st, cnt, out);
            }
            hipEventRecord(b, st);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("%-20s %7.2f us per launch\n", c.name, ms * 1000 / R);
        }
    }
    return 0;
}
