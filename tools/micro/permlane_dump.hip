// Dumps both results of v_permlane32_swap / v_permlane16_swap for x = lane, y = 100 + lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *out) {
    const unsigned l = threadIdx.x, x = l, y = 100 + l;
    const auto a = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    out[l] = a[0]; out[64 + l] = a[1]; out[128 + l] = b[0]; out[192 + l] = b[1];
}
int main() {
    unsigned *d, h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char *n[4] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]"};
    for (int t = 0; t < 4; t++) {
        printf("%s:", n[t]);
        for (int l = 0; l < 64; l++) printf(" %u", h[t * 64 + l]);
        printf("\n");
    }
    return 0;
}
