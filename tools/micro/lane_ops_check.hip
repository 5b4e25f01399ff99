// Checks the cross-lane helpers of quant_amd/csrc/mfma_util.hpp (permlane swaps, DPP wave
// shifts) against __shfl_xor / __shfl_up / __shfl_down on the GPU.  Exit 0 = all equal.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../quant_amd/csrc/mfma_util.hpp"
using namespace qvq;

__global__ void k(unsigned *out) {
    const int lane = threadIdx.x;
    const unsigned x = lane * 2654435761u + 12345u;
    out[0 * 64 + lane] = xor16_u32(x) == (unsigned)__shfl_xor(x, 16);
    out[1 * 64 + lane] = xor32_u32(x) == (unsigned)__shfl_xor(x, 32);
    out[2 * 64 + lane] = wave_prev_u32(x) == (unsigned)__shfl_up(x, 1);
    out[3 * 64 + lane] = wave_next_u32(x) == (unsigned)__shfl_down(x, 1);
    const float f = (float)x * 1e-3f;
    out[4 * 64 + lane] = xor16_f32(f) == __shfl_xor(f, 16) && xor32_f32(f) == __shfl_xor(f, 32);
}

int main() {
    unsigned *d, h[5 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    const char *names[5] = {"xor16", "xor32", "prev", "next", "f32"};
    for (int t = 0; t < 5; t++) {
        int nb = 0;
        for (int l = 0; l < 64; l++) nb += h[t * 64 + l] != 1;
        printf("%s: %s (%d lanes differ)\n", names[t], nb ? "FAIL" : "ok", nb);
        bad += nb;
    }
    return bad ? 1 : 0;
}
