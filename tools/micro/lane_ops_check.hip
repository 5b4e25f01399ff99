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
    // two-operand swaps (the search's reduce-scatter): x and y differ
    const unsigned y = x ^ 0xA5A5A5A5u;
    const LanePair s32 = swap32_u32(x, y), s16 = swap16_u32(x, y);
    // every lane runs every shuffle (a shuffle under a divergent ternary reads inactive lanes)
    const unsigned y_m32 = __shfl(y, (lane + 32) & 63), x_p32 = __shfl(x, (lane + 32) & 63);
    const unsigned y_m16 = __shfl(y, (lane + 48) & 63), x_p16 = __shfl(x, (lane + 16) & 63);
    const unsigned e32lo = lane < 32 ? x : y_m32;
    const unsigned e32hi = lane < 32 ? x_p32 : y;
    const bool odd = (lane >> 4) & 1;
    const unsigned e16lo = odd ? y_m16 : x;
    const unsigned e16hi = odd ? y : x_p16;
    out[5 * 64 + lane] = s32.lo == e32lo && s32.hi == e32hi;
    out[6 * 64 + lane] = s16.lo == e16lo && s16.hi == e16hi;
}

int main() {
    unsigned *d, h[7 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    const char *names[7] = {"xor16", "xor32", "prev", "next", "f32", "swap32", "swap16"};
    for (int t = 0; t < 7; t++) {
        int nb = 0;
        for (int l = 0; l < 64; l++) nb += h[t * 64 + l] != 1;
        printf("%s: %s (%d lanes differ)\n", names[t], nb ? "FAIL" : "ok", nb);
        bad += nb;
    }
    return bad ? 1 : 0;
}
