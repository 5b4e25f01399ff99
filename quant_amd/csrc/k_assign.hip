// k_assign.hip -- nearest-code-vector search (src/Quantizer.cpp:24-32 semantics).
//
//  assign_small_kernel D = 12, K <= 32: expanded fp32 scores per code vector; exact centroid
//                      sums in per-lane register runs (LDS copies).  K >= 64 runs the
//                      32x32x16 MFMA search of k_mf32.hip (launch_assign_mfma dispatches).
//  assign_valu_kernel  any Dp <= 64, fp32 direct form (x-c)^2 with an fp32 error bound.
//  recheck_kernel      fp64 distances of flagged rows in the reference build's order.
#include <cstdlib>

#include "common.hpp"
#include "mfma_util.hpp"
#include "kd_walk.hpp"

namespace qvq {


// =======================================================================================
// MFMA search
// =======================================================================================
constexpr int MF_LDS_MAX = 160 * 1024;

struct MfLds {
    uint32_t c32, sums, cnt, plut, total;
};
// LDS carve-up: code-vector rows (Kp x 56 B + 16 B pad) | [fp32 codebook Kp x 48 B] |
// [sums K x 12 x 8 B | counts | term LUT 256 x 8 B].  Kp = K rounded up to 32 (tile pairs).
__host__ __device__ inline MfLds mf_lds_layout(uint32_t K, bool fuse, bool staged) {
    const uint32_t Kp = (K + 31) & ~31u;
    MfLds L;
    uint32_t o = Kp * MF_ROW_BYTES + 16;
    L.c32 = o;
    if (staged) o += Kp * MF_D * 4;
    L.sums = o;
    if (fuse) o += K * MF_D * 8;
    L.cnt = o;
    if (fuse) o += ((K + 1) & ~1u) * 4;
    L.plut = o;
    if (fuse) o += 256 * 8;
    L.total = o;
    return L;
}
uint32_t mf_fuse_max_k() {
    uint32_t K = 32;
    while (mf_lds_layout(2 * K, true, false).total <= MF_LDS_MAX) K *= 2;
    return K;
}
bool mf_can_search(uint32_t K) { return mf_lds_layout(K, false, false).total <= MF_LDS_MAX; }


typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int MF_SMALL_K = 32;

// ---------------------------------------------------------------------------------------
// Small codebooks (K <= MF_SMALL_K): direct fp32 scan of all SK code vectors per row, rows in
// per-lane runs.  Each wave owns a contiguous range of rows; lane L takes every 64th row of
// it (coalesced loads and stores), four rows per iteration.  At small K a lane's consecutive
// rows (64 blocks apart in the image) mostly share their code vector: their exact terms
// (u << 16 | lo per component, no carry within 256 rows) are added in registers and go to the
// LDS sums only when the index changes.  Flag rule and sums as in assign_mf32_kernel.
// ---------------------------------------------------------------------------------------
__host__ __device__ constexpr uint32_t small_copy_stride(uint32_t SK) { return SK * (MF_D + 1) + 1; }
// Copies of the small kernel's sums: up to 64 (one per lane) while they fit ~112 KB of LDS.
static uint32_t small_copies(uint32_t SK) {
    uint32_t C = 64;
    while (C > 1 && (size_t)C * small_copy_stride(SK) * 8 + 256 > MF_LDS_MAX / 2 + 32 * 1024) C /= 2;
    return C;
}
static size_t small_lds(uint32_t SK, uint32_t C) { return (size_t)C * small_copy_stride(SK) * 8 + 256; }

// PACK: the run registers hold two components per register and part.  For word q of a row
// (components 4q..4q+3, u = byte ^ 0x80): au[2q] += u bytes 0 and 2 as 16-bit fields, au[2q+1]
// += bytes 1 and 3 (one v_and / v_perm of the centred word each, no per-component extract), and
// al[2q], al[2q+1] the lo8 lookups of the same pairs.  A run holds <= 256 rows, so every field
// stays below 2^16.  ~14 VALU per row fewer than one (u << 16 | lo) register per component.
template <int SK, bool FUSE, bool PACK, int NW>
__global__ __launch_bounds__(NW * 64) void assign_small_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, uint32_t K, const float *__restrict__ g_E32,
    const uint64_t *__restrict__ g_plut, MfThresholds th, uint64_t rows_per_lane, uint32_t copies,
    uint32_t *__restrict__ A, uint32_t *__restrict__ flags, unsigned *__restrict__ flag_cnt,
    uint64_t *__restrict__ part, uint32_t *__restrict__ part_cnt, uint64_t *__restrict__ z1, uint32_t nz1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // LDS: lo8 (256 B, first: a byte's lookup address is the byte itself, no base add) | C
    // copies of the sums, copy c = [d][k] (SK*D u64) then counts [k] (SK u64), stride
    // S = SK*(D+1) + 1 (odd: the copies of 16 consecutive lanes sit on different banks).
    // SK-strided, so a flush addresses copy + d*SK + cur with immediate offsets.
    // Lane L flushes into copy L mod C, so the flushes of a wave's lanes -- all at once at
    // the end, mostly to the same code vector at small K -- rarely hit one address.
    constexpr uint32_t S = small_copy_stride(SK);
    uint8_t *lo8 = lds;   // low part of each byte's exact term (high part: b ^ 0x80)
    // The same table addressed as LDS byte 0 (the kernel has no static LDS, so the dynamic
    // block starts there): lookups take the byte as their address, with no base add per byte.
    const __attribute__((address_space(3))) uint8_t *lo8_at0 =
        (const __attribute__((address_space(3))) uint8_t *)(uintptr_t)0;
    uint64_t *cps = reinterpret_cast<uint64_t *>(lds + 256);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: its rows' bases in SGPRs
    // The wave owns rows [wbase, wbase + nw); lane L takes rows wbase + L + 64 t, so every load
    // and store instruction of the wave covers 64 consecutive rows (768 contiguous bytes).  The
    // wave's base pointers are uniform (SGPRs) and a lane's rows 32-bit offsets from them (N <
    // 2^32), so every access is one SGPR base + one VGPR offset: no 64-bit row or address per row
    // in VGPRs (with them the kernel spilled 15 VGPRs from K = 4, ~20 MB of scratch traffic each
    // way per launch).
    const uint64_t wbase = ((uint64_t)blockIdx.x * NW + wave) * 64 * rows_per_lane;
    const uint32_t nw = (uint32_t)(wbase < N ? min(64 * rows_per_lane, N - wbase) : 0);   // the wave's rows
    const uint32_t nclamp = nw ? nw - 1 : 0;
    const uint8_t *codes_w = codes + (wbase < N ? wbase : 0) * MF_D;
    uint32_t *A_w = A + (wbase < N ? wbase : 0);
    const uint32_t row0 = (uint32_t)wbase;   // flags hold global rows (N < 2^32)
    // four rows of this lane (off + 64 r), two iterations ahead; branch-free (rows past the
    // wave's end read its last row and are masked later), so the loads stay in flight
    auto load4 = [&](uint32_t off, uint32_t (&w)[4][3]) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t o = min(off + 64 * r, nclamp);
            const uint32_t *p = reinterpret_cast<const uint32_t *>(codes_w + o * MF_D);
            w[r][0] = p[0];
            w[r][1] = p[1];
            w[r][2] = p[2];
        }
    };
    // the first group's loads go out before the LDS set-up, under its latency
    uint32_t wa[4][3], wb[4][3];
    load4(lane, wa);
    if (FUSE) {
        for (uint32_t i = tid; i < copies * S; i += (NW * 64)) cps[i] = 0;
        if (tid < 256) lo8[tid] = (uint8_t)(g_plut[tid] & 0xFF);
        if (blockIdx.x == 0) {   // the correction slabs G (+) and G + 1 (-), after all G others
            for (uint32_t i = tid; i < 2 * K * MF_D; i += (NW * 64)) part[(uint64_t)gridDim.x * K * MF_D + i] = 0;
            for (uint32_t i = tid; i < 2 * K; i += (NW * 64)) part_cnt[(uint64_t)gridDim.x * K + i] = 0;
        }
        // copy 1 of the final sums (assign_mf32_kernel's note)
        for (uint32_t i = blockIdx.x * (NW * 64) + tid; i < nz1; i += gridDim.x * (NW * 64)) z1[i] = 0;
    }
    __syncthreads();
    uint64_t *mine = cps + (size_t)((tid & 63) % copies) * S;

    uint32_t acc[MF_D + 1];
    uint32_t cur = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i <= MF_D; i++) acc[i] = 0;
    auto flush = [&]() {
        if (cur != 0xFFFFFFFFu && acc[MF_D]) {
#pragma unroll
            for (int d = 0; d < MF_D; d++) {
                uint32_t u, lo;
                if (PACK) {   // component 4q + j: register 2q + (j & 1), field j >> 1
                    const int reg = 2 * (d / 4) + (d & 1), sh = 16 * ((d % 4) >> 1);
                    u = (acc[reg] >> sh) & 0xFFFF;
                    lo = (acc[6 + reg] >> sh) & 0xFFFF;
                } else {
                    u = acc[d] >> 16;
                    lo = acc[d] & 0xFFFF;
                }
                atomicAdd((unsigned long long *)&mine[d * SK + cur], (unsigned long long)(((uint64_t)u << 32) | lo));
            }
            atomicAdd((unsigned long long *)&mine[MF_D * SK + cur], (unsigned long long)acc[MF_D]);
        }
#pragma unroll
        for (int i = 0; i <= MF_D; i++) acc[i] = 0;
    };
    // Rows r0 + 64 r (r < 4) of this lane, their words in w.  Expanded scores (the MFMA
    // search's, in fp32): score = n + sum_d w_d c''_d = 2^t (||x-c||^2 - ||x-mu||^2), with w
    // the exact centred byte integers -- 12 FMAs per code vector instead of the direct form's
    // 24 VALU.  Error bound (engine.cpp mfma_setup, e0 / e1): per row from sum_d |w_d|, which
    // is at most 2 sum_d |u_d - 127| + D (v_sad_u8 of the u = b ^ 0x80 bytes against 127).
    auto process = [&](const uint32_t (&w)[4][3], uint32_t r0) {
        // four rows at once: each code vector's terms are loaded once (scalar) for all four,
        // and the four score chains are independent.  From SK = 32 rows go in pairs through
        // v_pk_fma_f32 (two fp32 FMAs per lane and instruction, each rounded as fmaf: the
        // scores are the scalar chain's bit for bit): K = 32 81 -> 75 us at C3; below it the
        // per-row sums dominate and the packed form measured 2-14 % slower (profiles/r02h).
        constexpr bool PK = SK >= 32;
        f32x2 x[2][MF_D];
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int d = 0; d < MF_D; d++)
                x[p][d] = __builtin_elementwise_fma(   // byte_w of both rows, one v_pk_fma_f32
                    f32x2{(float)(((w[2 * p][d / 4] ^ 0x80808080u) >> (8 * (d % 4))) & 0xFF),
                          (float)(((w[2 * p + 1][d / 4] ^ 0x80808080u) >> (8 * (d % 4))) & 0xFF)},
                    f32x2{2.f, 2.f}, f32x2{-255.f, -255.f});
        float r1[4], r2[4];
        uint32_t idx[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            r1[r] = INFINITY;
            r2[r] = INFINITY;
            idx[r] = 0;
        }
#pragma unroll 2
        for (int j = 0; j < SK; j++) {
            // wave-uniform: scalar loads into SGPRs (VALU reads them as operands), not LDS
            // broadcasts, which cost the full 64-lane return bandwidth.  Padding rows (j >= K)
            // have n = 1e30 and never win.
            const float *cj = g_E32 + j * 16;
            float cr[MF_D + 1];
#pragma unroll
            for (int d = 0; d <= MF_D; d++) cr[d] = cj[d];
#pragma unroll
            for (int p = 0; p < 2; p++) {
                f32x2 s = f32x2{cr[MF_D], cr[MF_D]};
                if (PK) {
#pragma unroll
                    for (int d = 0; d < MF_D; d++) s = __builtin_elementwise_fma(x[p][d], f32x2{cr[d], cr[d]}, s);
                } else {
#pragma unroll
                    for (int d = 0; d < MF_D; d++) {
                        s.x = __fmaf_rn(x[p][d].x, cr[d], s.x);
                        s.y = __fmaf_rn(x[p][d].y, cr[d], s.y);
                    }
                }
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int r = 2 * p + h;
                    r2[r] = med3f(r1[r], r2[r], s[h]);
                    idx[r] = s[h] < r1[r] ? (uint32_t)j : idx[r];
                    r1[r] = min2f(r1[r], s[h]);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t row = r0 + 64 * r;   // the wave's row
            const uint32_t rk = idx[r];
            const bool valid = row < nw;
            uint32_t sad = 0;
#pragma unroll
            for (int q = 0; q < 3; q++) sad = __builtin_amdgcn_sad_u8(w[r][q] ^ 0x80808080u, 0x7F7F7F7Fu, sad);
            const float thr = __fmaf_rn((float)(2 * sad + MF_D), th.e1, th.e0);
            const bool flagged = valid && !(r2[r] - r1[r] > thr);
            if (flagged) flags[atomicAdd(flag_cnt, 1u)] = row0 + row;
            if (FUSE && valid) {   // provisional index, as in assign_mf32_kernel
                if (rk != cur || acc[MF_D] == 256) {   // 16-bit fields hold 256 rows
                    flush();
                    cur = rk;
                }
                if (PACK) {
#pragma unroll
                    for (int q = 0; q < 3; q++) {
                        const uint32_t wq = w[r][q], c = wq ^ 0x80808080u;
                        acc[2 * q] += c & 0x00FF00FFu;                                // u of 4q, 4q + 2
                        acc[2 * q + 1] += __builtin_amdgcn_perm(0u, c, 0x0C030C01u);  // u of 4q + 1, 4q + 3
                        acc[6 + 2 * q] += (uint32_t)lo8_at0[wq & 0xFF] | (uint32_t)lo8_at0[(wq >> 16) & 0xFF] << 16;
                        acc[7 + 2 * q] += (uint32_t)lo8_at0[(wq >> 8) & 0xFF] | (uint32_t)lo8_at0[wq >> 24] << 16;
                    }
                } else {
#pragma unroll
                    for (int d = 0; d < MF_D; d++) {
                        const uint32_t b = (w[r][d / 4] >> (8 * (d % 4))) & 0xFF;
                        acc[d] += (b ^ 0x80u) << 16 | lo8_at0[b];
                    }
                }
                acc[MF_D] += 1;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (r0 + 64 * r < nw) A_w[r0 + 64 * r] = idx[r];
    };
    // Two row groups per trip, each group's words loaded one group ahead into the other
    // buffer (no register copies, so the loads stay in flight under the previous group).
    // The trip count is wave-uniform; rows past nw are masked inside process.
    for (uint32_t ru = 0; ru < nw; ru += 512) {
        load4(ru + 256 + lane, wb);
        process(wa, ru + lane);
        if (ru + 256 >= nw) break;
        load4(ru + 512 + lane, wa);
        process(wb, ru + 256 + lane);
    }
    if (FUSE) {
        flush();
        __syncthreads();
        uint64_t *pdst = part + (uint64_t)blockIdx.x * K * MF_D;   // slab layout [d][k]
        uint32_t *cdst = part_cnt + (uint64_t)blockIdx.x * K;
        // P threads per slab entry ([d][k]), each summing copies j, j + P, ...; the P partial
        // sums meet by xor shuffles inside the wave.  One thread per entry summed all `copies`
        // (64 at K <= 8) in a serial chain of LDS reads while the other waves idled.
        const uint32_t E = K * (MF_D + 1);
        uint32_t lp = 0;   // log2 P
        while ((2u << lp) <= copies && (2u << lp) * E <= (uint32_t)(NW * 64) && lp < 6) lp++;
        const uint32_t P = 1u << lp;
        for (uint32_t b = 0; b < E * P; b += (NW * 64)) {   // uniform trips: every lane shuffles
            const uint32_t i = b + tid, e = i >> lp, j = i & (P - 1);
            uint64_t v = 0;
            if (e < E) {
                const uint32_t d = e / K, k = e - d * K;
                for (uint32_t c = j; c < copies; c += P) v += cps[(size_t)c * S + d * SK + k];
            }
            for (uint32_t o = 1; o < P; o <<= 1) {
                const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, (int)o);
                const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), (int)o);
                v += ((uint64_t)hi << 32) | lo;
            }
            if (j == 0 && e < E) {
                if (e < K * MF_D) pdst[e] = v;
                else cdst[e - K * MF_D] = (uint32_t)v;
            }
        }
    }
}

hipError_t launch_assign_mfma(hipStream_t s, int grid, bool fuse, const uint8_t *codes, uint64_t N,
                              const _Float16 *cb_rows, const float *E32, uint32_t K, const float *C32,
                              const uint64_t *plut,
                              const MfThresholds &th, uint32_t *A, uint32_t *flags, unsigned *flag_cnt,
                              uint64_t *part, uint32_t *part_cnt, const uint32_t *perm, const int32_t *tint,
                              uint64_t *z1, uint32_t nz1) {
    if (!fuse) z1 = nullptr, nz1 = 0;   // (cleared by the fused kernels' set-up only)
    if (K <= MF_SMALL_K && E32) {   // E32 is padded up to 32 rows (n = 1e30)
        const uint32_t sk = K <= 2 ? 2 : K <= 4 ? 4 : K <= 8 ? 8 : K <= 16 ? 16 : 32;
        // rows per lane: a multiple of 4 covering N over grid x waves x 64 lanes
        const uint32_t copies = fuse ? small_copies(sk) : 1;
        const size_t slds = fuse ? small_lds(sk, copies) : 256;
        // packed run registers with fused sums.  Blocks of 16 waves (4 per SIMD): 12-wave blocks
        // measured 1-10 % slower, also with three row groups in flight (profiles/r03d/ab_small.txt)
        const uint64_t lanes = (uint64_t)grid * 16 * 64;
        const uint64_t rpl = ((N + lanes - 1) / lanes + 3) / 4 * 4;
#define QVQ_SMALL(V)                                                                                              \
    do {                                                                                                          \
        if (fuse)                                                                                                 \
            hipLaunchKernelGGL((assign_small_kernel<V, true, true, 16>), dim3(grid), dim3(16 * 64), slds, s,      \
                               codes, N, K, E32, plut, th, rpl, copies, A, flags, flag_cnt, part, part_cnt, z1,  \
                               nz1);                                                                      \
        else                                                                                                      \
            hipLaunchKernelGGL((assign_small_kernel<V, false, false, 16>), dim3(grid), dim3(16 * 64), slds, s,    \
                               codes, N, K, E32, plut, th, rpl, copies, A, flags, flag_cnt, part, part_cnt, z1,  \
                               nz1);                                                                      \
    } while (0)
        switch (sk) {
        case 2: QVQ_SMALL(2); break;
        case 4: QVQ_SMALL(4); break;
        case 8: QVQ_SMALL(8); break;
        case 16: QVQ_SMALL(16); break;
        default: QVQ_SMALL(32); break;
        }
#undef QVQ_SMALL
        return hipGetLastError();
    }
    // the 32x32x16 form (k_mf32.hip)
    return launch_assign_mf32(s, grid, fuse, codes, N, cb_rows, K, C32, plut, th, A, flags, flag_cnt, part, part_cnt,
                              perm, tint, z1, nz1);
}

// =======================================================================================
// VALU fp32 search (any Dp)
// =======================================================================================
constexpr int ASSIGN_THREADS = 256;
constexpr int ASSIGN_LDS_BYTES = 64 * 1024;

template <int DP>
struct AssignCfg {
    static constexpr int R = DP <= 16 ? 4 : (DP <= 48 ? 2 : 1);   // rows per thread
};

// Each thread keeps R rows in registers; the codebook is staged in LDS (whole when it fits,
// else in tiles) and read by broadcast.  Per row: best and second-best fp32 distance; a gap
// inside 2*(alpha*sqrt(d2) + beta*d2) + gamma flags the row for the fp64 recheck.
template <int DP>
__global__ __launch_bounds__(ASSIGN_THREADS) void assign_valu_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, const float *__restrict__ C32, uint32_t K, uint32_t KT,
    const float *__restrict__ lut32, float alpha, float beta, float gamma, uint32_t *__restrict__ A,
    uint32_t *__restrict__ flags, unsigned int *__restrict__ flag_cnt) {
    constexpr int R = AssignCfg<DP>::R;
    constexpr int D4 = DP / 4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *lut = smem;        // 256
    float *cb = smem + 256;   // KT x DP
    const int tid = threadIdx.x;
    lut[tid] = lut32[tid];
    const bool whole = K <= KT;
    if (whole) {
        const float4 *src = reinterpret_cast<const float4 *>(C32);
        float4 *dst = reinterpret_cast<float4 *>(cb);
        for (uint32_t i = tid; i < K * D4; i += ASSIGN_THREADS) dst[i] = src[i];
    }
    __syncthreads();
    const uint64_t rows_per_block = (uint64_t)ASSIGN_THREADS * R;
    const uint64_t nchunks = (N + rows_per_block - 1) / rows_per_block;
    for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
        float x[R][DP];
        uint64_t row[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            row[r] = chunk * rows_per_block + (uint64_t)r * ASSIGN_THREADS + tid;
            if (row[r] < N) {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(codes + row[r] * DP);
#pragma unroll
                for (int q = 0; q < D4; q++) {
                    const uint32_t v = w[q];
                    x[r][4 * q + 0] = lut[v & 0xFF];
                    x[r][4 * q + 1] = lut[(v >> 8) & 0xFF];
                    x[r][4 * q + 2] = lut[(v >> 16) & 0xFF];
                    x[r][4 * q + 3] = lut[v >> 24];
                }
            } else {
#pragma unroll
                for (int d = 0; d < DP; d++) x[r][d] = 0.f;
            }
        }
        float b1[R], b2[R];
        uint32_t bi[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            b1[r] = INFINITY;
            b2[r] = INFINITY;
            bi[r] = 0;
        }
        for (uint32_t k0 = 0; k0 < K; k0 += KT) {
            const uint32_t kn = min(KT, K - k0);
            if (!whole) {
                __syncthreads();
                const float4 *src = reinterpret_cast<const float4 *>(C32 + (uint64_t)k0 * DP);
                float4 *dst = reinterpret_cast<float4 *>(cb);
                for (uint32_t i = tid; i < kn * D4; i += ASSIGN_THREADS) dst[i] = src[i];
                __syncthreads();
            }
            for (uint32_t kk = 0; kk < kn; kk++) {
                const float4 *c4 = reinterpret_cast<const float4 *>(cb + kk * DP);
                float acc[R];
#pragma unroll
                for (int r = 0; r < R; r++) acc[r] = 0.f;
#pragma unroll
                for (int q = 0; q < D4; q++) {
                    const float4 cq = c4[q];
#pragma unroll
                    for (int r = 0; r < R; r++) {
                        float t;
                        t = x[r][4 * q + 0] - cq.x; acc[r] = __fmaf_rn(t, t, acc[r]);
                        t = x[r][4 * q + 1] - cq.y; acc[r] = __fmaf_rn(t, t, acc[r]);
                        t = x[r][4 * q + 2] - cq.z; acc[r] = __fmaf_rn(t, t, acc[r]);
                        t = x[r][4 * q + 3] - cq.w; acc[r] = __fmaf_rn(t, t, acc[r]);
                    }
                }
                const uint32_t k = k0 + kk;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    b2[r] = med3f(b1[r], b2[r], acc[r]);
                    bi[r] = acc[r] < b1[r] ? k : bi[r];
                    b1[r] = fminf(b1[r], acc[r]);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (row[r] < N) {
                A[row[r]] = bi[r];
                const float thr = 2.f * (alpha * sqrtf(b2[r]) + beta * b2[r]) + gamma;
                if (!(b2[r] - b1[r] > thr)) flags[atomicAdd(flag_cnt, 1u)] = (uint32_t)row[r];
            }
        }
    }
}

#define QVQ_FOR_EACH_DP(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

hipError_t launch_assign_valu(hipStream_t s, int num_cu, uint32_t Dp, const uint8_t *codes, uint64_t N,
                              const float *C32, uint32_t K, const float *lut32, float alpha, float beta, float gamma,
                              uint32_t *A, uint32_t *flags, unsigned *flag_cnt) {
    const uint32_t KT = std::min<uint32_t>(K, (ASSIGN_LDS_BYTES - 1024) / (Dp * 4));
    const size_t lds = 1024 + (size_t)KT * Dp * 4;
    switch (Dp) {
#define X(DPV)                                                                                                 \
    case DPV: {                                                                                                \
        const uint64_t rpb = (uint64_t)ASSIGN_THREADS * AssignCfg<DPV>::R;                                    \
        const int grid = (int)std::min<uint64_t>((N + rpb - 1) / rpb, (uint64_t)num_cu * 8);                  \
        hipLaunchKernelGGL(assign_valu_kernel<DPV>, dim3(grid), dim3(ASSIGN_THREADS), lds, s, codes, N, C32, K, \
                           KT, lut32, alpha, beta, gamma, A, flags, flag_cnt);                                 \
        return hipGetLastError();                                                                              \
    }
        QVQ_FOR_EACH_DP(X)
#undef X
    }
    return hipErrorInvalidValue;
}

// =======================================================================================
// fp64 recheck of flagged rows
// =======================================================================================
// One wave per row, lanes stride over the codebook (staged in LDS when it fits).  The row
// gets the fp64 argmin (lowest index on exact ties); rows whose two best fp64 distances are
// within tie_rel go to the host kd-tree.  With sums != nullptr the resolved rows' exact
// terms are added to the global sums (the fused search skipped them).
constexpr int RECHECK_THREADS = 1024;
constexpr int RECHECK_WAVES = RECHECK_THREADS / 64;
constexpr size_t RECHECK_LDS = 160 * 1024;

// Codebook rows in LDS use an odd stride (in doubles), so the 32 lanes of a ds_read_b64
// group, each on a different code vector, hit different banks.
__host__ __device__ inline uint32_t recheck_stride(uint32_t D) { return D | 1u; }

// Recheck of flagged rows.  fp32 direct distances to all K code vectors (C32, staged in
// LDS when it fits); each lane keeps its best two, the wave takes the minimum m.  Only code
// vectors with d32 - m <= 2(alpha sqrt(d32) + beta d32) + gamma -- the search's rigorous fp32
// error band, so every other code vector is farther in exact arithmetic by much more than
// the tie tolerance -- get the fp64 distance in the reference's order (ref_l2_hd); a lane
// whose second-best is inside the band rescans its code vectors.  Rows whose fp64 best and
// second are within tie_rel are exact ties for the reference: listed in ties (A gets the
// lowest index for now) for kd_resolve_kernel or the host.

// LDS row stride in floats: Dp, or Dp + 4 so that it is 4 mod 8 dwords (16-lane b128 reads
// of 16 consecutive rows then cover all 64 banks once).
__host__ __device__ constexpr uint32_t recheck_c32_stride(uint32_t Dp) { return (Dp % 8 == 4) ? Dp : Dp + 4; }

template <int DT>
__device__ inline float d32_row(const float *__restrict__ xr, const float *__restrict__ c, uint32_t Dp) {
    float acc = 0.f;
    const uint32_t n4 = DT ? (uint32_t)(DT + 3) / 4 : Dp / 4;
#pragma unroll
    for (uint32_t q = 0; q < (DT ? (uint32_t)(DT + 3) / 4 : n4); q++) {
        const float4 cq = reinterpret_cast<const float4 *>(c)[q];
        const float4 xq = reinterpret_cast<const float4 *>(xr)[q];
        float e;
        e = xq.x - cq.x; acc = __fmaf_rn(e, e, acc);
        e = xq.y - cq.y; acc = __fmaf_rn(e, e, acc);
        e = xq.z - cq.z; acc = __fmaf_rn(e, e, acc);
        e = xq.w - cq.w; acc = __fmaf_rn(e, e, acc);
    }
    return acc;   // padding components are 0 in both x and c
}

// LDS: byte LUT (256 doubles) | per wave the fp64 row and the fp32 row | staged fp32 codebook.
constexpr size_t RECHECK_LDS_BASE = 256 * 8 + (size_t)RECHECK_WAVES * 64 * 12;

// Each wave takes flagged rows f = wave id, + all waves, ...; rows are wave-private (no
// block-wide barrier after the staging).  The flag index is fetched two rows ahead and the
// row's bytes one row ahead, so the dependent chain flags -> codes never stalls a row.
template <bool STAGED, int DT>
__global__ __launch_bounds__(RECHECK_THREADS) void recheck_kernel(
    const uint8_t *__restrict__ codes, uint32_t Dp, uint32_t D, const uint32_t *__restrict__ flags,
    const unsigned int *__restrict__ flag_cnt, const double *__restrict__ C64, const float *__restrict__ g_C32,
    uint32_t K, const double *__restrict__ lut64, float alpha, float beta, float gamma, double tie_rel, double tie_abs,
    uint32_t *__restrict__ A, uint32_t *__restrict__ ties, unsigned int *__restrict__ tie_cnt,
    uint64_t *__restrict__ xslab, uint32_t *__restrict__ xcnt, const uint64_t *__restrict__ plut) {
    extern __shared__ __attribute__((aligned(16))) double rsm[];
    constexpr int W = RECHECK_WAVES;
    double *lut = rsm;                                             // [256] exact byte values
    double *xs = rsm + 256;                                        // [W][64] fp64 row
    float *x32 = reinterpret_cast<float *>(xs + W * 64);           // [W][64] fp32 row (zero padded)
    float *c32s = x32 + W * 64;                                    // [K][CS] when staged
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned nflag = *flag_cnt;
    // rows go round the blocks first (f = blockIdx + grid * wave ...), so a level's few flagged
    // rows spread over the CUs instead of 16 to a CU on the first few
    if (nflag == 0 || blockIdx.x >= nflag) return;
    const uint32_t CS = STAGED ? recheck_c32_stride(Dp) : Dp;
    const unsigned fstride = gridDim.x * W;
    unsigned f = blockIdx.x + gridDim.x * wave;
    // two-deep prefetch: row index of f + fstride, bytes of row f
    uint32_t row = f < nflag ? flags[f] : 0;
    uint32_t byte = (f < nflag && lane < (int)D) ? codes[(uint64_t)row * Dp + lane] : 0;
    uint32_t arow = f < nflag ? A[row] : 0;   // the search's index (only this wave writes it)
    uint32_t row_n = f + fstride < nflag ? flags[f + fstride] : 0;
    for (uint32_t i = threadIdx.x; i < 256; i += RECHECK_THREADS) lut[i] = lut64[i];
    if (STAGED) {
        for (uint32_t i = threadIdx.x; i < K * (Dp / 4); i += RECHECK_THREADS) {
            const uint32_t k = i / (Dp / 4), q = i - k * (Dp / 4);
            reinterpret_cast<float4 *>(c32s + (size_t)k * CS)[q] = reinterpret_cast<const float4 *>(g_C32)[i];
        }
    }
    __syncthreads();
    const float *C32 = STAGED ? c32s : g_C32;
    double *xw = xs + wave * 64;
    float *xr = x32 + wave * 64;
    auto within = [&](float d, float m) { return d - m <= 2.f * (alpha * sqrtf(d) + beta * d) + gamma; };
    for (; f < nflag; f += fstride) {
        const uint32_t crow = row, cbyte = byte, carow = arow;
        row = row_n;
        byte = (f + fstride < nflag && lane < (int)D) ? codes[(uint64_t)row * Dp + lane] : 0;
        arow = f + fstride < nflag ? A[row] : 0;
        row_n = f + 2 * fstride < nflag ? flags[f + 2 * fstride] : 0;
        const double v = lane < (int)D ? lut[cbyte] : 0.0;
        xw[lane] = v;
        xr[lane] = (float)v;
        wave_lds_sync();
        // fp32 direct distance to code vector k: the row in registers for a known width
        constexpr int NQ = DT > 0 ? (DT + 3) / 4 : 1;
        float4 xq[NQ];
        if constexpr (DT > 0) {
#pragma unroll
            for (int q = 0; q < NQ; q++) xq[q] = reinterpret_cast<const float4 *>(xr)[q];
        }
        auto d32 = [&](uint32_t k) -> float {
            if constexpr (DT > 0) {
                const float4 *c4 = reinterpret_cast<const float4 *>(C32 + (size_t)k * CS);
                float acc = 0.f;
#pragma unroll
                for (int q = 0; q < NQ; q++) {
                    const float4 cq = c4[q];
                    float e;
                    e = xq[q].x - cq.x; acc = __fmaf_rn(e, e, acc);
                    e = xq[q].y - cq.y; acc = __fmaf_rn(e, e, acc);
                    e = xq[q].z - cq.z; acc = __fmaf_rn(e, e, acc);
                    e = xq[q].w - cq.w; acc = __fmaf_rn(e, e, acc);
                }
                return acc;
            } else {
                return d32_row<0>(xr, C32 + (size_t)k * CS, Dp);
            }
        };
        float b1 = INFINITY, b2 = INFINITY;
        uint32_t kb = 0;
        for (uint32_t k = lane; k < K; k += 64) {
            const float d = d32(k);
            b2 = med3f(b1, b2, d);
            kb = d < b1 ? k : kb;
            b1 = min2f(b1, d);
        }
        // distances are >= 0, so their bit patterns order like the values
        const float m = __uint_as_float(wave_min_u32(__float_as_uint(b1)));
        double d1 = INFINITY, d2 = INFINITY;
        uint32_t k1 = 0xFFFFFFFFu;
        auto take = [&](uint32_t k) {
            const double d = ref_l2_cv(xw, C64, k, D);
            if (d < d1 || (d == d1 && k < k1)) {
                d2 = d1;
                d1 = d;
                k1 = k;
            } else if (d < d2) {
                d2 = d;
            }
        };
        if (within(b2, m)) {   // rare: more than one candidate on this lane
            for (uint32_t k = lane; k < K; k += 64)
                if (within(d32(k), m)) take(k);
        } else if (within(b1, m)) {
            take(kb);
        }
        {   // wave merge on DPP: (d1, k1) the lexicographic minimum; d2 the second-smallest
            // candidate, i.e. the winner lane's d2 or any other lane's d1
            const double m1 = wave_min_f64<4>(d1);
            const uint32_t mk = wave_min_u32(d1 == m1 ? k1 : 0xFFFFFFFFu);
            const bool win = d1 == m1 && k1 == mk;
            d2 = wave_min_f64<4>(win ? d2 : d1);
            d1 = m1;
            k1 = mk;
        }
        if (in_tie_band(d1, d2, tie_rel, tie_abs)) {   // a tie for the reference: the kd-tree decides
            if (lane == 0) ties[atomicAdd(tie_cnt, 1u)] = crow;   // A keeps the provisional index
        } else {
            // the search's index (its terms are in the slabs when fused); mostly unchanged
            const uint32_t from = __builtin_amdgcn_readfirstlane(carow);
            if (k1 != from) {
                if (xslab) move_row_terms(codes, Dp, D, crow, from, k1, K, xslab, xcnt, plut, lane);
                if (lane == 0) A[crow] = k1;
            }
        }
        wave_lds_sync();   // this row's reads of xw / xr before the next row's writes
    }
}

// The recheck for codebooks too big for LDS (C4: K = 4096, D = 48, 850 KB of fp32 rows):
// the block's 16 waves take 16 flagged rows at a time and sweep the codebook together in
// staged chunks of RC_CHUNK code vectors, so each chunk crosses L2 once per 16 rows instead
// of once per row (recheck_kernel<false> streamed the whole table per row: C4 level 12 spent
// ~450 us there).  Same per-row logic as recheck_kernel; the rare row with two candidates on
// one lane rescans the table from global memory.
constexpr uint32_t RC_CHUNK = 512;
template <int DT>
__global__ __launch_bounds__(RECHECK_THREADS) void recheck_chunked_kernel(
    const uint8_t *__restrict__ codes, uint32_t Dp, uint32_t D, const uint32_t *__restrict__ flags,
    const unsigned int *__restrict__ flag_cnt, const double *__restrict__ C64, const float *__restrict__ g_C32,
    uint32_t K, const double *__restrict__ lut64, float alpha, float beta, float gamma, double tie_rel, double tie_abs,
    uint32_t *__restrict__ A, uint32_t *__restrict__ ties, unsigned int *__restrict__ tie_cnt,
    uint64_t *__restrict__ xslab, uint32_t *__restrict__ xcnt, const uint64_t *__restrict__ plut,
    const uint32_t *__restrict__ perm, const int32_t *__restrict__ tint, float qscale) {
    static_assert(DT > 0 && DT % 4 == 0, "a known padded width");
    extern __shared__ __attribute__((aligned(16))) double rsm[];
    __shared__ int32_t win_lo, win_hi;
    constexpr int W = RECHECK_WAVES;
    constexpr int NQ = DT / 4;
    constexpr uint32_t CS = recheck_c32_stride(DT);
    double *lut = rsm;                                     // [256] exact byte values
    double *xs = rsm + 256;                                // [W][64] fp64 row
    float *x32 = reinterpret_cast<float *>(xs + W * 64);   // [W][64] fp32 row (zero padded)
    float *cch = x32 + W * 64;                             // [RC_CHUNK][CS] staged chunk
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned nflag = *flag_cnt;
    if (nflag == 0 || blockIdx.x * W >= nflag) return;
    for (uint32_t i = threadIdx.x; i < 256; i += RECHECK_THREADS) lut[i] = lut64[i];
    double *xw = xs + wave * 64;
    float *xr = x32 + wave * 64;
    auto within = [&](float d, float m) { return d - m <= 2.f * (alpha * sqrtf(d) + beta * d) + gamma; };
    auto d32_at = [&](const float *c, const float4 (&xq)[NQ]) {
        const float4 *c4 = reinterpret_cast<const float4 *>(c);
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const float4 cq = c4[q];
            float e;
            e = xq[q].x - cq.x; acc = __fmaf_rn(e, e, acc);
            e = xq[q].y - cq.y; acc = __fmaf_rn(e, e, acc);
            e = xq[q].z - cq.z; acc = __fmaf_rn(e, e, acc);
            e = xq[q].w - cq.w; acc = __fmaf_rn(e, e, acc);
        }
        return acc;
    };
    // groups of W rows: block-uniform trip count (every wave joins every chunk's barriers)
    for (uint32_t g = blockIdx.x; g * W < nflag; g += gridDim.x) {
        const uint32_t f = g * W + wave;
        const bool have = f < nflag;
        const uint32_t crow = have ? flags[f] : 0;
        const uint32_t cbyte = (have && lane < (int)D) ? codes[(uint64_t)crow * Dp + lane] : 0;
        const uint32_t carow = have ? A[crow] : 0;
        const double v = lane < (int)D ? lut[cbyte] : 0.0;
        __syncthreads();   // lut staged; the previous group's reads of xw / xr are done
        xw[lane] = v;
        xr[lane] = (float)v;
        wave_lds_sync();
        float4 xq[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) xq[q] = reinterpret_cast<const float4 *>(xr)[q];
        float b1 = INFINITY, b2 = INFINITY;
        uint32_t kb = 0;
        // perm (the search's pruned order): only the positions whose tiles the projection bound
        // admits for some row of the group.  A row's best distance is at most its distance to the
        // search's index (fp32, d_A); every candidate of the fp32 band below lies within d_A plus
        // the band plus its own fp32 error, so a tile whose envelope gap g has sx^2 g^2 / D above
        // that holds none.
        uint32_t P0 = 0, P1 = K;
        if (perm) {
            if (threadIdx.x == 0) {
                win_lo = 0x7FFFFFFF;
                win_hi = -1;
            }
            __syncthreads();
            if (have) {
                uint32_t su = lane < (int)D ? (cbyte ^ 0x80u) : 0u;
                float e = lane < (int)D ? xr[lane] - g_C32[(size_t)carow * Dp + lane] : 0.f;
                float dA = e * e;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {
                    su += __shfl_xor(su, o);
                    dA += __shfl_xor(dA, o);
                }
                const int32_t qw = 2 * (int32_t)su - 255 * (int32_t)D;
                const float U = (dA + 4.f * (alpha * sqrtf(dA) + beta * dA) + 4.f * gamma) * 1.001f;
                const float bw = U * qscale * 1.00001f + 1.0f;
                const uint32_t nt = (K + 31) / 32;
                int32_t lo = 0x7FFFFFFF, hi = -1;
                for (uint32_t t = lane; t < nt; t += 64) {
                    const float gap = (float)max(0, max(tint[2 * t] - qw, qw - tint[2 * t + 1]));
                    if (gap * gap <= bw) {
                        lo = min(lo, (int32_t)t);
                        hi = max(hi, (int32_t)t);
                    }
                }
                lo = (int32_t)(wave_min_u32((uint32_t)lo ^ 0x80000000u) ^ 0x80000000u);
                hi = (int32_t)(~wave_min_u32(~((uint32_t)hi ^ 0x80000000u)) ^ 0x80000000u);
                if (lane == 0 && hi >= 0) {
                    atomicMin(&win_lo, lo);
                    atomicMax(&win_hi, hi);
                }
            }
            __syncthreads();
            P0 = win_hi >= 0 ? 32 * (uint32_t)win_lo : 0;
            P1 = win_hi >= 0 ? min(K, 32 * (uint32_t)win_hi + 32) : 0;   // (positions >= K: padding)
        }
        for (uint32_t c0 = P0; c0 < P1; c0 += RC_CHUNK) {
            const uint32_t n = min(RC_CHUNK, P1 - c0);
            __syncthreads();   // the previous chunk's reads are done
            for (uint32_t i = threadIdx.x; i < n * NQ; i += RECHECK_THREADS) {
                const uint32_t k = i / NQ, q = i - k * NQ;
                const uint32_t src = perm ? perm[c0 + k] : c0 + k;
                reinterpret_cast<float4 *>(cch + (size_t)k * CS)[q] =
                    src < K ? reinterpret_cast<const float4 *>(g_C32 + (size_t)src * Dp)[q] : make_float4(1e18f, 1e18f, 1e18f, 1e18f);
            }
            __syncthreads();
            if (have)
                for (uint32_t k = lane; k < n; k += 64) {
                    const float d = d32_at(cch + (size_t)k * CS, xq);
                    b2 = med3f(b1, b2, d);
                    kb = d < b1 ? c0 + k : kb;   // a position
                    b1 = min2f(b1, d);
                }
        }
        if (perm && have) kb = perm[kb];   // the position's code vector
        if (!have) continue;
        const float m = __uint_as_float(wave_min_u32(__float_as_uint(b1)));   // distances >= 0
        double d1 = INFINITY, d2 = INFINITY;
        uint32_t k1 = 0xFFFFFFFFu;
        auto take = [&](uint32_t k) {
            const double d = ref_l2_cv(xw, C64, k, D);
            if (d < d1 || (d == d1 && k < k1)) {
                d2 = d1;
                d1 = d;
                k1 = k;
            } else if (d < d2) {
                d2 = d;
            }
        };
        if (within(b2, m)) {   // rare: more than one candidate on this lane: its positions again
            for (uint32_t p = P0 + lane; p < P1; p += 64) {
                const uint32_t k = perm ? perm[p] : p;
                if (within(d32_at(g_C32 + (size_t)k * Dp, xq), m)) take(k);
            }
        } else if (within(b1, m)) {
            take(kb);
        }
        {   // wave merge: (d1, k1) the lexicographic minimum, d2 the second-smallest candidate
            const double m1 = wave_min_f64<4>(d1);
            const uint32_t mk = wave_min_u32(d1 == m1 ? k1 : 0xFFFFFFFFu);
            const bool win = d1 == m1 && k1 == mk;
            d2 = wave_min_f64<4>(win ? d2 : d1);
            d1 = m1;
            k1 = mk;
        }
        if (in_tie_band(d1, d2, tie_rel, tie_abs)) {   // a tie for the reference: the kd-tree decides
            if (lane == 0) ties[atomicAdd(tie_cnt, 1u)] = crow;
        } else {
            const uint32_t from = __builtin_amdgcn_readfirstlane(carow);
            if (k1 != from) {
                if (xslab) move_row_terms(codes, Dp, D, crow, from, k1, K, xslab, xcnt, plut, lane);
                if (lane == 0) A[crow] = k1;
            }
        }
    }
}

template <bool S, int DT>
static void launch_recheck_variant(hipStream_t s, int grid, size_t lds, const uint8_t *codes, uint32_t Dp, uint32_t D,
                                   const uint32_t *flags, const unsigned *flag_cnt, const double *C64,
                                   const float *C32, uint32_t K, const double *lut64, float alpha, float beta,
                                   float gamma, double tie_rel, double tie_abs, uint32_t *A, uint32_t *ties, unsigned *tie_cnt,
                                   uint64_t *xslab, uint32_t *xcnt, const uint64_t *plut) {
    hipLaunchKernelGGL((recheck_kernel<S, DT>), dim3(grid), dim3(RECHECK_THREADS), lds, s, codes, Dp, D, flags,
                       flag_cnt, C64, C32, K, lut64, alpha, beta, gamma, tie_rel, tie_abs, A, ties, tie_cnt, xslab, xcnt, plut);
}

hipError_t launch_recheck(hipStream_t s, int num_cu, const uint8_t *codes, uint32_t Dp, uint32_t D,
                          const uint32_t *flags, const unsigned *flag_cnt, const double *C64, const float *C32,
                          uint32_t K, const double *lut64, float alpha, float beta, float gamma, double tie_rel, double tie_abs,
                          uint32_t *A, uint32_t *ties, unsigned *tie_cnt, uint64_t *xslab, uint32_t *xcnt,
                          const uint64_t *plut, const uint32_t *perm, const int32_t *tint, float qscale) {
    if (Dp % 4 || Dp > 64) return hipErrorInvalidValue;
    const size_t base = RECHECK_LDS_BASE;
    const size_t cb = (size_t)K * recheck_c32_stride(Dp) * 4;
    const bool staged = base + cb <= RECHECK_LDS;
    const size_t lds = base + (staged ? cb : 0);
    // too big for LDS: the chunked sweep for the widths it is built for
    if (!staged && (Dp == 12 || Dp == 48)) {
        const size_t clds = base + (size_t)RC_CHUNK * recheck_c32_stride(Dp) * 4;
        if (Dp == 12)
            hipLaunchKernelGGL(recheck_chunked_kernel<12>, dim3(num_cu), dim3(RECHECK_THREADS), clds, s, codes, Dp, D,
                               flags, flag_cnt, C64, C32, K, lut64, alpha, beta, gamma, tie_rel, tie_abs, A, ties, tie_cnt,
                               xslab, xcnt, plut, perm, tint, qscale);
        else
            hipLaunchKernelGGL(recheck_chunked_kernel<48>, dim3(num_cu), dim3(RECHECK_THREADS), clds, s, codes, Dp, D,
                               flags, flag_cnt, C64, C32, K, lut64, alpha, beta, gamma, tie_rel, tie_abs, A, ties, tie_cnt,
                               xslab, xcnt, plut, perm, tint, qscale);
        return hipGetLastError();
    }
#define QVQ_RC(SS, DT)                                                                                             \
    launch_recheck_variant<SS, DT>(s, num_cu, lds, codes, Dp, D, flags, flag_cnt, C64, C32, K, lut64, alpha, beta, \
                                   gamma, tie_rel, tie_abs, A, ties, tie_cnt, xslab, xcnt, plut)
    if (Dp == 12) {
        if (staged) QVQ_RC(true, 12); else QVQ_RC(false, 12);
    } else if (Dp == 48) {
        if (staged) QVQ_RC(true, 48); else QVQ_RC(false, 48);
    } else {
        if (staged) QVQ_RC(true, 0); else QVQ_RC(false, 0);
    }
#undef QVQ_RC
    return hipGetLastError();
}

static int kd_waves(const KdView &kd, uint32_t K) { return kd_waves_within(kd, K, RECHECK_LDS); }

bool kd_resolve_fits(const KdView &kd, uint32_t K) { return kd.depth > 0 && kd_waves(kd, K) > 0; }

__global__ __launch_bounds__(KDR_MAX_WAVES * 64) void kd_resolve_kernel(KdArgs a, const unsigned *__restrict__ tie_cnt,
                                                                        int W, int whole_block) {
    extern __shared__ __attribute__((aligned(16))) double ksm[];
    kd_resolve_block(a, *tie_cnt, blockIdx.x, gridDim.x, W, ksm, whole_block != 0);
}

hipError_t launch_kd_resolve(hipStream_t s, const uint8_t *codes, uint32_t Dp, uint32_t D, const uint32_t *ties,
                             const unsigned *tie_cnt, const double *C64, uint32_t K, const double *lut64,
                             const KdView &kd, uint32_t *A, uint64_t *xslab, uint32_t *xcnt, const uint64_t *plut,
                             uint64_t *xsums) {
    int W = kd.depth > 0 ? kd_waves(kd, K) : 0;
    if (W == 0) return hipErrorInvalidValue;
    // big K * D (C3 level 10, C4 from K = 256): a block per tie, its 16 waves on the point
    // distances
    const bool whole = (size_t)K * D >= 8192;
    if (whole) W = 1;
    const size_t lds = kd_tree_bytes(kd) + (size_t)W * kd_wave_bytes(kd, K);
    const KdArgs a{codes, Dp, D, ties, C64, K, lut64, kd, A, xslab, xcnt, plut, xsums};
    hipLaunchKernelGGL(kd_resolve_kernel, dim3(KDR_BLOCKS), dim3(whole ? 64 * KDR_MAX_WAVES : 64 * W), lds, s, a, tie_cnt,
                       W, whole ? 1 : 0);
    return hipGetLastError();
}

// The kd-tree ties and the slabs' column reduce in one launch (fused sums, one rank): blocks
// below KDR_BLOCKS answer ties (kd_resolve_block; their moves go to copy 1 of the sums, which the
// finalize adds), the others reduce 64 columns each into copy 0.  The two touch disjoint data
// (the slabs hold the search's and the recheck's terms only), so neither waits for the other,
// and a level without ties pays one launch instead of two.
__global__ __launch_bounds__(1024) void kd_reduce_kernel(KdArgs a, const unsigned *__restrict__ tie_cnt, int W,
                                                         int whole_block, const uint64_t *__restrict__ part,
                                                         const uint32_t *__restrict__ part_cnt, uint32_t G,
                                                         uint32_t nsub, uint64_t *__restrict__ sums) {
    extern __shared__ __attribute__((aligned(16))) double ksm[];
    if (blockIdx.x < (uint32_t)KDR_BLOCKS) {
        kd_resolve_block(a, *tie_cnt, blockIdx.x, KDR_BLOCKS, W, ksm, whole_block != 0);
        return;
    }
    reduce_columns_block(part, part_cnt, G, nsub, a.K, a.D, sums, blockIdx.x - KDR_BLOCKS,
                         reinterpret_cast<uint64_t *>(ksm));
}

bool kd_reduce_fits(const KdView &kd, uint32_t K) { return kd_resolve_fits(kd, K); }

hipError_t launch_kd_reduce(hipStream_t s, const uint8_t *codes, uint32_t Dp, uint32_t D, const uint32_t *ties,
                            const unsigned *tie_cnt, const double *C64, uint32_t K, const double *lut64,
                            const KdView &kd, uint32_t *A, const uint64_t *plut, const uint64_t *part,
                            const uint32_t *part_cnt, uint32_t G, uint32_t nsub, uint64_t *sums, uint64_t *sums1) {
    int W = kd.depth > 0 ? kd_waves(kd, K) : 0;
    if (W == 0 || nsub > G) return hipErrorInvalidValue;
    const bool whole = (size_t)K * D >= 8192;
    if (whole) W = 1;
    const size_t lds = std::max(kd_tree_bytes(kd) + (size_t)W * kd_wave_bytes(kd, K), (size_t)2 * 16 * 64 * 8);
    // sums1 (the finalize's copy 1) takes the ties' moves
    const KdArgs a{codes, Dp, D, ties, C64, K, lut64, kd, A, nullptr, nullptr, plut, sums1};
    const uint64_t cols = (uint64_t)K * D + K;
    hipLaunchKernelGGL(kd_reduce_kernel, dim3((int)(KDR_BLOCKS + (cols + 63) / 64)), dim3(1024), lds, s, a, tie_cnt,
                       W, whole ? 1 : 0, part, part_cnt, G, nsub, sums);
    return hipGetLastError();
}

}  // namespace qvq
