// vox_hip_gemmf.hip -- k_gemmf: the stream-K MFMA GEMM of the encoder's multi-row chunks.
//
// C[m][n] (op)= sum_k x[m][k] W[n][k] (voxtral_kernels.c:197-240: vox_linear_bf16's sgemm
// on the bf16->f32 weights, M > 1), with x given as bf16 planes hi + mid (+ lo) of the f32
// rows (the NP-term split of k_gemm2: products with the exact bf16 weights are exact, the
// planes carry x to ~2^-16 (NP = 2) or exactly (NP = 3)) and both operands in the
// fragment-major layout of k_frag_pack / frag_at: every 1 KiB of either is one
// v_mfma_f32_16x16x32_bf16 operand fragment (16 rows x 32 k, lane-linear).
//
// Block = 4 WR waves, tile = RB row blocks of 16 x 4 NG column groups of 16; wave w owns
// column groups (w % 4) NG .. + NG - 1 against row share w / 4 (RB / WR row blocks): W
// fragments per column slot, planes per row share, both through LDS.  K runs in 64-deep
// stages:
//   * planes: global_load_lds (LDS-DMA, no VGPRs) into a 3-slot LDS ring, 2 stages ahead;
//     each 1 KiB chunk lands lane-linear and is read back by one conflict-free ds_read_b128;
//   * weights: straight to VGPRs through a buffer descriptor, a 3-deep register ring, 2
//     stages ahead;
//   * one counted s_waitcnt vmcnt + one raw s_barrier per stage (the barrier retires the
//     stage's DMA for every wave and frees the slot the next DMA overwrites).
// Work = tiles x stages, split evenly over one block per CU (stream-K: M = 677 has 288 QKV
// tiles, N = 1280 only 60, so a fixed tile grid leaves CUs idle or needs a split-K reduce
// kernel).  A block walks its unit range in order; a tile whose stages span several blocks
// is finished by the block holding its stage 0 -- it reaches that tile at the END of its
// range, when the blocks holding the tile's later stages (at the START of theirs) have long
// published their partial tiles: write-through (sc1) stores, every wave's vmcnt drain, a
// barrier, one relaxed agent-scope flag store of the launch epoch (MI355X_MICROARCH.md
// "Valid forms", row 1).  The owner polls the flag from one lane (bounded), reads the
// partial with sc1 loads and adds the partials in block order, then runs the epilogue.  A
// wait that times out (another kernel holding the CUs the publishing block needs) makes the
// owner compute that stage range itself: the same code and summation order, the same bits
// (tests/test_gpu_gemm_planes.py forces it); a device counter records each such recompute.
// The epoch must be new for every launch, so a launch is never captured into a graph (the
// engine refuses it while its stream is capturing).
#include "vox_hip_internal.h"
#include "vox_hip_dev.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdlib.h>

namespace vox {

#ifndef VOX_GF_DIAG
#define VOX_GF_DIAG 0  // tools/kbench diagnostics only: 1 = no MFMA, 2 = no DMA (stale LDS)
#endif

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void g_void_t;

// s_waitcnt with only the vector-memory counter bounded (gfx9 encoding: vmcnt [3:0] and
// [15:14], expcnt [6:4] = 7, lgkmcnt [11:8] = 15: no wait on those)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

struct GemmfArgs {
    const uint16_t* xs;  // planes [rb][3][16][K] (frag_at)
    int K, M;
    const uint8_t* W;    // fragment-major bf16 [N / 16][K / 64][2][1 KiB]
    int N;
    const float* bias;   // [N] or null
    float* C;            // f32 output [M][ldc] (SWIGLU: [M][N / 2]) unless xo
    int ldc;
    uint16_t* xo;        // SWIGLU: the gate rows as planes [rb][3][16][N / 2] (the w2 input)
    float* ws;           // [G][4 waves x RB x NG x 64 lanes x 4] partial tiles: slot b = block b's
    int* flags;          // [G] epoch of the partial tile block b published
    int* recomputes;     // count of stage ranges an owner computed itself (wait timed out)
    int wait_ticks;      // owner's bounded wait per partial (< 0: never wait, always recompute)
    int epoch;
    int S, NT, T;        // K stages, column tiles, tiles
    long long U;         // T * S work units
    int MT;              // row tiles
    int colmajor;        // tile order: 0 = t = mt NT + nt (row tile major), 1 = t = nt MT + mt
};


constexpr int GF_TIMEOUT_TICKS = 5000;  // s_memrealtime ticks (100 MHz): 50 us of waiting
static int g_gemmf_wait = GF_TIMEOUT_TICKS;  // vox_hip_set_gemmf_wait (tests force the backstop)

// NWV = 4 WR waves: wave w takes column slot w % 4 (NG groups) and row share w / 4 (RB / WR
// row blocks); with WR = 2 two waves share each SIMD, so one's fragment reads overlap the
// other's MFMAs
template <int NP, int RB, int NG, int WR>
struct GfCfg {
    static constexpr int NWV = 4 * WR;              // waves per block
    static constexpr int RBW = RB / WR;             // row blocks per wave
    static constexpr int CH = RB * NP * 2;          // 1 KiB plane chunks per stage
    static constexpr int CW = 4 * NG * 2;           // 1 KiB weight chunks per stage (4 column slots)
    static constexpr int NA = CH / NWV;             // plane chunks per wave
    static constexpr int NB = CW / NWV;             // weight chunks per wave
    static constexpr int SLOT = (CH + CW) * 512;    // bf16 elements per LDS slot: planes, then weights
    static_assert(CH % NWV == 0 && CW % NWV == 0 && RB % WR == 0, "chunks must split over the waves");
};

// one stage's loads into ring slot SL, all LDS-DMA (no VGPR-destination load in the loop:
// hipcc waits vmcnt(0) at the use of one, which would drain the DMA ring every stage)
template <int NP, int RB, int NG, int WR, int SL>
__device__ __forceinline__ void gf_issue(const uint16_t* xb, size_t plane, const uint8_t* wt, int KB, int s,
                                         uint16_t* lds, int wave, int lane) {
    using C = GfCfg<NP, RB, NG, WR>;
    if (VOX_GF_DIAG == 2) return;
    uint16_t* dst = lds + SL * C::SLOT;
#pragma unroll
    for (int i = 0; i < C::NA; i++) {
        const int c = wave + C::NWV * i;  // chunk: row block c / (2 NP), plane (c / 2) % NP, half c % 2
        const int rb = c / (NP * 2), p = (c >> 1) % NP, t = c & 1;
        const uint16_t* src = xb + ((size_t)rb * 3 + p) * plane + (size_t)(s * 2 + t) * 512 + lane * 8;
        __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)(dst + c * 512), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < C::NB; i++) {
        const int j = wave + C::NWV * i;  // weight chunk: column group j / 2 of the tile, half j % 2
        const uint8_t* src = wt + ((size_t)(j >> 1) * KB + s) * 2048 + (j & 1) * 1024 + lane * 16;
        __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)(dst + (C::CH + j) * 512), 16, 0, 0);
    }
}

// The fragments of one half stage (32 of the 64 k) in registers (every row block of the
// wave's share: rows past M are computed and discarded, which keeps the reads and MFMAs
// branch-free).
template <int NP, int RB, int NG, int WR>
struct GfHalf {
    bf16x8 w[NG];
    bf16x8 x[RB / WR][NP];
};

// read half T of ring slot SL's fragments (10 ds_read_b128 for 128 x 128 tiles, two planes)
template <int NP, int RB, int NG, int WR, int SL, int T>
__device__ __forceinline__ void gf_read(const uint16_t* lds, int wave, int lane, GfHalf<NP, RB, NG, WR>& f) {
    using C = GfCfg<NP, RB, NG, WR>;
    const uint16_t* src = lds + SL * C::SLOT;
    const int wc = wave & 3, r0 = (wave >> 2) * C::RBW;
#pragma unroll
    for (int g = 0; g < NG; g++)
        f.w[g] = *reinterpret_cast<const bf16x8*>(src + (C::CH + (wc * NG + g) * 2 + T) * 512 + lane * 8);
#pragma unroll
    for (int i = 0; i < C::RBW; i++)
#pragma unroll
        for (int p = 0; p < NP; p++)
            f.x[i][p] = *reinterpret_cast<const bf16x8*>(src + (((r0 + i) * NP + p) * 2 + T) * 512 + lane * 8);
}

template <int NP, int RB, int NG, int WR>
__device__ __forceinline__ void gf_mma(const GfHalf<NP, RB, NG, WR>& f, f32x4 (&acc)[RB / WR][NG]) {
    if (VOX_GF_DIAG == 1) {
        acc[0][0][0] += __builtin_bit_cast(float, (uint32_t)f.x[0][0][0] & 0x3f00u);  // keep the reads live
        return;
    }
#pragma unroll
    for (int i = 0; i < RB / WR; i++)
#pragma unroll
        for (int p = 0; p < NP; p++)
#pragma unroll
            for (int g = 0; g < NG; g++)
                acc[i][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.w[g], f.x[i][p], acc[i][g], 0, 0, 0);
}

// lgkmcnt(0) only (vmcnt 63, expcnt 7: no wait on those)
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4)); }

// stages [s0, s1) of tile (mt, nt) accumulated into acc, software-pipelined by half stages:
//   LDS ring of 3 slots (stage x in slot (x - s0) % 3), DMA three stages ahead;
//   while the MFMAs of one half stage run, the wave reads the next half stage's fragments
//   (H0 = k 0..31, H1 = k 32..63 of a stage), so within the wave the matrix pipe and the LDS
//   reads overlap instead of alternating.
// Iteration s (H0 of stage s already in registers):
//   read H1(s) | MFMAs H0(s) | lgkmcnt(0)
//   wait for stage s + 1's DMA (stage s + 2's may stay in flight) -> barrier (every wave's DMA
//   landed; every wave done reading stage s's slot) -> DMA stage s + 3 into stage s's slot ->
//   read H0(s + 1) | MFMAs H1(s) | lgkmcnt(0)
template <int NP, int RB, int NG, int WR>
__device__ __forceinline__ void gf_stages(const GemmfArgs& a, uint16_t* lds, int mt, int nt, int s0, int s1,
                                          f32x4 (&acc)[RB / WR][NG]) {
    using C = GfCfg<NP, RB, NG, WR>;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int KB = a.K >> 6;
    const size_t plane = (size_t)SK_ROWS * a.K;                 // elements per plane of a row block
    const uint16_t* xb = a.xs + (size_t)(mt * RB) * 3 * plane;  // this row tile's planes
    const uint8_t* wt = a.W + (size_t)nt * 4 * NG * KB * 2048;  // this column tile's weight groups
    GfHalf<NP, RB, NG, WR> H0, H1;
    gf_issue<NP, RB, NG, WR, 0>(xb, plane, wt, KB, s0, lds, wave, lane);
    if (s0 + 1 < s1) gf_issue<NP, RB, NG, WR, 1>(xb, plane, wt, KB, s0 + 1, lds, wave, lane);
    if (s0 + 2 < s1) gf_issue<NP, RB, NG, WR, 2>(xb, plane, wt, KB, s0 + 2, lds, wave, lane);
    // stage s0's DMA landed (stages s0 + 1, s0 + 2 may stay in flight)
    if (VOX_GF_DIAG == 2) {
    } else if (s0 + 2 < s1) wait_vm<2 * (C::NA + C::NB)>();
    else if (s0 + 1 < s1) wait_vm<C::NA + C::NB>();
    else wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    gf_read<NP, RB, NG, WR, 0, 0>(lds, wave, lane, H0);
    wait_lgkm0();
#define GF_STAGE(J)                                                                                              \
    if (s + J < s1) {                                                                                            \
        gf_read<NP, RB, NG, WR, J, 1>(lds, wave, lane, H1);                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                                       \
        gf_mma<NP, RB, NG, WR>(H0, acc);                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                                       \
        wait_lgkm0();                                                                                            \
        if (s + J + 1 < s1) {                                                                                    \
            if (VOX_GF_DIAG == 2) {                                                                              \
            } else if (s + J + 2 < s1) wait_vm<C::NA + C::NB>();                                                 \
            else wait_vm<0>();                                                                                   \
            asm volatile("" ::: "memory");                                                                       \
            __builtin_amdgcn_s_barrier();                                                                        \
            asm volatile("" ::: "memory");                                                                       \
            if (s + J + 3 < s1) gf_issue<NP, RB, NG, WR, J>(xb, plane, wt, KB, s + J + 3, lds, wave, lane);      \
            gf_read<NP, RB, NG, WR, (J + 1) % 3, 0>(lds, wave, lane, H0);                                        \
        }                                                                                                        \
        __builtin_amdgcn_sched_barrier(0);                                                                       \
        gf_mma<NP, RB, NG, WR>(H1, acc);                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                                       \
        wait_lgkm0();                                                                                            \
    }
    for (int s = s0; s < s1; s += 3) {
        GF_STAGE(0)
        GF_STAGE(1)
        GF_STAGE(2)
    }
#undef GF_STAGE
    // the ring is reused by the next range: every wave done reading before anyone re-issues
    __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ long long gf_bound(long long U, int G, int b) { return U * b / G; }

// epilogue of one 16 x 16 output fragment of weight group gg for row m (lane & 15 of its row
// block): columns n = gg * 16 + (lane >> 4) * 4 + e.  EPI_SWIGLU: groups (gg, gg + 1) = the
// (w1, w3) rows of 16 hidden units (upload_w13 interleave; gg even), v1 = group gg + 1.
template <int EPI>
__device__ __forceinline__ void gf_out(const GemmfArgs& a, int m, int gg, int lane, const f32x4& v0, const f32x4& v1) {
    if (EPI == EPI_SWIGLU) {
        const int h0 = (gg >> 1) * 16 + (lane >> 4) * 4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = silu(v0[e]) * v1[e];
        if (a.xo) {
            const int H = a.N >> 1;
            uint32_t hp[2], mp[2], lq[2];
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
                uint16_t h_0, m_0, l_0, h_1, m_1, l_1;
                split3(v[e], h_0, m_0, l_0);
                split3(v[e + 1], h_1, m_1, l_1);
                hp[e / 2] = h_0 | ((uint32_t)h_1 << 16);
                mp[e / 2] = m_0 | ((uint32_t)m_1 << 16);
                lq[e / 2] = l_0 | ((uint32_t)l_1 << 16);
            }
            *reinterpret_cast<uint2*>(a.xo + frag_at(m, H, 0, h0)) = make_uint2(hp[0], hp[1]);
            *reinterpret_cast<uint2*>(a.xo + frag_at(m, H, 1, h0)) = make_uint2(mp[0], mp[1]);
            *reinterpret_cast<uint2*>(a.xo + frag_at(m, H, 2, h0)) = make_uint2(lq[0], lq[1]);
        } else {
            *reinterpret_cast<float4*>(a.C + (size_t)m * a.ldc + h0) = make_float4(v[0], v[1], v[2], v[3]);
        }
        return;
    }
    const int n = gg * 16 + (lane >> 4) * 4;
    float4 v = make_float4(v0[0], v0[1], v0[2], v0[3]);
    if (a.bias) {
        const float4 bb = *reinterpret_cast<const float4*>(a.bias + n);
        v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
    }
    float4* cp = reinterpret_cast<float4*>(a.C + (size_t)m * a.ldc + n);
    if (EPI == EPI_RESID) {
        const float4 o = *cp;
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    } else if (EPI == EPI_GELU) {
        v.x = gelu_tanh(v.x); v.y = gelu_tanh(v.y); v.z = gelu_tanh(v.z); v.w = gelu_tanh(v.w);
    } else if (EPI == EPI_GELU_ERF) {
        v.x = gelu_erf(v.x); v.y = gelu_erf(v.y); v.z = gelu_erf(v.z); v.w = gelu_erf(v.w);
    }
    *cp = v;
}

template <int EPI, int NP, int RB, int NG, int WR>
__global__ __launch_bounds__(256 * WR, 1) void k_gemmf(const GemmfArgs a) {
    using C = GfCfg<NP, RB, NG, WR>;
    constexpr int RBW = C::RBW;
    extern __shared__ __attribute__((aligned(16))) uint16_t gf_lds[];
    // the owner's flag mask, one 8-byte word past the ring (the same array)
    unsigned long long* s_okm = reinterpret_cast<unsigned long long*>(gf_lds + 3 * C::SLOT);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wc = wave & 3, r0 = (wave >> 2) * RBW;
    const int G = gridDim.x, b = blockIdx.x;
    const long long u0 = gf_bound(a.U, G, b), u1 = gf_bound(a.U, G, b + 1);
    constexpr int TILE = C::NWV * RBW * NG * 256;  // floats of one partial tile (waves x RBW x NG x 64 lanes x 4)
    const int rbm = (a.M + 15) >> 4;                // row blocks holding rows
    const __amdgpu_buffer_rsrc_t Ws = __builtin_amdgcn_make_buffer_rsrc(a.ws, 0, 0x7fffffff, 0x00020000);
    // this lane's f32x4 of (wave, i, g) in a partial tile
    auto poff = [&](int slotb, int i, int g) {
        return (int)(((size_t)slotb * TILE + ((size_t)(wave * RBW + i) * NG + g) * 256 + lane * 4) * 4);
    };
    long long u = u0;
    while (u < u1) {
        const int t = (int)(u / a.S), s0 = (int)(u % a.S);
        const int s1 = (int)min((long long)a.S, s0 + (u1 - u));
        const int mt = a.colmajor ? t % a.MT : t / a.NT, nt = a.colmajor ? t / a.MT : t % a.NT;
        f32x4 acc[RBW][NG];
#pragma unroll
        for (int i = 0; i < RBW; i++)
#pragma unroll
            for (int g = 0; g < NG; g++) acc[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        gf_stages<NP, RB, NG, WR>(a, gf_lds, mt, nt, s0, s1, acc);
        u += s1 - s0;
        if (s0 > 0) {
            // a later part of tile t: publish it for the tile's owner (write-through stores,
            // every wave drains, one flag store)
#pragma unroll
            for (int i = 0; i < RBW; i++)
#pragma unroll
                for (int g = 0; g < NG; g++)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][g]), Ws, poff(b, i, g), 0, 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) __hip_atomic_store(&a.flags[b], a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        // stage 0 is ours: add the later parts in block order, then the epilogue.  The lanes of
        // wave 0 poll the later blocks' flags together (bounded), so the owner waits for the
        // last of them once instead of one flag round trip per block
        const long long tend = (long long)(t + 1) * a.S;
        int npb = 0;
        while (b + 1 + npb < G && gf_bound(a.U, G, b + 1 + npb) < tend) npb++;
        // npb <= 62: launch_gemmf refuses a minimum stage count that would let more blocks touch a tile
        if (npb > 0) {
            if (wave == 0) {
                const bool mine = lane < npb;
                bool ok = !mine;
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (a.wait_ticks >= 0) {
                    if (!ok) ok = __hip_atomic_load(&a.flags[b + 1 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == a.epoch;
                    if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > (unsigned long long)a.wait_ticks) break;
                    __builtin_amdgcn_s_sleep(2);
                }
                // every recompute is counted (vox_hip_stream_profile): a timeout that fires in
                // production costs the owner the whole stage range, so it must not stay silent
                if (mine && !ok) __hip_atomic_fetch_add(a.recomputes, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long okm = __builtin_amdgcn_ballot_w64(mine && ok);
                if (lane == 0) *s_okm = okm;
            }
            __syncthreads();
            const unsigned long long okm = *s_okm;
            __syncthreads();
            for (int k = 0; k < npb; k++) {
                const int pb = b + 1 + k;
                f32x4 part[RBW][NG];
                if ((okm >> k) & 1) {
#pragma unroll
                    for (int i = 0; i < RBW; i++)
#pragma unroll
                        for (int g = 0; g < NG; g++)
                            part[i][g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(Ws, poff(pb, i, g), 0, 16));
                } else {
                    // the publishing block has not run: its stage range of this tile, computed here
#pragma unroll
                    for (int i = 0; i < RBW; i++)
#pragma unroll
                        for (int g = 0; g < NG; g++) part[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
                    const int q0 = (int)(gf_bound(a.U, G, pb) - (long long)t * a.S);
                    const int q1 = (int)(min(gf_bound(a.U, G, pb + 1), tend) - (long long)t * a.S);
                    gf_stages<NP, RB, NG, WR>(a, gf_lds, mt, nt, q0, q1, part);
                }
#pragma unroll
                for (int i = 0; i < RBW; i++)
#pragma unroll
                    for (int g = 0; g < NG; g++) acc[i][g] += part[i][g];
            }
        }
        // epilogue: lane holds outputs n = group * 16 + (lane >> 4) * 4 + e for row m = rb * 16 + (lane & 15)
#pragma unroll
        for (int i = 0; i < RBW; i++) {
            const int rb = mt * RB + r0 + i;
            if (rb >= rbm) break;
            const int m = rb * 16 + (lane & 15);
            if (m >= a.M) continue;
#pragma unroll
            for (int g = 0; g < NG; g += (EPI == EPI_SWIGLU ? 2 : 1))
                gf_out<EPI>(a, m, (nt * 4 + wc) * NG + g, lane, acc[i][g], acc[i][EPI == EPI_SWIGLU ? g + 1 : g]);
        }
    }
}

// ---------------------------------------------------------------------------
static int g_cus = 0;
int g_gemmf_blocks = -1;  // grid size (0 = one block per CU; -1: read VOX_HIP_GEMMF_BLOCKS once)
int g_gemmf_rb = -1;     // row blocks per tile with two planes (0 = by shape; 4 or 8; -1: VOX_HIP_GEMMF_RB once)
VOX_KB_KNOB(g_gemmf_minu, 0);  // tools/kbench knob: least stages per block (0 = max(4, half a tile))
int g_gemmf_order = -1;  // 1 = column-tile-major unit order (a weight tile's row tiles adjacent), 2 = row-tile-major, 0 = by shape (-1: VOX_HIP_GEMMF_ORDER once)
// waves per block with two planes: 16 (4 row shares of a 128- or 64-row tile: 32 x 32 or 16 x
// 32 per wave, four waves per SIMD) by default, 8 with VOX_HIP_GEMMF_WR=2 (64 x 32 per wave,
// two per SIMD).  Same unit ranges, same per-output summation order: the same bits.  tools/
// kbench (profiles/r4_kbench_gemmf_wr4.txt): M = 677 W1|W3 47.9 -> 44.6, W2 25.6 -> 23.8 us,
// QKV / wo equal; M = 1024 W1|W3 54.5 -> 48.4 us.  Three planes keep 8 (24 chunks a stage).
int g_gemmf_wr = -1;

template <int EPI, int NP, int RB, int NG, int WR>
static hipError_t gemmf_launch(const GemmfArgs& a, int G, hipStream_t st) {
    using C = GfCfg<NP, RB, NG, WR>;
    static bool attr = false;
    const size_t lds = (size_t)3 * C::SLOT * 2 + 16;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemmf<EPI, NP, RB, NG, WR>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL((k_gemmf<EPI, NP, RB, NG, WR>), dim3(G), dim3(256 * WR), lds, st, a);
    return hipGetLastError();
}

size_t gemmf_ws_floats(int blocks) { return (size_t)blocks * (8 * 2 * 4 * 256); }

int gemmf_grid() {
    if (!g_cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_cus <= 0)
            g_cus = 256;
    }
    if (g_gemmf_blocks < 0) {
        // VOX_HIP_GEMMF_BLOCKS: blocks of the stream-K grid (default one per CU); fewer leave
        // CUs to kernels running beside an encoder pass (the scheduler's overlap)
        const char* e = getenv("VOX_HIP_GEMMF_BLOCKS");
        const int v = e ? atoi(e) : 0;
        g_gemmf_blocks = v > 0 && v <= 4 * g_cus ? v : 0;
    }
    return g_gemmf_blocks ? g_gemmf_blocks : g_cus;
}

size_t gemmf_flag_ints() { return (size_t)gemmf_grid() + 1; }
int set_gemmf_wait(int ticks) {
    const int old = g_gemmf_wait;
    g_gemmf_wait = ticks;
    return old;
}

bool gemmf_ok(int M, int N, int K) { return M > 0 && M <= 1024 && K % 64 == 0 && N % 128 == 0; }

hipError_t launch_gemmf(int epi, int np, const uint16_t* xs, int K, int M, const void* Wf, int N, const float* bias,
                        float* C, int ldc, uint16_t* xo, float* ws, size_t ws_floats, int* flags, int epoch,
                        hipStream_t st) {
    // tiles: 128 x 128 with two planes; 64 x 128 with three (a 3-slot ring of 8 row blocks'
    // three planes would not fit the 160 KB of LDS); 16 waves with two planes (g_gemmf_wr),
    // 8 with three
    constexpr int NG = 2, WR = 2;
    if (g_gemmf_rb < 0) {
        // VOX_HIP_GEMMF_RB=4: 64-row tiles on every shape (a 96 KB LDS ring instead of 144 KB,
        // which leaves room on a CU for kernels running beside an encoder pass)
        const char* e = getenv("VOX_HIP_GEMMF_RB");
        const int v = e ? atoi(e) : 0;
        g_gemmf_rb = (v == 4 || v == 8) ? v : 0;
    }
    if (!gemmf_ok(M, N, K) || (np != 2 && np != 3) || !ws || !flags || (g_gemmf_rb && g_gemmf_rb != 4 && g_gemmf_rb != 8))
        return hipErrorInvalidValue;
    // two planes: 128-row tiles while they alone give every CU a tile; narrower outputs (the
    // N = 1280 wo / W2 passes: 10 column tiles) take 64-row tiles -- a stream-K tile split over
    // many blocks costs more than the lower weight reuse (kbench, profiles/r3_gemmf_sweep.txt)
    // (wider per-wave tiles -- 64 x 64 with 4 waves, 32 x 64 with 8 -- measured slower on every
    // encoder shape: DESIGN.md 14.2, profiles/r4_kbench_gemmf*.txt)
    const int NGx = NG;
    const int t8 = ((M + 127) / 128) * (N / (64 * NG));
    const int RB = np == 3 ? 4 : g_gemmf_rb ? g_gemmf_rb : (t8 >= gemmf_grid() ? 8 : 4);
    GemmfArgs a;
    a.xs = xs; a.K = K; a.M = M; a.W = static_cast<const uint8_t*>(Wf); a.N = N; a.bias = bias; a.C = C; a.ldc = ldc;
    a.xo = xo; a.ws = ws; a.flags = flags; a.epoch = epoch;
    a.recomputes = flags + gemmf_grid();  // the counter past the flags (gemmf_flag_ints())
    a.wait_ticks = g_gemmf_wait;
    a.S = K / 64;
    a.NT = N / (64 * NGx);
    a.MT = (M + 16 * RB - 1) / (16 * RB);
    a.T = a.MT * a.NT;
    // unit order: with three planes (64-row tiles) and more than 4 row tiles the row-tile-major
    // order runs 1.2-2.2x slower than the column-tile-major one (a weight tile's row tiles
    // adjacent) on the encoder shapes at 7 / 11 / 13 row tiles (M = 400 / 677 / 800) and on the
    // decoder's (K >= 3072, the stacked prefills) at 7 and 11; at 8 and 16 row tiles of the
    // encoder shapes it is 1-7 % faster (tools/kbench, profiles/r5_kbench_gemmf_order_m.txt,
    // r5_kbench_gemmfx.txt).  VOX_HIP_GEMMF_ORDER / g_gemmf_order: 1 / 2 force either.
    if (g_gemmf_order < 0) {
        const char* e = getenv("VOX_HIP_GEMMF_ORDER");
        const int v = e ? atoi(e) : 0;
        g_gemmf_order = (v == 1 || v == 2) ? v : 0;
    }
    a.colmajor = g_gemmf_order ? g_gemmf_order == 1 : (np == 3 && a.MT > 4 && (a.MT % 4 != 0 || K > 2048));
    a.U = (long long)a.T * a.S;
    // one block per CU, but every block at least half a tile's stages (and 4): a tile split
    // over many blocks costs its owner one partial-tile read per extra block.  One or two row
    // tiles (M <= 128 with three planes: prefills, the flush chunk) leave too few tiles for
    // that: an eighth of a tile (and 6) spreads the weights over 2-4x the CUs -- decoder prefill
    // M = 38: wo 25.3 -> 15.8, w2 48.6 -> 22.3, QKV 20.5 -> 15.6 us; encoder M = 25-70: wo 15.3
    // -> 11.5-12.9, w2 28.9 -> 16.2-17.5 us; at 7+ row tiles the half-tile rule stays faster
    // (tools/kbench VOX_KB_ONLY=gemmfm, profiles/r5_kbench_gemmf_minu.txt)
    const long long minu = g_gemmf_minu ? g_gemmf_minu
                           : a.MT <= 2 ? std::max(6, a.S / 8) : std::max(4, (a.S + 1) / 2);
    // the owner polls the flags of its tile's later blocks with the lanes of one wave: a tile
    // may span at most 64 of them (ceil(S / minu) + 1 blocks touch a tile)
    if ((a.S + minu - 1) / minu + 2 > 64) return hipErrorInvalidConfiguration;
    int G = gemmf_grid();
    if ((long long)G * minu > a.U) G = (int)std::max(1LL, a.U / minu);
    // one partial tile per block: (4 WR waves) x (RB / WR) x NGx x 64 lanes x 4 floats
    if ((size_t)G * 4 * RB * NGx * 256 > ws_floats) return hipErrorInvalidConfiguration;  // workspace too small
#define GF_EPI(E)                                                                               \
    if (epi == E)                                                                               \
        return np == 3 ? gemmf_launch<E, 3, 4, NG, WR>(a, G, st)                                \
               : g_gemmf_wr == 4 ? (RB == 8 ? gemmf_launch<E, 2, 8, NG, 4>(a, G, st)             \
                                            : gemmf_launch<E, 2, 4, NG, 4>(a, G, st))            \
               : RB == 8 ? gemmf_launch<E, 2, 8, NG, WR>(a, G, st) : gemmf_launch<E, 2, 4, NG, WR>(a, G, st);
    if (g_gemmf_wr < 0) {
        const char* e = getenv("VOX_HIP_GEMMF_WR");
        g_gemmf_wr = (e && atoi(e) == 2) ? 2 : 4;
    }

    GF_EPI(EPI_STORE) GF_EPI(EPI_RESID) GF_EPI(EPI_GELU) GF_EPI(EPI_GELU_ERF) GF_EPI(EPI_SWIGLU)
#undef GF_EPI
    return hipErrorInvalidValue;
}

}  // namespace vox
