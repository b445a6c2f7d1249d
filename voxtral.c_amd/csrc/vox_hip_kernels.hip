// vox_hip_kernels.hip -- CDNA4 (gfx950) kernels for the Voxtral hot path.
//
// Layout conventions (DESIGN.md "Data layout in HBM"):
//   activations  f32 row-major [rows, features]
//   weights      bf16 row-major [out, in] (nn.Linear layout, voxtral_safetensors.c:446-451);
//                decoder/encoder Q|K|V merged row-wise, W1|W3 interleaved in 16-row groups
//                (rows 32g..32g+15 = w1[16g..], rows 32g+16..32g+31 = w3[16g..])
//   KV caches    f32 rolling buffers [cap][kv_heads*head_dim] per layer, slot = pos % cap
//                (decoder: IEEE half in the opt-in 16-bit mode, VOX_DECODER_KV_FP16)
//   rope tables  f32 [pos][head_dim/2][2] (cos, sin) computed on the host with the
//                reference's float powf/cosf/sinf (voxtral_kernels.c:617-629)
//
// Numerics: every kernel keeps the reference's f32 arithmetic: f32 activations times
// exact bf16->f32 weights, f32 accumulation (voxtral_kernels.c:154-240).  The MFMA GEMM
// (M>1) splits each f32 activation into NSPLIT bf16 terms (hi + mid + lo for NSPLIT=3
// reproduces the f32 value exactly), so products against the exact-bf16 weights are
// exact and only the summation order differs from the CPU sgemm.
#include "vox_hip_internal.h"
#include "vox_hip_dev.h"

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <algorithm>
#include <string.h>
#include <stdlib.h>

namespace vox {

// ============================================================================
// Decoder KV element type.  f32 by default (the CPU reference's cache); the opt-in 16-bit
// mode (VOX_DECODER_KV_FP16, voxtral.c:189-190, voxtral_decoder.c:180-243) stores IEEE half:
// stores round to nearest even, loads widen to f32, all arithmetic stays f32.  Kernels that
// read the ring are templated on the element type; the two single-store epilogues (decode
// QKV GEMV, batched RoPE + append) take it as a uniform runtime flag.
// ============================================================================
typedef _Float16 kvh_t;
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
template <class T> __device__ __forceinline__ float4 kv_ld4(const T* p) {
    if constexpr (sizeof(T) == 4) {
        return *reinterpret_cast<const float4*>(p);
    } else {
        const h16x4 h = *reinterpret_cast<const h16x4*>(p);
        return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
    }
}
template <class T> __device__ __forceinline__ float2 kv_ld2(const T* p) {
    if constexpr (sizeof(T) == 4) {
        return *reinterpret_cast<const float2*>(p);
    } else {
        const h16x2 h = *reinterpret_cast<const h16x2*>(p);
        return make_float2((float)h[0], (float)h[1]);
    }
}
template <class T> __device__ __forceinline__ float kv_round(float v) { return (float)(T)v; }
template <class T> __device__ __forceinline__ void kv_st2(T* p, float a, float b) {
    if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float2*>(p) = make_float2(a, b);
    } else {
        *reinterpret_cast<h16x2*>(p) = h16x2{(T)a, (T)b};
    }
}
// element e of a ring (f32 or half by the flag) written as the pair (a, b) at e, e + 1
__device__ __forceinline__ void kv_st2_rt(float* base, size_t e, float a, float b, int kv16) {
    if (kv16) kv_st2(reinterpret_cast<kvh_t*>(base) + e, a, b);
    else kv_st2(base + e, a, b);
}

// ============================================================================
// Row-wise RMSNorm (+ optional ada scale), M>1 paths.  voxtral_kernels.c:475-492,
// voxtral_decoder.c:564-570.  One block per row.
// ============================================================================
__global__ __launch_bounds__(256) void k_rmsnorm_rows(const float* __restrict__ x, int ldx,
                                                      float* __restrict__ y, int ldy,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ ada, int D,
                                                      float eps) {
    __shared__ float red[4];
    const float* xr = x + (size_t)blockIdx.x * ldx;
    float* yr = y + (size_t)blockIdx.x * ldy;
    float ss = 0.f;
    for (int i = threadIdx.x; i < D; i += 256) ss = fmaf(xr[i], xr[i], ss);
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    float tot = red[0] + red[1] + red[2] + red[3];
    float inv = 1.0f / sqrtf(tot / (float)D + eps);
    for (int i = threadIdx.x; i < D; i += 256) {
        float v = xr[i] * inv * w[i];
        if (ada) v *= (1.0f + ada[i]);
        yr[i] = v;
    }
}

// ============================================================================
// Pipelined MFMA GEMM (the M>1 path of prefill, adapter, conv stem and the twins):
// C[M,N] (op)= A[M,K] (f32) * W[N,K]^T (bf16, or int8 with per-row scales: the Q8 "fused
// dequant -> bf16 MFMA" path, voxtral_kernels.c:320-393; an int8 weight is exact in bf16 and
// the row scale is applied to the f32 result, s * sum(x q), where the reference sums x (q s)).
// Block tile 128x128, 4 waves in 2x2, each wave 64x64 = 4x4 v_mfma_f32_16x16x32_bf16
// tiles (the large wave tile keeps the LDS fragment traffic of the 3 A planes under the
// LDS rate).  K advances in 64-deep stages: the stage's A (f32) and W tiles are loaded to
// registers one stage ahead (issued before the current stage's MFMAs), split into the three
// bf16 planes hi/mid/lo (A = hi + mid + lo exactly; Q8 weights -> exact bf16) and written
// to one of two LDS buffers, so one barrier per stage suffices.  Epilogues: store, residual
// add, GELU (tanh / erf), SwiGLU pairs and EPI_PARTIAL for split-K slices over blockIdx.z.
// ============================================================================
#define G2_M 128
#define G2_N 128
#define G2_K 64
#define G2_LDS (G2_K + 8)  // padded bf16 row (144 B)
#ifndef VOX_G2_DIAG
#define VOX_G2_DIAG 0  // kbench diagnostics only: 1 = no MFMA, 2 = no staging
#endif

// k_gemm2 staging: 32 A floats and 32 W elements per thread (row t/2, k half (t&1)*32)
// AV = A float4 per thread: 8 (256 threads, 128-column tiles) or 4 (512 threads, 256-column
// tiles); W: 32 elements per thread either way
template <int AV>
struct G2Regs {  // one stage's staging registers (constant-indexed arrays: kept in VGPRs)
    float4 a[AV];
    uint4 w[4];
};

template <int WQ8, int AV>
__device__ __forceinline__ void g2_load(G2Regs<AV>& r, const float* __restrict__ Ap, const uint16_t* __restrict__ Wp,
                                        const int8_t* __restrict__ Wq, int ko) {
    const float4* a = reinterpret_cast<const float4*>(Ap + ko);
#pragma unroll
    for (int i = 0; i < AV; i++) r.a[i] = a[i];
    if (WQ8) {
        const uint4* q = reinterpret_cast<const uint4*>(Wq + ko);
        r.w[0] = q[0];
        r.w[1] = q[1];
    } else {
        const uint4* w = reinterpret_cast<const uint4*>(Wp + ko);
#pragma unroll
        for (int i = 0; i < 4; i++) r.w[i] = w[i];
    }
}

// split A into the hi/mid/lo bf16 planes (exact), W to bf16 (Q8: exact), into one LDS buffer
template <int WQ8, int NP, int AV>
__device__ __forceinline__ void g2_store(const G2Regs<AV>& r, uint16_t* base, int srow, int sk, int wrow, int wk,
                                         float amask) {
    constexpr int PLANE = 128 * (64 + 8);
    const float4* ra = r.a;
    const uint4* rw = r.w;
#pragma unroll
    for (int i = 0; i < AV; i += 2) {
        float v[8] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w, ra[i + 1].x, ra[i + 1].y, ra[i + 1].z, ra[i + 1].w};
        uint32_t t[NP][8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            float r = v[e] * amask;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const uint32_t bb = f2bf(r);
                t[p][e] = bb;
                r = r - __uint_as_float(bb << 16);
            }
        }
#pragma unroll
        for (int p = 0; p < NP; p++) {
            uint4 pk;
            pk.x = t[p][0] | (t[p][1] << 16);
            pk.y = t[p][2] | (t[p][3] << 16);
            pk.z = t[p][4] | (t[p][5] << 16);
            pk.w = t[p][6] | (t[p][7] << 16);
            *reinterpret_cast<uint4*>(base + p * PLANE + srow * 72 + sk + 4 * i) = pk;
        }
    }
    uint16_t* wb = base + NP * PLANE + wrow * 72 + wk;
    if (WQ8) {
        const uint32_t d[8] = {rw[0].x, rw[0].y, rw[0].z, rw[0].w, rw[1].x, rw[1].y, rw[1].z, rw[1].w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t h[8];
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
                h[bb] = __float_as_uint(i8f(d[2 * i], bb)) >> 16;
                h[4 + bb] = __float_as_uint(i8f(d[2 * i + 1], bb)) >> 16;
            }
            uint4 pk;
            pk.x = h[0] | (h[1] << 16);
            pk.y = h[2] | (h[3] << 16);
            pk.z = h[4] | (h[5] << 16);
            pk.w = h[6] | (h[7] << 16);
            *reinterpret_cast<uint4*>(wb + 8 * i) = pk;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) *reinterpret_cast<uint4*>(wb + 8 * i) = rw[i];
    }
}

// NP = activation planes: 3 (hi + mid + lo = the exact f32 value) or 2 (hi + lo: the value
// to ~2^-18 relative; the default, see gemm_planes and DESIGN.md section 5)
// WN = waves along N: 2 (128 x 128 tile, 256 threads) or 4 (128 x 256 tile, 512 threads: each
// A stage feeds twice the columns, so the activations are re-read from L2 half as often;
// bf16 weights with two planes, so the stage buffer stays 73.7 KB and two blocks share a CU)
template <int EPI, int WQ8, int NP = 3, int WN = 2>
__global__ __launch_bounds__(128 * WN, 2) void k_gemm2(const float* __restrict__ A, int lda,
                                                       const void* __restrict__ W, int K, int M, int N,
                                                       const float* __restrict__ wscale,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ C, int ldc) {
    extern __shared__ __attribute__((aligned(16))) uint16_t g2_lds[];
    // [plane 0..NP-1 = A hi/(mid)/lo][128][G2_LDS], then W [64 WN][G2_LDS]
    constexpr int PLANE = G2_M * G2_LDS;
    constexpr int AV = WN == 2 ? 8 : 4;   // A float4 per thread
    constexpr int TPR = 16 / AV;          // threads per A row
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / WN, wc = wave % WN;
    const int m0 = blockIdx.y * G2_M, n0 = blockIdx.x * (64 * WN);
    const int Ks = K / gridDim.z, kb = blockIdx.z * Ks;
    const int nst = Ks / G2_K;
    // staging: A row t / TPR, 4 AV consecutive k; W row t / 2, 32 consecutive k at (t & 1) * 32
    const int srow = tid / TPR, sk = (tid % TPR) * 4 * AV;
    const int wrow = tid >> 1, wk = (tid & 1) * 32;
    const int arow = min(m0 + srow, M - 1);
    const float amask = (m0 + srow) < M ? 1.0f : 0.0f;
    const float* Ap = A + (size_t)arow * lda + kb + sk;
    const uint16_t* Wp = static_cast<const uint16_t*>(W) + (size_t)(n0 + wrow) * K + kb + wk;
    const int8_t* Wq = static_cast<const int8_t*>(W) + (size_t)(n0 + wrow) * K + kb + wk;

    G2Regs<AV> rg;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    g2_load<WQ8, AV>(rg, Ap, Wp, Wq, 0);
    const int fr = lane & 15, fk = (lane >> 4) * 8;
    for (int st = 0; st < nst; st++) {
        if (st) __syncthreads();  // the previous stage's fragments have been read
#if VOX_G2_DIAG != 2
        g2_store<WQ8, NP, AV>(rg, g2_lds, srow, sk, wrow, wk, amask);
        if (st + 1 < nst) g2_load<WQ8, AV>(rg, Ap, Wp, Wq, (st + 1) * G2_K);  // in flight during this stage's MFMAs
#endif
        __syncthreads();
#if VOX_G2_DIAG == 1
        continue;
#endif
        const uint16_t* base = g2_lds;
#pragma unroll
        for (int kk = 0; kk < G2_K; kk += 32) {
            bf16x8 bfrag[4];
#pragma unroll
            for (int ni = 0; ni < 4; ni++)
                bfrag[ni] = *reinterpret_cast<const bf16x8*>(base + NP * PLANE + (wc * 64 + ni * 16 + fr) * G2_LDS + kk + fk);
#pragma unroll
            for (int p = 0; p < NP; p++)
#pragma unroll
                for (int mi = 0; mi < 4; mi++) {
                    const bf16x8 afrag = *reinterpret_cast<const bf16x8*>(base + p * PLANE + (wr * 64 + mi * 16 + fr) * G2_LDS + kk + fk);
#pragma unroll
                    for (int ni = 0; ni < 4; ni++)
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afrag, bfrag[ni], acc[mi][ni], 0, 0, 0);
                }
        }
    }

    // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + r
    const int cc = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
    for (int mi = 0; mi < 4; mi++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int m = m0 + wr * 64 + mi * 16 + rq + r;
            if (m >= M) continue;
            if (EPI == EPI_PARTIAL) {
#pragma unroll
                for (int ni = 0; ni < 4; ni++)
                    C[((size_t)blockIdx.z * M + m) * N + n0 + wc * 64 + ni * 16 + cc] = acc[mi][ni][r];
            } else if (EPI == EPI_SWIGLU) {
                // 16-row interleave: tiles (0,1) and (2,3) are (w1, w3) of one unit group
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int nb = n0 + wc * 64 + h * 32;
                    float gt = acc[mi][2 * h][r], up = acc[mi][2 * h + 1][r];
                    if (WQ8) {
                        gt *= wscale[nb + cc];
                        up *= wscale[nb + 16 + cc];
                    }
                    C[(size_t)m * ldc + (nb >> 5) * 16 + cc] = silu(gt) * up;
                }
            } else {
#pragma unroll
                for (int ni = 0; ni < 4; ni++) {
                    const int n = n0 + wc * 64 + ni * 16 + cc;
                    float v = acc[mi][ni][r];
                    if (WQ8) v *= wscale[n];
                    if (bias) v += bias[n];
                    float* cp = C + (size_t)m * ldc + n;
                    if (EPI == EPI_STORE) *cp = v;
                    else if (EPI == EPI_RESID) *cp += v;
                    else if (EPI == EPI_GELU) *cp = gelu_tanh(v);
                    else if (EPI == EPI_GELU_ERF) *cp = gelu_erf(v);
                }
            }
        }
    }
}
constexpr size_t G2_LDS_BYTES = (size_t)4 * G2_M * G2_LDS * 2;  // 73,728 B: two blocks per CU
// Activation planes of the M > 1 GEMMs (k_gemm2, k_gemmf): 3 by default (hi + mid + lo = the
// f32 activation exactly, so the products with the exact-bf16 weights are exact and only the
// summation order differs from the reference's f32 sgemm, voxtral_kernels.c:197-240);
// VOX_HIP_GEMM_PLANES=2 / vox_hip_set_gemm_planes(2) is the faster approximate split (hi +
// lo, ~2^-18 relative per activation: full-size jfk logits 1.5e-5 / adapter rows 1.4e-5 of
// the largest magnitude against the 5e-5 bar, ids identical; ~20 % less GEMM time).
int g_gemm_planes = 0;
static int gemm_planes() {
    if (!g_gemm_planes) {
        const char* e = getenv("VOX_HIP_GEMM_PLANES");
        g_gemm_planes = (e && atoi(e) == 2) ? 2 : 3;
    }
    return g_gemm_planes;
}
int gemm_planes_np() { return gemm_planes(); }
int set_gemm_planes(int np) {
    if (np != 2 && np != 3) return -1;
    g_gemm_planes = np;
    return 0;
}

// ============================================================================
// Split-K finish: sum the S partial tiles in slice order (deterministic), then the GEMM
// epilogue (Q8 row scale, bias, residual / GELU / SwiGLU pairing).
// One thread per output element; part is [S][M][N].
// ============================================================================
template <int EPI>
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* __restrict__ part, int S, int M, int N,
                                                       const float* __restrict__ wscale,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ C, int ldc) {
    const int NO = EPI == EPI_SWIGLU ? N / 2 : N;  // output columns
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)M * NO) return;
    const int m = (int)(idx / NO), j = (int)(idx % NO);
    const size_t MN = (size_t)M * N;
    if (EPI == EPI_SWIGLU) {
        const int n1 = (j >> 4) * 32 + (j & 15), n3 = n1 + 16;  // w1 / w3 rows of unit j
        float g = 0.f, u = 0.f;
        for (int z = 0; z < S; z++) {
            g += part[z * MN + (size_t)m * N + n1];
            u += part[z * MN + (size_t)m * N + n3];
        }
        if (wscale) {
            g *= wscale[n1];
            u *= wscale[n3];
        }
        C[(size_t)m * ldc + j] = silu(g) * u;
        return;
    }
    float v = 0.f;
    for (int z = 0; z < S; z++) v += part[z * MN + (size_t)m * N + j];
    if (wscale) v *= wscale[j];
    if (bias) v += bias[j];
    float* cp = C + (size_t)m * ldc + j;
    if (EPI == EPI_STORE) *cp = v;
    else if (EPI == EPI_RESID) *cp += v;
    else if (EPI == EPI_GELU) *cp = gelu_tanh(v);
    else if (EPI == EPI_GELU_ERF) *cp = gelu_erf(v);
}

// ============================================================================
// RoPE + KV append for M>1 rows (voxtral_encoder.c:580-607, voxtral_decoder.c:531-541).
// qkv [M, qd + 2*kvd] -> q [M, qd] roped; K/V ring slots (pos0 + i) % cap.
// ============================================================================
template <class KT>
__global__ __launch_bounds__(256) void k_rope_kv(const float* __restrict__ qkv, int M, int qd,
                                                 int kvd, int hd, const float* __restrict__ rope,
                                                 int pos0, float* __restrict__ q,
                                                 float* __restrict__ Kc, float* __restrict__ Vc,
                                                 int cap) {
    const int i = blockIdx.x;
    const int ld = qd + 2 * kvd;
    const float* row = qkv + (size_t)i * ld;
    const float* rp = rope + (size_t)i * hd;  // rope rows for rows i (pos0 + i)
    const int slot = (pos0 + i) % cap;
    KT* kr = reinterpret_cast<KT*>(Kc) + (size_t)slot * kvd;
    KT* vr = reinterpret_cast<KT*>(Vc) + (size_t)slot * kvd;
    for (int p = threadIdx.x; p < qd / 2; p += 256) {
        int d = (2 * p) % hd / 2;
        float c = rp[2 * d], s = rp[2 * d + 1];
        float x0 = row[2 * p], x1 = row[2 * p + 1];
        q[(size_t)i * qd + 2 * p] = x0 * c - x1 * s;
        q[(size_t)i * qd + 2 * p + 1] = x0 * s + x1 * c;
    }
    for (int p = threadIdx.x; p < kvd / 2; p += 256) {
        int d = (2 * p) % hd / 2;
        float c = rp[2 * d], s = rp[2 * d + 1];
        float x0 = row[qd + 2 * p], x1 = row[qd + 2 * p + 1];
        kv_st2(kr + 2 * p, x0 * c - x1 * s, x0 * s + x1 * c);
    }
    for (int p = threadIdx.x; p < kvd / 2; p += 256) kv_st2(vr + 2 * p, row[qd + kvd + 2 * p], row[qd + kvd + 2 * p + 1]);
}

// k_rope_kv over the stacked rows of a batched encoder pass: block = one row, its stream found
// from the row offsets (same operations per row as k_rope_kv)
__global__ __launch_bounds__(256) void k_rope_kv_rows(const float* __restrict__ qkv, int qd, int kvd, int hd,
                                                      const float* __restrict__ rope_table, const EncRows er,
                                                      float* __restrict__ q, int cap) {
    const int row = blockIdx.x;
    int b = 0;
    while (b + 1 < er.B && row >= er.off[b + 1]) b++;
    const int i = row - er.off[b];
    const int ld = qd + 2 * kvd;
    const float* xr = qkv + (size_t)row * ld;
    const float* rp = rope_table + (size_t)(er.pos0[b] + i) * hd;
    const int slot = (er.pos0[b] + i) % cap;
    float* kr = er.Kc[b] + (size_t)slot * kvd;
    float* vr = er.Vc[b] + (size_t)slot * kvd;
    for (int p = threadIdx.x; p < qd / 2; p += 256) {
        int d = (2 * p) % hd / 2;
        float c = rp[2 * d], sn = rp[2 * d + 1];
        float x0 = xr[2 * p], x1 = xr[2 * p + 1];
        q[(size_t)row * qd + 2 * p] = x0 * c - x1 * sn;
        q[(size_t)row * qd + 2 * p + 1] = x0 * sn + x1 * c;
    }
    for (int p = threadIdx.x; p < kvd / 2; p += 256) {
        int d = (2 * p) % hd / 2;
        float c = rp[2 * d], sn = rp[2 * d + 1];
        float x0 = xr[qd + 2 * p], x1 = xr[qd + 2 * p + 1];
        kv_st2(kr + 2 * p, x0 * c - x1 * sn, x0 * sn + x1 * c);
    }
    for (int p = threadIdx.x; p < kvd / 2; p += 256) kv_st2(vr + 2 * p, xr[qd + kvd + 2 * p], xr[qd + kvd + 2 * p + 1]);
}

// ============================================================================
// Causal / windowed attention for M>1 queries (encoder chunks, decoder prefill) with the
// semantics of vox_causal_attention (voxtral_kernels.c:541-611) at logical positions: query
// i sits at q_pos0+i and sees keys p with max(k_first, qp-window+1) <= p <= qp.  On f32 MFMA
// (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation).  ns > 1 (few query rows,
// a long key range): blockIdx.z takes the z-th of ns key ranges and writes an unnormalised
// (o, m, l) partial per query row to part[(h * M + q) * ns + z][HD + 2], merged in z order
// by k_attn_tiled_combine.  Block = (head, 16
// queries, key range z) of 4 waves; wave w takes the range's 16-key chunks w, w+4, ...  Per
// chunk: S^T = K Q^T, A = the K rows straight from the cache, B = the block's query rows held
// in registers (lane l: row l & 15, dims [g HD/4, (g+1) HD/4) of group g = l >> 4); online
// softmax on the accumulator (keys 4g + i in the registers, query l & 15 on the lane); then
// O += P V with P taken from the S^T registers as the A operand (no LDS) and V as B (lane l:
// dims [NB j, NB j + NB) of rows 4g + c).  The next chunk's K / V load while the current one
// computes.  The four waves' (o, m, l) meet in LDS at the end.  (A VALU kernel that staged
// K / V tiles in LDS was bound by their reads: 160 ds_read_b128 per thread per 64-key tile.)
// ============================================================================
// BAT: a batched encoder pass -- blockIdx.z = stream * ns + key split; Q / O / the partials'
// rows are the stacked rows (stream b's from er.off[b], M = the stacked total), Kc / Vc /
// q_pos0 / the stream's row count come from er.
template <int HD, class KT = float, int BAT = 0>
__global__ __launch_bounds__(256) void k_attn_mf(const float* __restrict__ Q, int ldq, const float* __restrict__ Kc,
                                                 const float* __restrict__ Vc, int cap, float* __restrict__ O,
                                                 int ldo, int M, int H, int KVH, int q_pos0, int k_first, int window,
                                                 float scale, int ns, float* __restrict__ part,
                                                 const EncRows er = EncRows{}, uint16_t* __restrict__ xs = nullptr) {
    constexpr int DG = HD / 4;   // S^T: dims per lane group
    constexpr int NB = HD / 16;  // P V: output dims per lane (d = NB j + b)
    __shared__ float sm[4][16], sl[4][16];
    __shared__ __attribute__((aligned(16))) float so[4][16][HD + 4];
    const int zsplit = BAT ? (int)blockIdx.z % ns : (int)blockIdx.z;
    // query blocks in reverse order: under the causal mask the last rows see the most keys,
    // so the longest blocks are dispatched first and the short ones fill the tail
    const int qbi = (int)gridDim.y - 1 - (int)blockIdx.y;
    int rbase = 0, Mr = M;  // first stacked row of this stream, its row count
    if (BAT) {
        const int zb = (int)blockIdx.z / ns;
        rbase = er.off[zb];
        Mr = er.nr[zb];
        q_pos0 = er.pos0[zb];
        Kc = er.Kc[zb];
        Vc = er.Vc[zb];
        if (qbi * 16 >= Mr) return;  // uniform per block
    }
    const int h = blockIdx.x, q0 = qbi * 16;
    const int kvh = h / (H / KVH), kvd = KVH * HD;
    const int nq = min(16, Mr - q0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int j = lane & 15, g = lane >> 4;
    float qv[DG];
    {
        const float* qr = Q + (size_t)(rbase + q0 + j) * ldq + h * HD + g * DG;
#pragma unroll
        for (int t = 0; t < DG; t += 4) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (j < nq) v = *reinterpret_cast<const float4*>(qr + t);
            qv[t] = v.x; qv[t + 1] = v.y; qv[t + 2] = v.z; qv[t + 3] = v.w;
        }
    }
    const int qfirst = q_pos0 + q0, qlast = q_pos0 + q0 + nq - 1;
    int kstart = max(qfirst - window + 1, k_first);
    int kend = qlast;
    if (ns > 1) {
        const int span = ((kend - kstart + 1 + ns - 1) / ns + 15) / 16 * 16;
        kstart += zsplit * span;
        kend = min(kend, kstart + span - 1);
    }
    const int qp = q_pos0 + q0 + j;  // the query of this lane's S^T column
    float m = -1e30f, l = 0.f;
    f32x4 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K row kb + j (dims of group g) and V rows kb + 4g + c (dims [NB j, NB j + NB)); rows
    // past kend are clamped to it (their scores are masked)
    float kv[DG], vv[4][NB];
    auto load = [&](int kb, float* kd, float (*vd)[NB]) {
        const KT* kr = reinterpret_cast<const KT*>(Kc) + (size_t)(min(kb + j, kend) % cap) * kvd + kvh * HD + g * DG;
#pragma unroll
        for (int t = 0; t < DG; t += 4) {
            const float4 v = kv_ld4(kr + t);
            kd[t] = v.x; kd[t + 1] = v.y; kd[t + 2] = v.z; kd[t + 3] = v.w;
        }
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const KT* vr = reinterpret_cast<const KT*>(Vc) + (size_t)(min(kb + 4 * g + c, kend) % cap) * kvd + kvh * HD + NB * j;
#pragma unroll
            for (int b = 0; b < NB; b += 4) {
                const float4 v = kv_ld4(vr + b);
                vd[c][b] = v.x; vd[c][b + 1] = v.y; vd[c][b + 2] = v.z; vd[c][b + 3] = v.w;
            }
        }
    };
    int kb = kstart + wave * 16;
    if (kb <= kend) load(kb, kv, vv);
    for (; kb <= kend; kb += 64) {
        float kn[DG], vn[4][NB];
        if (kb + 64 <= kend) load(kb + 64, kn, vn);
        // S^T = K Q^T over two accumulators (alternate dims)
        f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = s0;
#pragma unroll
        for (int t = 0; t < DG; t += 2) {
            s0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[t], qv[t], s0, 0, 0, 0);
            s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[t + 1], qv[t + 1], s1, 0, 0, 0);
        }
        float p[4];
        float cmax = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int kp = kb + 4 * g + i;
            const bool valid = j < nq && kp <= kend && kp <= qp && kp >= qp - window + 1 && kp >= k_first;
            p[i] = valid ? (s0[i] + s1[i]) * scale : -INFINITY;
            cmax = fmaxf(cmax, p[i]);
        }
        cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
        cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
        const float mnew = fmaxf(m, cmax);
        float ps = 0.f;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            p[i] = (p[i] == -INFINITY) ? 0.f : expf(p[i] - mnew);
            ps += p[i];
        }
        ps += __shfl_xor(ps, 16, 64);
        ps += __shfl_xor(ps, 32, 64);
        const float alpha = expf(m - mnew);
        l = l * alpha + ps;
        m = mnew;
        // output rows 4g + i are queries 4g + i: their rescale factor sits on lane 4g + i
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float a = __shfl(alpha, 4 * g + i, 64);
#pragma unroll
            for (int b = 0; b < NB; b++) acc[b][i] *= a;
        }
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int b = 0; b < NB; b++) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(p[c], vv[c][b], acc[b], 0, 0, 0);
        if (kb + 64 <= kend) {
#pragma unroll
            for (int t = 0; t < DG; t++) kv[t] = kn[t];
#pragma unroll
            for (int c = 0; c < 4; c++)
#pragma unroll
                for (int b = 0; b < NB; b++) vv[c][b] = vn[c][b];
        }
    }
    // merge the waves: query r = tid >> 4, dims [(tid & 15) NB, +NB)
    if (g == 0) {
        sm[wave][j] = m;
        sl[wave][j] = l;
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int b = 0; b < NB; b++) so[wave][4 * g + i][NB * j + b] = acc[b][i];
    __syncthreads();
    const int r = tid >> 4, d0 = (tid & 15) * NB;
    if (r >= nq) return;
    float mx = -1e30f;
#pragma unroll
    for (int w = 0; w < 4; w++) mx = fmaxf(mx, sm[w][r]);
    float f[4], den = 0.f;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        f[w] = expf(sm[w][r] - mx);
        den = fmaf(f[w], sl[w][r], den);
    }
    float num[NB];
#pragma unroll
    for (int e = 0; e < NB; e++) {
        num[e] = 0.f;
#pragma unroll
        for (int w = 0; w < 4; w++) num[e] = fmaf(f[w], so[w][r][d0 + e], num[e]);
    }
    if (ns > 1) {
        float* pp = part + ((size_t)(h * M + rbase + q0 + r) * ns + zsplit) * (HD + 2);
#pragma unroll
        for (int e = 0; e < NB; e++) pp[d0 + e] = num[e];
        if ((tid & 15) == 0) {
            pp[HD] = mx;
            pp[HD + 1] = den;
        }
    } else if (xs) {
        // the output row straight into the fragment-major planes of the wo input (H * HD
        // columns; what k_split_fplanes made of O), four dims per 8-byte piece of each plane
        const float inv = den > 0.f ? 1.0f / den : 0.f;
        const int row = rbase + q0 + r, K = H * HD;
#pragma unroll
        for (int e0 = 0; e0 < NB; e0 += 4) {
            uint16_t hh[4], mm[4], ll[4];
#pragma unroll
            for (int e = 0; e < 4; e++) split3(num[e0 + e] * inv, hh[e], mm[e], ll[e]);
            const int k = h * HD + d0 + e0;
            *reinterpret_cast<uint2*>(xs + frag_at(row, K, 0, k)) = make_uint2(hh[0] | ((uint32_t)hh[1] << 16), hh[2] | ((uint32_t)hh[3] << 16));
            *reinterpret_cast<uint2*>(xs + frag_at(row, K, 1, k)) = make_uint2(mm[0] | ((uint32_t)mm[1] << 16), mm[2] | ((uint32_t)mm[3] << 16));
            *reinterpret_cast<uint2*>(xs + frag_at(row, K, 2, k)) = make_uint2(ll[0] | ((uint32_t)ll[1] << 16), ll[2] | ((uint32_t)ll[3] << 16));
        }
    } else {
        const float inv = den > 0.f ? 1.0f / den : 0.f;
        float* op = O + (size_t)(rbase + q0 + r) * ldo + h * HD + d0;
#pragma unroll
        for (int e = 0; e < NB; e++) op[e] = num[e] * inv;
    }
}

// merge of k_attn_mf's ns key-range partials: one block per (head, query row); with xs the
// row goes straight into the fragment-major planes of the wo input (H * HD columns)
template <int HD>
__global__ __launch_bounds__(HD) void k_attn_tiled_combine(const float* __restrict__ part, int ns, int M,
                                                           float* __restrict__ O, int ldo, uint16_t* __restrict__ xs) {
    __shared__ __attribute__((aligned(16))) float sv[HD];
    const int h = blockIdx.x, q = blockIdx.y, d = threadIdx.x;
    const float* pp = part + (size_t)(h * M + q) * ns * (HD + 2);
    // every split's (max, sum, value) loads in flight together (chunks of 8 splits); the
    // merge runs in split order as before
    float mx = -1e30f, num = 0.f, den = 0.f;
    for (int z0 = 0; z0 < ns; z0 += 8) {
        float zm[8], zl[8], zv[8];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const float* pz = pp + (size_t)min(z0 + c, ns - 1) * (HD + 2);
            zm[c] = pz[HD];
            zl[c] = pz[HD + 1];
            zv[c] = pz[d];
        }
        // rescale the running sums when a later chunk raises the max
        float cm = mx;
#pragma unroll
        for (int c = 0; c < 8; c++)
            if (z0 + c < ns) cm = fmaxf(cm, zm[c]);
        if (cm > mx) {
            const float r = expf(mx - cm);
            num *= r;
            den *= r;
            mx = cm;
        }
#pragma unroll
        for (int c = 0; c < 8; c++)
            if (z0 + c < ns) {
                const float f = expf(zm[c] - mx);
                den = fmaf(f, zl[c], den);
                num = fmaf(f, zv[c], num);
            }
    }
    const float v = den > 0.f ? num * (1.0f / den) : 0.f;
    if (!xs) {
        O[(size_t)q * ldo + h * HD + d] = v;
        return;
    }
    sv[d] = v;
    __syncthreads();
    if (d < HD / 8) {
        const float4 a = *reinterpret_cast<const float4*>(&sv[d * 8]), b = *reinterpret_cast<const float4*>(&sv[d * 8 + 4]);
        const float w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t hp[4], mp[4], lp[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            uint16_t h0, m0, l0, h1, m1, l1;
            split3(w[e], h0, m0, l0);
            split3(w[e + 1], h1, m1, l1);
            hp[e / 2] = h0 | ((uint32_t)h1 << 16);
            mp[e / 2] = m0 | ((uint32_t)m1 << 16);
            lp[e / 2] = l0 | ((uint32_t)l1 << 16);
        }
        const int K = gridDim.x * HD, k = h * HD + d * 8;
        *reinterpret_cast<uint4*>(xs + frag_at(q, K, 0, k)) = make_uint4(hp[0], hp[1], hp[2], hp[3]);
        *reinterpret_cast<uint4*>(xs + frag_at(q, K, 1, k)) = make_uint4(mp[0], mp[1], mp[2], mp[3]);
        *reinterpret_cast<uint4*>(xs + frag_at(q, K, 2, k)) = make_uint4(lp[0], lp[1], lp[2], lp[3]);
    }
}

// ============================================================================
// M=1 weight-streaming GEMV with fused prologue / epilogue (decoder step).
//
// A block (4 waves) owns groups of RB rows and streams them with K split across its
// waves: wave w reads the 1-KiB chunk blocks j*4+w of every row, so each wave keeps only
// its quarter of x in registers (loaded once per block, normalised there when PRO_NORM),
// never stages x through LDS, and a launch needs no more blocks than CUs x 4 to stay
// balanced (grid-stride over groups).  Weights: 16-B non-temporal loads straight to
// VGPRs (cdna_hip_programming.md "GEMV / M <= 16" row).  Partial sums meet in LDS; wave
// 0 applies the epilogue.  Summation order is fixed (deterministic).
// ============================================================================
// stream_fill_alts (voxtral.c:955-1010) partials for one logit: running max / sum of
// exp for the softmax, and an ascending-id-stable top-4 of ids >= TOKEN_TEXT_MIN (rows
// arrive in ascending order, so a strict '>' keeps the lower id first on ties).
__device__ __forceinline__ void alt_row(float v, int r, float& am, float& as, float (&tv)[4], int (&ti)[4]) {
    if (v > am) {
        as = as * expf(am - v) + 1.0f;
        am = v;
    } else {
        as += expf(v - am);
    }
    if (r >= ALT_TEXT_MIN && v > tv[3]) {
        int k = 3;
        while (k > 0 && v > tv[k - 1]) {
            tv[k] = tv[k - 1];
            ti[k] = ti[k - 1];
            k--;
        }
        tv[k] = v;
        ti[k] = r;
    }
}

template <int EPI, int RB>
__device__ __forceinline__ void gemv_rows(int g, int (&rows)[RB]) {
#pragma unroll
    for (int i = 0; i < RB; i++) {
        if (EPI == EPI_SWIGLU) {
            // pair i = (w1 row, w3 row) of hidden unit u = g*RB/2 + i/2 (16-row interleave)
            const int u = g * (RB / 2) + (i >> 1);
            rows[i] = ((u >> 4) << 5) + (u & 15) + ((i & 1) << 4);
        } else {
            rows[i] = g * RB + i;
        }
    }
}

// Weight rows come in through a buffer descriptor: the row offset is wave-uniform (an SGPR
// soffset) and each lane keeps one 32-bit chunk offset per K round (voff), instead of a
// 64-bit address per (row, round) -- the register count sets how many blocks stay resident.
// Non-temporal (aux = 2: nt): every weight byte is read once per step.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int RB, int KQ>
__device__ __forceinline__ void gemv_load(__amdgpu_buffer_rsrc_t W, int rowbytes, const int (&rows)[RB],
                                          const int (&voff)[KQ], uint4 (&wv)[KQ][RB]) {
#pragma unroll
    for (int j = 0; j < KQ; j++)
#pragma unroll
        for (int i = 0; i < RB; i++) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(W, voff[j], rows[i] * rowbytes, 2);
            wv[j][i] = make_uint4(v.x, v.y, v.z, v.w);
        }
}

// Q8 rows (WQ8): 16-B chunks of 16 int8, so a lane holds 16 x values per chunk, and the
// group's RB row scales are fetched with its weights (applied before the epilogue:
// y = scale * sum + bias, voxtral_kernels.c:316).
#ifdef VOX_GEMV_STAMPS
// diagnostic build only (tools/kbench_stamps): per block s_memrealtime at entry, when the
// first group's weights have been consumed, and at exit
__device__ unsigned long long* g_gemv_stamps;
#define GEMV_STAMP(k) \
    do { if (g_gemv_stamps && tid == 0) g_gemv_stamps[(size_t)blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define GEMV_STAMP(k) do {} while (0)
#endif

template <int PRO, int EPI, int RB, int KQ, int WQ8>
__global__ __launch_bounds__(256) void k_gemv(GemvArgs a) {
    constexpr int XPC = WQ8 ? 4 : 2;  // float4 of x per 16-B chunk
    __shared__ float red[2][4][RB];
    __shared__ float sred[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int K = a.K, KC = WQ8 ? K >> 4 : K >> 3;
    const int ngroups = a.rows / RB;
    // Groups: block b takes b, b + G, b + 2G, ... (static; run-time claims measured 3-4x
    // slower)
    const int G = gridDim.x;
    int g = blockIdx.x;
    int rows[RB];
    uint4 wv[KQ][RB];
    float wsc[RB];
    GEMV_STAMP(0);
    bool first_group = true;
    const int rowbytes = K * (WQ8 ? 1 : 2);
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), 0, a.rows * rowbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wnone = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.W), 0, 0, 0x00020000);
    // chunk offsets per K round; chunks past K (K not a multiple of 16 B * 256) re-load
    // chunk 0 and meet x = 0: every load is unconditional, so hipcc issues them all before
    // the first wait (a guarded load makes it wait vmcnt(0) at each branch join)
    int voff[KQ];
#pragma unroll
    for (int j = 0; j < KQ; j++) {
        const int c0 = (j * 4 + wave) * 64 + lane;
        voff[j] = (c0 < KC ? c0 : 0) * 16;
    }
    // first group's weights are independent of x: issue them before the prologue
    gemv_rows<EPI, RB>(g, rows);
    gemv_load<RB, KQ>(wrs, rowbytes, rows, voff, wv);
    if ((EPI == EPI_LOGITS || EPI == EPI_LOGITS_ALT) && WQ8 && wave == 0) {
#pragma unroll
        for (int i = 0; i < RB; i++) wsc[i] = a.wscale[rows[i]];
    }

    float4 xr[KQ][XPC];
    // bf16: the RMSNorm weights (and ada) go out with x -- independent of the row sum, so the
    // prologue waits for one L2 round trip instead of two (C2 +0.7 %, W1|W3 21.0 -> 20.8 us);
    // Q8 (16 x values per chunk) keeps them after the sum: the early registers cost it 0.5 %
    // (profiles/r5_gemv_prologue_ab.txt)
    constexpr bool EARLY = PRO != PRO_NONE && !WQ8;
    constexpr int NXP = EARLY ? XPC : 1;
    float4 nwr[KQ][NXP], adr[KQ][NXP];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < KQ; j++) {
        const int c = (j * 4 + wave) * 64 + lane;
        const float4* xp = reinterpret_cast<const float4*>(a.x) + XPC * (c < KC ? c : 0);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int h = 0; h < XPC; h++) {
            const float4 xv = xp[h];
            xr[j][h] = c < KC ? xv : z;
        }
        if (EARLY) {
            const int cc = c < KC ? c : 0;
            const float4* wp = reinterpret_cast<const float4*>(a.norm_w) + XPC * cc;
            const float4* ap = reinterpret_cast<const float4*>(PRO == PRO_NORM_ADA ? a.ada : a.norm_w) + XPC * cc;
#pragma unroll
            for (int h = 0; h < NXP; h++) {
                nwr[j][h] = wp[h];
                if (PRO == PRO_NORM_ADA) adr[j][h] = ap[h];
            }
        }
        if (PRO != PRO_NONE) {
#pragma unroll
            for (int h = 0; h < XPC; h++) {
                const float4 v = xr[j][h];
                ss = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, fmaf(v.w, v.w, ss))));
            }
        }
    }
    if (PRO != PRO_NONE) {
        // RMSNorm prologue (voxtral_kernels.c:475-492; ada: voxtral_decoder.c:742-745)
        ss = wave_sum(ss);
        if (lane == 0) sred[wave] = ss;
        __syncthreads();
        const float tot = sred[0] + sred[1] + sred[2] + sred[3];
        const float inv = 1.0f / sqrtf(tot / (float)K + a.eps);
#pragma unroll
        for (int j = 0; j < KQ; j++) {
            const int c0 = (j * 4 + wave) * 64 + lane;
            const int c = c0 < KC ? c0 : 0;
            const float4* wp = reinterpret_cast<const float4*>(a.norm_w) + XPC * c;
            const float4* ap = reinterpret_cast<const float4*>(PRO == PRO_NORM_ADA ? a.ada : a.norm_w) + XPC * c;
#pragma unroll
            for (int h = 0; h < XPC; h++) {
                float4 v = xr[j][h];
                const float4 nw = EARLY ? nwr[j][h % NXP] : wp[h];
                v.x = v.x * inv * nw.x; v.y = v.y * inv * nw.y;
                v.z = v.z * inv * nw.z; v.w = v.w * inv * nw.w;
                if (PRO == PRO_NORM_ADA) {
                    const float4 ad = EARLY ? adr[j][h % NXP] : ap[h];
                    v.x *= (1.0f + ad.x); v.y *= (1.0f + ad.y);
                    v.z *= (1.0f + ad.z); v.w *= (1.0f + ad.w);
                }
                xr[j][h] = v;
            }
        }
    }

    constexpr bool QKVE = (EPI == EPI_QKV || EPI == EPI_QKV_BIAS);
    int lp = 0;
    if (QKVE) lp = a.state ? a.state[0] : a.pos;
    float best = -INFINITY;
    int besti = 0x7fffffff;
    // EPI_LOGITS_ALT: online softmax partial (max, sum exp) and the 4 largest text logits
    float am = -INFINITY, as = 0.f, tv[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int ti[4] = {-1, -1, -1, -1};
    // Epilogue ownership: lane l of wave 0 finishes row l (STORE / RESID) or row pair
    // (2l, 2l+1) (QKV rope pairs, SWIGLU w1/w3 pairs), so the epilogue's reads (residual,
    // bias, rope, Q8 scales) go out in parallel at the top of the iteration instead of one
    // dependent round trip per row after the reduction.  The LM head keeps one lane (its
    // running argmax is sequential over ascending rows).
    constexpr bool LOGIT = (EPI == EPI_LOGITS || EPI == EPI_LOGITS_ALT);
    constexpr bool PAIRED = (QKVE || EPI == EPI_SWIGLU);
    constexpr int NL = LOGIT ? 1 : (PAIRED ? RB / 2 : RB);
    const bool owner = wave == 0 && lane < NL;
    const int i0 = PAIRED ? 2 * lane : lane;
    int buf = 0;
    for (;;) {
        const int gcur = g;
        // epilogue inputs of this group (independent of the dot products)
        int er0 = 0, er1 = 0;
        float ein0 = 0.f, ein1 = 0.f, esc0 = 1.f, esc1 = 1.f, eb0 = 0.f, eb1 = 0.f;
        if (!LOGIT && owner) {
            int rr[RB];
            gemv_rows<EPI, RB>(gcur, rr);
#pragma unroll
            for (int i = 0; i < RB; i++) {
                if (i == i0) er0 = rr[i];
                if (i == i0 + 1) er1 = rr[i];
            }
            if (WQ8) {
                esc0 = a.wscale[er0];
                if (PAIRED) esc1 = a.wscale[er1];
            }
            if (EPI == EPI_RESID) ein0 = a.y[er0] + (a.bias ? a.bias[er0] : 0.f);
            if (EPI == EPI_STORE) ein0 = a.bias ? a.bias[er0] : 0.f;
            if (EPI == EPI_QKV_BIAS) {
                eb0 = a.bias[er0];
                eb1 = a.bias[er1];
            }
            if (QKVE && er0 < a.qd + a.kvd) {
                const int col = er0 < a.qd ? er0 : er0 - a.qd;
                const float* rp = a.rope + (size_t)lp * a.hd + ((col % a.hd) & ~1);
                ein0 = rp[0];
                ein1 = rp[1];
            }
        }
        float acc[RB];
#pragma unroll
        for (int i = 0; i < RB; i++) acc[i] = 0.f;
#pragma unroll
        for (int j = 0; j < KQ; j++)
#pragma unroll
            for (int i = 0; i < RB; i++) {
                if (WQ8) acc[i] = dot16q(wv[j][i], reinterpret_cast<const float4(&)[4]>(xr[j]), acc[i]);
                else acc[i] = dot8(wv[j][i], xr[j][0], xr[j][XPC - 1], acc[i]);
            }
        if (first_group) {
            GEMV_STAMP(1);
            first_group = false;
        }
        int rcur[RB];
        float scur[RB];
        if (LOGIT) {
#pragma unroll
            for (int i = 0; i < RB; i++) {
                rcur[i] = rows[i];
                scur[i] = WQ8 ? wsc[i] : 1.0f;
            }
        }
        g += G;
        // The next group's loads go out before this group's reduction, unconditionally: a
        // load under `if (more)` keeps the old weight registers alive across the branch and
        // doubles the weight register set (fewer resident blocks).  Past the last group they
        // go through a zero-length descriptor: the range check returns zeros, no traffic.
        {
            const bool more = g < ngroups;
            gemv_rows<EPI, RB>(more ? g : 0, rows);
            gemv_load<RB, KQ>(more ? wrs : wnone, rowbytes, rows, voff, wv);
            if (LOGIT && WQ8 && wave == 0) {
#pragma unroll
                for (int i = 0; i < RB; i++) wsc[i] = a.wscale[rows[i]];
            }
        }
#pragma unroll
        for (int i = 0; i < RB; i++) acc[i] = wave_sum(acc[i]);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < RB; i++) red[buf][wave][i] = acc[i];
        }
        __syncthreads();
        if (!LOGIT && owner) {
            float v0 = ((red[buf][0][i0] + red[buf][1][i0]) + red[buf][2][i0]) + red[buf][3][i0];
            float v1 = 0.f;
            if (PAIRED) v1 = ((red[buf][0][i0 + 1] + red[buf][1][i0 + 1]) + red[buf][2][i0 + 1]) + red[buf][3][i0 + 1];
            if (WQ8) {
                v0 *= esc0;
                v1 *= esc1;
            }
            if (EPI == EPI_QKV_BIAS) {
                v0 += eb0;
                v1 += eb1;
            }
            if (EPI == EPI_STORE || EPI == EPI_RESID) {
                a.y[er0] = ein0 + v0;  // RESID: residual + bias were read at the top
            } else if (EPI == EPI_SWIGLU) {
                a.y[gcur * (RB / 2) + lane] = silu(v0) * v1;
            } else if (QKVE) {
                if (er0 < a.qd + a.kvd) {
                    const float o0 = v0 * ein0 - v1 * ein1, o1 = v0 * ein1 + v1 * ein0;
                    if (er0 < a.qd) {
                        a.y[er0] = o0;
                        a.y[er1] = o1;
                    } else {
                        kv_st2_rt(a.Kc, (size_t)(lp % a.cap) * a.kvd + (er0 - a.qd), o0, o1, a.kv16);
                    }
                } else {
                    kv_st2_rt(a.Vc, (size_t)(lp % a.cap) * a.kvd + (er0 - a.qd - a.kvd), v0, v1, a.kv16);
                }
            }
        }
        if (LOGIT && wave == 0 && lane == 0) {
            float v[RB];
#pragma unroll
            for (int i = 0; i < RB; i++) {
                v[i] = ((red[buf][0][i] + red[buf][1][i]) + red[buf][2][i]) + red[buf][3][i];
                if (WQ8) v[i] *= scur[i];
            }
#pragma unroll
            for (int i = 0; i < RB; i++) {
                a.y[rcur[i]] = v[i];
                // first max wins (voxtral_decoder.c:771-779): rows ascend within a block
                if (v[i] > best) { best = v[i]; besti = rcur[i]; }
                if (EPI == EPI_LOGITS_ALT) alt_row(v[i], rcur[i], am, as, tv, ti);
            }
        }
        buf ^= 1;
        if (g >= ngroups) break;
    }
    GEMV_STAMP(2);
    if ((EPI == EPI_LOGITS || EPI == EPI_LOGITS_ALT) && wave == 0 && lane == 0) {
        a.part_val[blockIdx.x] = best;
        a.part_idx[blockIdx.x] = besti;
        if (EPI == EPI_LOGITS_ALT) {
            float* pa = a.part_alt + (size_t)blockIdx.x * ALT_PART;
            pa[0] = am;
            pa[1] = as;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                pa[2 + k] = tv[k];
                pa[6 + k] = __int_as_float(ti[k]);
            }
        }
    }
}

// ============================================================================
// Decode attention (one query per head, GQA group of <= 4 heads per kv head).
// Keys: the last min(lp+1, window) logical positions (voxtral_decoder.c:731-733 after
// compaction; voxtral_kernels.c:554-560).  A block owns up to 256 consecutive keys and HPB
// query heads of one kv head; each of its 16 waves takes 16 keys (lanes = key x quarter of
// head_dim for Q.K, lanes = dims for P.V, every K/V load shared by the block's heads) and
// the waves merge in LDS.  HPB = 1 (short contexts): one block per query head, so the
// Q.K / P.V issue work of a kv head spreads over 4 CUs; the grid's y index is laid out so
// that the 4 blocks of one kv head land on one XCD (blocks b and b+8 share an L2) and read
// the K/V rows through the same L2.  HPB = 4 (long contexts): one block per kv head and
// 256-key split, K/V read once.  With one split the block writes the attention output
// directly; otherwise it writes an (o, m, l) partial and the last of the split blocks of a
// kv head to arrive merges them (arrival count past the partials).
// ============================================================================
// NWV = waves per block: 16 (256 keys: one block per head covers short contexts, no
// combine) or 8 (128-key blocks for long contexts: twice the blocks, half the K/V bytes per
// CU; tools/kbench: L = 4096 11.9 us against 14.5 with 64-key and 19.2 with 32-key blocks).
constexpr int ATT_CH = 16;      // keys per wave
constexpr int ATT_WAVES = 16;   // waves per short-context block (1024 threads)
constexpr int ATT_BK = ATT_CH * ATT_WAVES;  // keys per short-context block
constexpr int ATT_LWAVES = 8;   // waves per long-context block (512 threads)
constexpr int ATT_LBK = ATT_CH * ATT_LWAVES;  // keys per long-context block
constexpr int ATT_MIN_BK = 64;      // smallest block (kbench variant): sizes the partials
constexpr int ATT_MAX_PARTS = 128;  // partials per head the merging block combines

template <int HD, int HPB, int DBG = 0, int FUSE = 0, int NWV = ATT_WAVES, class KT = float>
__global__ __launch_bounds__(NWV * 64) void k_attn_decode(const AttnPtrs P, int cap, int pos_host,
                                                          int window, float scale, int H, int KVH,
                                                          int maxs, const AttnFuse F = AttnFuse{}, int kvfast = 0) {
    constexpr int NT = NWV * 64, BK = NWV * ATT_CH;
    const int zb = blockIdx.z;  // stream of a batched step (0 for a single stream)
    // batched step: ring, position and liveness from the slot table (a stopped slot's blocks
    // leave at once; uniform per block)
    const BatchSlot* __restrict__ sl = P.slots ? P.slots + zb : nullptr;
    if (sl && !sl->live) return;
    const float* __restrict__ q = P.q[zb];
    const KT* __restrict__ Kc = reinterpret_cast<const KT*>(sl ? sl->Kc + P.ring_off : (const char*)P.Kc[zb]);
    const KT* __restrict__ Vc = reinterpret_cast<const KT*>(sl ? sl->Vc + P.ring_off : (const char*)P.Vc[zb]);
    const int* __restrict__ state = sl ? nullptr : P.state[zb];
    float* __restrict__ part = P.part[zb];
    float* __restrict__ out = P.out[zb];
    constexpr int DQ = HD / 4;   // dims per lane for Q.K
    constexpr int DPL = HD / 64; // dims per lane for P.V
    __shared__ __attribute__((aligned(16))) float sQ[HPB][HD];
    __shared__ float sM[NWV][4], sL[NWV][4];
    __shared__ __attribute__((aligned(16))) float sO[NWV][HPB][HD];
    __shared__ __attribute__((aligned(16))) float sKn[FUSE ? HD : 1], sVn[FUSE ? HD : 1];  // the new key's K / V
    const int hpk = H / KVH;
    // kvfast (HPB 4): grid x = key range * KVH + kv head, so the kv heads of one key range (the
    // 8 slices of the same K/V rows) are neighbouring blocks
    const int kvh = HPB == 1 ? (int)blockIdx.y % KVH : kvfast ? (int)blockIdx.x % KVH : (int)blockIdx.y;
    const int h0 = HPB == 1 ? kvh * hpk + (int)blockIdx.y / KVH : kvh * hpk;  // first query head
    const int nh = HPB == 1 ? 1 : hpk;  // heads in this block (<= 4)
    const int sb = (HPB != 1 && kvfast) ? (int)blockIdx.x / KVH : (int)blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kvd = KVH * HD;
    unsigned long long ts[10];
    if (DBG == 4) {
        ts[0] = __builtin_amdgcn_s_memtime();
        ts[8] = __builtin_amdgcn_s_memrealtime();
    }
    // DBG 4: the wave's phase stamps to part[0] (single stream: [y][wave]) or, fused batched,
    // to out[0] ([z][y][x][wave])
    auto dbg_dump = [&]() {
        if (DBG == 4) {
            ts[5] = __builtin_amdgcn_s_memtime();
            ts[9] = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) {
                const size_t bi = P.slots ? (((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * NWV
                                          : (size_t)blockIdx.y * 16;
                unsigned long long* d = reinterpret_cast<unsigned long long*>(FUSE ? P.out[0] : P.part[0]) + (bi + wave) * 10;
                for (int i = 0; i < 10; i++) d[i] = ts[i];
            }
        }
    };
    // the query does not depend on the step state: its load goes out first
    constexpr int QPT = (HPB * HD + NT - 1) / NT;
    float qreg[QPT];
#pragma unroll
    for (int i = 0; i < QPT; i++) qreg[i] = (!FUSE && tid + i * NT < nh * HD) ? q[(size_t)h0 * HD + tid + i * NT] : 0.f;
    const int lp = sl ? sl->pos : state ? state[0] : pos_host;
    const int L = min(lp + 1, window);
    const int first = lp - L + 1;
    const int S = (L + BK - 1) / BK;
    if (sb >= S) return;  // uniform per block
    const int k0 = first + sb * BK + wave * ATT_CH;  // >= 0
    const int kn = min(ATT_CH, lp + 1 - k0);  // may be <= 0 for trailing waves
    const int kk = lane & 15, dq = lane >> 4;
    // ring slots: one modulo per wave, then a wrap test per key
    const int slot0 = k0 % cap;

    // K and V of this wave's 16 keys.  KROW (head_dim 128): load i covers 8 keys x one
    // 128-B quarter row (lane = key (lane >> 3) + 8 (i & 1), 16 B at (lane & 7)), so a wave
    // instruction touches 8 whole cache lines instead of 16 B of 64 lines: the CU's address
    // path took 6400 cycles per wave for the quarter-row-per-lane pattern (tools/kbench DBG 4).
    constexpr bool KROW = (HD == 128);
    float4 kv[DQ / 4];
    float vv[ATT_CH][DPL];
    {
        if (KROW) {
#pragma unroll
            for (int i = 0; i < DQ / 4; i++) {
                const int key = (lane >> 3) + 8 * (i & 1);
                int sk = slot0 + (key < kn ? key : 0);
                sk = sk >= cap ? sk - cap : sk;
                kv[i] = kv_ld4(Kc + (size_t)sk * kvd + kvh * HD + (i >> 1) * DQ + (lane & 7) * 4);
            }
        } else {
            int sk = slot0 + (kk < kn ? kk : 0);
            sk = sk >= cap ? sk - cap : sk;
            const KT* kr = Kc + (size_t)sk * kvd + kvh * HD + dq * DQ;
#pragma unroll
            for (int i = 0; i < DQ / 4; i++) kv[i] = kv_ld4(kr + 4 * i);
        }
#pragma unroll
        for (int k = 0; k < ATT_CH; k++) {
            int sv = slot0 + (k < kn ? k : 0);
            sv = sv >= cap ? sv - cap : sv;
            const KT* vr = Vc + (size_t)sv * kvd + kvh * HD + lane * DPL;
            if (DPL == 2) {
                const float2 t = kv_ld2(vr);
                vv[k][0] = t.x;
                vv[k][DPL - 1] = t.y;
            } else {
                vv[k][0] = (float)vr[0];
            }
        }
    }
    if (DBG == 4) ts[6] = __builtin_amdgcn_s_memtime();
    const bool holds_new = sb == S - 1;  // the split whose keys end at the new position lp
    if (FUSE) {
        // RoPE of this block's query heads and, in the split holding lp, of the new key plus
        // the KV append (voxtral_decoder.c:709-722), from the QKV slabs of stream zb; the
        // cache loads above went out first (the new key's K / V come from LDS below)
        const int qd = H * HD;
        const float* rp = F.rope + (size_t)lp * HD;
        const size_t slot = (size_t)(lp % cap) * kvd + kvh * HD;
        // jobs: query pairs [0, nq), then (split holding lp) new-key pairs and new-value dims
        const int nq = nh * HD / 2, nj = nq + (holds_new ? HD / 2 + HD : 0);
        for (int j = tid; j < nj; j += NT) {
            if (j < nq) {
                const int h = j / (HD / 2), d = j % (HD / 2);
                const int col = (h0 + h) * HD + 2 * d;
                const float2 xx = psum2(F.qkv, F.S, F.N, zb, col);
                const float x0 = xx.x, x1 = xx.y;
                const float c = rp[2 * d], sn = rp[2 * d + 1];
                sQ[h][2 * d] = x0 * c - x1 * sn;
                sQ[h][2 * d + 1] = x0 * sn + x1 * c;
            } else if (j < nq + HD / 2) {
                const int d = j - nq, col = qd + kvh * HD + 2 * d;
                const float2 xx = psum2(F.qkv, F.S, F.N, zb, col);
                const float x0 = xx.x, x1 = xx.y;
                const float c = rp[2 * d], sn = rp[2 * d + 1];
                // the new key as the cache holds it (rounded in the 16-bit mode)
                const float k0v = kv_round<KT>(x0 * c - x1 * sn), k1v = kv_round<KT>(x0 * sn + x1 * c);
                sKn[2 * d] = k0v;
                sKn[2 * d + 1] = k1v;
                kv_st2(const_cast<KT*>(Kc) + slot + 2 * d, k0v, k1v);
            } else {
                const int e = j - nq - HD / 2;
                const float v = kv_round<KT>(psum(F.qkv, F.S, F.N, zb, qd + kvd + kvh * HD + e));
                sVn[e] = v;
                const_cast<KT*>(Vc)[slot + e] = (KT)v;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < QPT; i++)
            if (tid + i * NT < nh * HD) sQ[(tid + i * NT) / HD][(tid + i * NT) % HD] = qreg[i];
    }
    if (DBG == 4) {
        __builtin_amdgcn_s_waitcnt(0);
        ts[7] = __builtin_amdgcn_s_memtime();
    }
    __syncthreads();
    if (FUSE && holds_new && lp >= k0 && lp < k0 + ATT_CH) {
        // this wave holds the new key (wave-uniform test): its K / V from LDS
        const int kl = lp - k0;
        if (KROW) {
            if ((lane >> 3) == (kl & 7)) {
#pragma unroll
                for (int i = 0; i < DQ / 4; i++)
                    if ((i & 1) == (kl >> 3)) kv[i] = *reinterpret_cast<const float4*>(&sKn[(i >> 1) * DQ + (lane & 7) * 4]);
            }
        } else if (kk == kl) {
#pragma unroll
            for (int i = 0; i < DQ / 4; i++) kv[i] = *reinterpret_cast<const float4*>(&sKn[dq * DQ + 4 * i]);
        }
#pragma unroll
        for (int k = 0; k < ATT_CH; k++)
            if (k == kl)
#pragma unroll
                for (int e = 0; e < DPL; e++) vv[k][e] = sVn[lane * DPL + e];
    }
    if (DBG == 4) ts[1] = __builtin_amdgcn_s_memtime();
    if (DBG == 3) {
        if (lane == 0) out[wave] = kv[0].x + vv[3][0];
        return;
    }

    float m[HPB], l[HPB], p[HPB], pb[HPB], o[HPB][DPL];
    if (KROW) {
        // lane (key r = lane >> 3, chunk c = lane & 7) sums its 16 dims of keys r and r + 8;
        // the 8 chunk lanes meet by DPP (xor 1, xor 2, half-row mirror), the 8 key groups by
        // row mirror and two cross-row shuffles
        const int r = lane >> 3, c = lane & 7;
#pragma unroll
        for (int h = 0; h < HPB; h++) {
            float aa = 0.f, ab = 0.f;
            if (h < nh) {
#pragma unroll
                for (int i = 0; i < DQ / 4; i++) {
                    const float4 qv = *reinterpret_cast<const float4*>(&sQ[h][(i >> 1) * DQ + c * 4]);
                    float& acc = (i & 1) ? ab : aa;
                    acc = fmaf(qv.x, kv[i].x, acc);
                    acc = fmaf(qv.y, kv[i].y, acc);
                    acc = fmaf(qv.z, kv[i].z, acc);
                    acc = fmaf(qv.w, kv[i].w, acc);
                }
            }
            aa += dpp<0xB1>(aa); aa += dpp<0x4E>(aa); aa += dpp<0x141>(aa);
            ab += dpp<0xB1>(ab); ab += dpp<0x4E>(ab); ab += dpp<0x141>(ab);
            const float sa = (r < kn) ? aa * scale : -INFINITY, sbv = (r + 8 < kn) ? ab * scale : -INFINITY;
            float mx = fmaxf(sa, sbv);
            mx = fmaxf(mx, dpp<0x140>(mx));
            mx = rows4_max(mx);  // the 4 rows of 16 lanes: 4 readlanes, no LDS round trip
            m[h] = (kn > 0) ? mx : -1e30f;
            p[h] = (r < kn) ? expf(sa - mx) : 0.f;
            pb[h] = (r + 8 < kn) ? expf(sbv - mx) : 0.f;
            float t = p[h] + pb[h];
            t += dpp<0x140>(t);
            t = rows4_sum(t);
            l[h] = t;
#pragma unroll
            for (int e = 0; e < DPL; e++) o[h][e] = 0.f;
        }
    } else {
        float sc[HPB];
#pragma unroll
        for (int h = 0; h < HPB; h++) {
            float acc = 0.f;
            if (h < nh) {
#pragma unroll
                for (int i = 0; i < DQ / 4; i++) {
                    const float4 qv = *reinterpret_cast<const float4*>(&sQ[h][dq * DQ + 4 * i]);
                    acc = fmaf(qv.x, kv[i].x, acc);
                    acc = fmaf(qv.y, kv[i].y, acc);
                    acc = fmaf(qv.z, kv[i].z, acc);
                    acc = fmaf(qv.w, kv[i].w, acc);
                }
            }
            acc += __shfl_xor(acc, 16, 64);
            acc += __shfl_xor(acc, 32, 64);
            sc[h] = (kk < kn) ? acc * scale : -INFINITY;
        }
#pragma unroll
        for (int h = 0; h < HPB; h++) {
            const float mx = row_max16(sc[h]);
            m[h] = (kn > 0) ? mx : -1e30f;
            p[h] = (kk < kn) ? expf(sc[h] - mx) : 0.f;
            pb[h] = 0.f;
            l[h] = row_sum16(p[h]);
#pragma unroll
            for (int e = 0; e < DPL; e++) o[h][e] = 0.f;
        }
    }
#pragma unroll
    for (int k = 0; k < ATT_CH; k++) {
#pragma unroll
        for (int h = 0; h < HPB; h++) {
            // the lane holding key k's weight (zero past the valid keys): a scalar broadcast
            const int src = KROW ? 8 * (k & 7) : k;
            const float pv = (KROW && k >= 8) ? pb[h] : p[h];
            const float pk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv), src));
#pragma unroll
            for (int e = 0; e < DPL; e++) o[h][e] = fmaf(pk, vv[k][e], o[h][e]);
        }
    }
    if (DBG == 1) {
        out[tid] = o[0][0] + m[0] + l[0];
        return;
    }
    if (DBG == 4) ts[2] = __builtin_amdgcn_s_memtime();
    // ---- merge the waves (in LDS): factors once per (wave, head), then a 16-term sum ----
    if (lane == 0) {
#pragma unroll
        for (int h = 0; h < HPB; h++) {
            sM[wave][h] = m[h];
            sL[wave][h] = l[h];
        }
    }
#pragma unroll
    for (int h = 0; h < HPB; h++)
        if (h < nh)
#pragma unroll
            for (int e = 0; e < DPL; e++) sO[wave][h][lane * DPL + e] = o[h][e];
    __syncthreads();
    if (DBG == 4) ts[3] = __builtin_amdgcn_s_memtime();
    // merge factors of head h, recomputed by every thread that needs them (no second barrier):
    // f_w = exp(m_w - M), den = sum f_w l_w added as the xor-4/8/16/32 lane tree did
    auto factors = [&](int h, float (&f)[NWV], float& den, float& M) {
        M = -1e30f;
#pragma unroll
        for (int i = 0; i < NWV; i++) M = fmaxf(M, sM[i][h]);
        float v[NWV];
#pragma unroll
        for (int w = 0; w < NWV; w++) {
            f[w] = expf(sM[w][h] - M);
            v[w] = f[w] * sL[w][h];
        }
#pragma unroll
        for (int st = 1; st < NWV; st *= 2)
#pragma unroll
            for (int w = 0; w < NWV; w += 2 * st) v[w] = v[w] + v[w + st];
        den = v[0];
    };
    if (DBG == 4) ts[4] = __builtin_amdgcn_s_memtime();
    if (FUSE && S == 1) {
        // output row zb straight into the wo input planes: 8 consecutive dims per thread
        for (int e = tid; e < nh * HD / 8; e += NT) {
            const int h = e / (HD / 8), d0 = (e % (HD / 8)) * 8;
            float fw[NWV], den, Mx;
            factors(h, fw, den, Mx);
            uint32_t hp[4], mp[4], lq[4];
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                float v2[2];
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    float num = 0.f;
#pragma unroll
                    for (int w = 0; w < NWV; w++) num = fmaf(fw[w], sO[w][h][d0 + i + u], num);
                    v2[u] = den > 0.f ? num * (1.0f / den) : 0.f;
                }
                uint16_t a0, b0, c0, a1, b1, c1;
                split3(v2[0], a0, b0, c0);
                split3(v2[1], a1, b1, c1);
                hp[i / 2] = a0 | ((uint32_t)a1 << 16);
                mp[i / 2] = b0 | ((uint32_t)b1 << 16);
                lq[i / 2] = c0 | ((uint32_t)c1 << 16);
            }
            const int kq = (h0 + h) * HD + d0;
            *reinterpret_cast<uint4*>(F.xs + frag_at(zb, H * HD, 0, kq)) = make_uint4(hp[0], hp[1], hp[2], hp[3]);
            *reinterpret_cast<uint4*>(F.xs + frag_at(zb, H * HD, 1, kq)) = make_uint4(mp[0], mp[1], mp[2], mp[3]);
            *reinterpret_cast<uint4*>(F.xs + frag_at(zb, H * HD, 2, kq)) = make_uint4(lq[0], lq[1], lq[2], lq[3]);
        }
        dbg_dump();
        return;
    }
    // partials (S > 1) go out write-through (sc1, like k_gemmf's partial tiles): the block
    // that merges them may sit on another XCD, behind another L2
    const __amdgpu_buffer_rsrc_t Pr = __builtin_amdgcn_make_buffer_rsrc(part, 0, 0x7fffffff, 0x00020000);
    for (int e = tid; e < nh * HD; e += NT) {
        const int h = e / HD, d = e % HD;
        float fw[NWV], den, Mx;
        factors(h, fw, den, Mx);
        float num = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; w++) num = fmaf(fw[w], sO[w][h][d], num);
        const int hh = h0 + h;
        if (S == 1) {
            out[(size_t)hh * HD + d] = den > 0.f ? num * (1.0f / den) : 0.f;
        } else {
            const int po = (int)(((size_t)hh * maxs + sb) * (HD + 2)) * 4;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(num), Pr, po + d * 4, 0, 16);
            if (d == 0) {
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(Mx), Pr, po + HD * 4, 0, 16);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(den), Pr, po + (HD + 1) * 4, 0, 16);
            }
        }
    }
    if (S > 1 && (DBG == 0 || DBG == 4)) {
        // the last of the S blocks of this kv head to finish merges the S partials of its
        // heads (the former k_attn_combine, one launch and its gap fewer per layer): stores
        // drained, one arrival count per (stream, kv head) just past the partials, reset by
        // the merging block for the next launch
        __shared__ int sLast;
        __shared__ float sCf[4][ATT_MAX_PARTS];
        __shared__ float sCden[4];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* cnt = reinterpret_cast<int*>(part + (size_t)H * maxs * (HD + 2)) + kvh;
        if (tid == 0) sLast = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
        __syncthreads();
        if (!sLast) {
            dbg_dump();
            return;
        }
        if (DBG == 4) ts[4] = __builtin_amdgcn_s_memtime();  // the merging block: ts5 - ts4 = merge
        auto pnum = [&](int h, int k, int d) {
            return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                Pr, (int)(((size_t)(h0 + h) * maxs + k) * (HD + 2) + d) * 4, 0, 16));
        };
        // output (h, d) = e of thread tid: its first 32 partial values go out before the merge
        // factors are known, so partials, maxima and sums share one round trip
        constexpr int PRE = 32;
        const bool own = tid < nh * HD;
        const int he = own ? tid / HD : 0, de = tid % HD;
        float t0[PRE];
#pragma unroll
        for (int j = 0; j < PRE; j++) t0[j] = (own && j < S) ? pnum(he, j, de) : 0.f;
        // merge factors per head (k_attn_combine's order): f_k = exp(m_k - M), den = the
        // wave sum of each lane's f_k l_k over k = lane, lane + 64
        for (int h = wave; h < nh; h += NWV) {
            const int hh = h0 + h;
            float mk[2], lk[2], mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int k = lane + 64 * j;
                const int po = (int)(((size_t)hh * maxs + k) * (HD + 2) + HD) * 4;
                mk[j] = k < S ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(Pr, po, 0, 16)) : -INFINITY;
                lk[j] = k < S ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(Pr, po + 4, 0, 16)) : 0.f;
                mx = fmaxf(mx, mk[j]);
            }
            mx = wave_max(mx);
            float den = 0.f;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int k = lane + 64 * j;
                if (k < S) {
                    const float f = expf(mk[j] - mx);
                    sCf[h][k] = f;
                    den = fmaf(f, lk[j], den);
                }
            }
            den = wave_sum(den);
            if (lane == 0) sCden[h] = den;
        }
        __syncthreads();
        __shared__ __attribute__((aligned(16))) float sRow[FUSE ? 4 : 1][FUSE ? HD : 1];
        for (int e = tid; e < nh * HD; e += NT) {
            const int h = e / HD, d = e % HD;
            float num = 0.f;
            int k = 0;
            if (e == tid) {
#pragma unroll
                for (int j = 0; j < PRE; j++)
                    if (j < S) num = fmaf(sCf[h][j], t0[j], num);
                k = PRE;
            }
            // past the preloaded ones: 16 partial loads in flight per step, in block order
            for (; k + 16 <= S; k += 16) {
                float t[16];
#pragma unroll
                for (int j = 0; j < 16; j++) t[j] = pnum(h, k + j, d);
#pragma unroll
                for (int j = 0; j < 16; j++) num = fmaf(sCf[h][k + j], t[j], num);
            }
            for (; k < S; k++) num = fmaf(sCf[h][k], pnum(h, k, d), num);
            const float den = sCden[h];
            const float v = den > 0.f ? num * (1.0f / den) : 0.f;
            if (FUSE) sRow[h][d] = v;
            else out[(size_t)(h0 + h) * HD + d] = v;
        }
        if (FUSE) {
            // the attention row of stream zb into the wo input planes, 8 dims per thread
            __syncthreads();
            for (int e = tid; e < nh * HD / 8; e += NT) {
                const int h = e / (HD / 8), d0 = (e % (HD / 8)) * 8;
                uint32_t hp[4], mp[4], lq[4];
#pragma unroll
                for (int i = 0; i < 8; i += 2) {
                    uint16_t a0, b0, c0, a1, b1, c1;
                    split3(sRow[h][d0 + i], a0, b0, c0);
                    split3(sRow[h][d0 + i + 1], a1, b1, c1);
                    hp[i / 2] = a0 | ((uint32_t)a1 << 16);
                    mp[i / 2] = b0 | ((uint32_t)b1 << 16);
                    lq[i / 2] = c0 | ((uint32_t)c1 << 16);
                }
                const int kq = (h0 + h) * HD + d0;
                *reinterpret_cast<uint4*>(F.xs + frag_at(zb, H * HD, 0, kq)) = make_uint4(hp[0], hp[1], hp[2], hp[3]);
                *reinterpret_cast<uint4*>(F.xs + frag_at(zb, H * HD, 1, kq)) = make_uint4(mp[0], mp[1], mp[2], mp[3]);
                *reinterpret_cast<uint4*>(F.xs + frag_at(zb, H * HD, 2, kq)) = make_uint4(lq[0], lq[1], lq[2], lq[3]);
            }
        }
        if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dbg_dump();
        return;
    }
    dbg_dump();
}

// ============================================================================
// Short-context decode attention of one stream (L <= 256 keys, head_dim 128, window >= 256):
// before 256 positions nothing has left the window and the ring has not wrapped, so the keys
// are ring slots 0..lp and a wave's 16 slots (16 * wave ..) are known without the step
// state.  Every K/V and q load goes out at kernel start beside the state read (in
// k_attn_decode they waited for it: ~2 us of the 6.4), each wave runs QK / softmax / PV on
// its own registers (no q staging barrier), and the 16 wave partials meet in LDS behind one
// barrier, the merge factors recomputed by each output thread.  Keys past lp are masked
// (their slots hold older, finite values or zeros).  Grid: one block per query head, the 4
// heads of a kv head on one XCD (blocks y, y + 8, ..: the K/V rows go through one L2).
// ============================================================================
// LATE = w > 0: waves w..15 (keys 16 w..255) read the position first and load only the keys
// inside the context (w = 8: a context of <= 128 keys moves half the K/V bytes through the
// CU); waves 0..w-1 keep the speculative loads
template <int HD, class KT = float, int LATE = 0>
__global__ __launch_bounds__(1024) void k_attn_short(const float* __restrict__ q, const KT* __restrict__ Kc,
                                                     const KT* __restrict__ Vc, const int* __restrict__ state,
                                                     int pos_host, float scale, int H, int KVH,
                                                     float* __restrict__ out) {
    static_assert(HD == 128, "k_attn_short: head_dim 128 layout");
    constexpr int NWV = 16, DQ = HD / 4, DPL = HD / 64;
    __shared__ float sM[NWV], sL[NWV];
    __shared__ __attribute__((aligned(16))) float sO[NWV][HD];
    const int hpk = H / KVH;
    const int kvh = (int)blockIdx.x % KVH, h = kvh * hpk + (int)blockIdx.x / KVH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kvd = KVH * HD, k0 = wave * ATT_CH;
    const int r = lane >> 3, c = lane & 7;
    // K: load i covers keys r + 8 (i & 1), quarter row i >> 1 (8 whole lines per instruction)
    float4 kv[DQ / 4];
    float2 vv[ATT_CH];
    int kpre = ATT_CH;
    if (LATE && wave >= LATE) kpre = min(ATT_CH, (state ? state[0] : pos_host) + 1 - k0);  // wave-uniform
    if (kpre > 0) {
#pragma unroll
        for (int i = 0; i < DQ / 4; i++)
            kv[i] = kv_ld4(Kc + (size_t)(k0 + r + 8 * (i & 1)) * kvd + kvh * HD + (i >> 1) * DQ + c * 4);
#pragma unroll
        for (int k = 0; k < ATT_CH; k++) vv[k] = kv_ld2(Vc + (size_t)(k0 + k) * kvd + kvh * HD + lane * DPL);
    } else {
#pragma unroll
        for (int i = 0; i < DQ / 4; i++) kv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < ATT_CH; k++) vv[k] = make_float2(0.f, 0.f);
    }
    float4 qv[4];
#pragma unroll
    for (int j = 0; j < 4; j++) qv[j] = *reinterpret_cast<const float4*>(q + (size_t)h * HD + j * DQ + c * 4);
    const int lp = state ? state[0] : pos_host;
    const int kn = min(ATT_CH, lp + 1 - k0);  // keys of this wave inside the context (<= 0: none)
    float aa = 0.f, ab = 0.f;
#pragma unroll
    for (int i = 0; i < DQ / 4; i++) {
        const float4 qq = qv[i >> 1];
        float& acc = (i & 1) ? ab : aa;
        acc = fmaf(qq.x, kv[i].x, acc);
        acc = fmaf(qq.y, kv[i].y, acc);
        acc = fmaf(qq.z, kv[i].z, acc);
        acc = fmaf(qq.w, kv[i].w, acc);
    }
    aa += dpp<0xB1>(aa); aa += dpp<0x4E>(aa); aa += dpp<0x141>(aa);
    ab += dpp<0xB1>(ab); ab += dpp<0x4E>(ab); ab += dpp<0x141>(ab);
    const float sa = (r < kn) ? aa * scale : -INFINITY, sbv = (r + 8 < kn) ? ab * scale : -INFINITY;
    float mx = fmaxf(sa, sbv);
    mx = fmaxf(mx, dpp<0x140>(mx));
    mx = rows4_max(mx);  // the 4 rows of 16 lanes: 4 readlanes, no LDS round trip
    const float m = (kn > 0) ? mx : -1e30f;
    const float p = (r < kn) ? expf(sa - mx) : 0.f, pb = (r + 8 < kn) ? expf(sbv - mx) : 0.f;
    float t = p + pb;
    t += dpp<0x140>(t);
    t = rows4_sum(t);
    float o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int k = 0; k < ATT_CH; k++) {
        const float pv = k >= 8 ? pb : p;
        const float pk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv), 8 * (k & 7)));
        const float2 v = k < kn ? vv[k] : make_float2(0.f, 0.f);
        o0 = fmaf(pk, v.x, o0);
        o1 = fmaf(pk, v.y, o1);
    }
    if (lane == 0) {
        sM[wave] = m;
        sL[wave] = t;
    }
    *reinterpret_cast<float2*>(&sO[wave][lane * DPL]) = make_float2(o0, o1);
    __syncthreads();
    if (tid < HD) {
        float M = -1e30f;
#pragma unroll
        for (int w = 0; w < NWV; w++) M = fmaxf(M, sM[w]);
        float den = 0.f, num = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; w++) {
            const float f = expf(sM[w] - M);
            den = fmaf(f, sL[w], den);
            num = fmaf(f, sO[w][tid], num);
        }
        out[(size_t)h * HD + tid] = den > 0.f ? num * (1.0f / den) : 0.f;
    }
}


// ============================================================================
// Step input: x = adapter[gen] + tok_emb[prev] (voxtral.c:1106-1113); the embedding row
// is bf16 (tok_embed_bf16_to_f32, voxtral.c:434-441) or, with esc, int8 times the row's
// scale (tok_embed_q8_to_f32, voxtral.c:443-451).
// ============================================================================
__device__ __forceinline__ float emb_at(const void* emb, const float* esc, int tok, int D, int i) {
    if (esc) return (float)static_cast<const int8_t*>(emb)[(size_t)tok * D + i] * esc[tok];
    return bf2f(static_cast<const uint16_t*>(emb)[(size_t)tok * D + i]);
}

__global__ __launch_bounds__(256) void k_embed_step(const float* __restrict__ adapter,
                                                    const void* __restrict__ emb,
                                                    const float* __restrict__ esc,
                                                    const int* __restrict__ state, int D,
                                                    float* __restrict__ x) {
    const int gi = state[1], tok = state[2];
    const float* a = adapter + (size_t)gi * D;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < D; i += gridDim.x * 256) x[i] = a[i] + emb_at(emb, esc, tok, D, i);
}

// prompt embeds for prefill rows (voxtral.c:1039-1048): token = BOS for logical row 0
__global__ __launch_bounds__(256) void k_embed_rows(const float* __restrict__ adapter,
                                                    const void* __restrict__ emb,
                                                    const float* __restrict__ esc, int row0,
                                                    int first_tok, int rest_tok, int D,
                                                    float* __restrict__ x) {
    const int r = blockIdx.x;
    const int tok = (row0 + r == 0) ? first_tok : rest_tok;
    const float* a = adapter + (size_t)(row0 + r) * D;
    for (int i = threadIdx.x; i < D; i += 256) x[(size_t)r * D + i] = a[i] + emb_at(emb, esc, tok, D, i);
}

// stream_fill_alts candidates (voxtral.c:955-1010) from the LM head's per-block partials:
// the softmax denominator S = sum_b s_b exp(m_b - M) and the 3 largest logits with id >=
// TOKEN_TEXT_MIN other than the chosen token (ties: lower id).  Writes the step's record
// {p_best, id1, p1, id2, p2, id3, p3, 0}, p = exp(l - M) * (1 / S); the host applies n_alt
// and the cutoff.  Called by all 256 threads of k_argmax_final after its barrier.
__device__ __forceinline__ bool alt_before(float va, int ia, float vb, int ib) {
    return va > vb || (va == vb && ia >= 0 && (ib < 0 || ia < ib));
}

// Block-wide (256 threads) merge of per-thread stream_fill_alts partials: the softmax (max,
// sum) pairs and the top-4 lists (alt_before order).  Thread 0 ends with the merged partial.
__device__ void alt_tree(float& m, float& su, float (&tv)[4], int (&ti)[4]) {
    __shared__ float sm[256], ss[256], stv[256][4];
    __shared__ int sti[256][4];
    const int t = threadIdx.x;
    sm[t] = m;
    ss[t] = su;
    for (int k = 0; k < 4; k++) {
        stv[t][k] = tv[k];
        sti[t][k] = ti[k];
    }
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) {
            const float m2 = sm[t + h], s2 = ss[t + h];
            float m1 = sm[t], s1 = ss[t];
            if (m2 > m1) {
                s1 = s1 * expf(m1 - m2) + s2;
                m1 = m2;
            } else if (s2 > 0.f) {
                s1 += s2 * expf(m2 - m1);
            }
            sm[t] = m1;
            ss[t] = s1;
            float ov[4];
            int oi[4];
            int a = 0, b = 0;
            for (int k = 0; k < 4; k++) {
                if (alt_before(stv[t][a], sti[t][a], stv[t + h][b], sti[t + h][b])) {
                    ov[k] = stv[t][a];
                    oi[k] = sti[t][a];
                    a++;
                } else {
                    ov[k] = stv[t + h][b];
                    oi[k] = sti[t + h][b];
                    b++;
                }
            }
            for (int k = 0; k < 4; k++) {
                stv[t][k] = ov[k];
                sti[t][k] = oi[k];
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        m = sm[0];
        su = ss[0];
        for (int k = 0; k < 4; k++) {
            tv[k] = stv[0][k];
            ti[k] = sti[0][k];
        }
    }
}

__device__ void alt_merge(const float* __restrict__ pa, int n, int best, float bestv, int step,
                          float* __restrict__ alts) {
    const int t = threadIdx.x;
    float m = -INFINITY, su = 0.f, tv[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int ti[4] = {-1, -1, -1, -1};
    for (int b = t; b < n; b += 256) {
        const float* p = pa + (size_t)b * ALT_PART;
        const float bm = p[0], bs = p[1];
        if (bm > m) {
            su = su * expf(m - bm) + bs;
            m = bm;
        } else if (bs > 0.f) {
            su += bs * expf(bm - m);
        }
        for (int k = 0; k < 4; k++) {
            const float v = p[2 + k];
            const int id = __float_as_int(p[6 + k]);
            if (id < 0 || id == best || !alt_before(v, id, tv[3], ti[3])) continue;
            int j = 3;
            while (j > 0 && alt_before(v, id, tv[j - 1], ti[j - 1])) {
                tv[j] = tv[j - 1];
                ti[j] = ti[j - 1];
                j--;
            }
            tv[j] = v;
            ti[j] = id;
        }
    }
    alt_tree(m, su, tv, ti);
    if (t == 0) {
        const float inv = 1.0f / su;
        float* r = alts + (size_t)step * ALT_REC;
        r[0] = expf(bestv - m) * inv;
        for (int k = 0; k < 3; k++) {
            const int id = ti[k];
            r[1 + 2 * k] = __int_as_float(id);
            r[2 + 2 * k] = id >= 0 ? expf(tv[k] - m) * inv : 0.f;
        }
        r[7] = 0.f;
    }
}

// Final argmax over per-block partials; advance the device-side step state
// state = {logical kv pos, next adapter row, prev token, step index} and, when adapter is
// given, build the next step's input x = adapter[row] + tok_emb[token] (voxtral.c:
// 1106-1113) so the next replay starts with its first GEMV.
__global__ __launch_bounds__(256) void k_argmax_final(const float* __restrict__ pv,
                                                      const int* __restrict__ pi, int n,
                                                      int* __restrict__ state,
                                                      int* __restrict__ tokens, int tokens_cap,
                                                      const float* __restrict__ adapter,
                                                      int adapter_rows,
                                                      const void* __restrict__ emb,
                                                      const float* __restrict__ esc, int D,
                                                      float* __restrict__ x,
                                                      const float* __restrict__ part_alt,
                                                      float* __restrict__ alts) {
    constexpr int XPT = 16;  // next-input elements per thread (D <= 4096)
    __shared__ float sv[4];
    __shared__ int si[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the step state and this thread's adapter elements of the next input do not depend on
    // the argmax: their loads go out with the partials' (one round trip, not three)
    const int st0 = state[0], st1 = state[1], step = state[3];
    const int srow = st1 + 1;
    const bool mk = adapter && srow < adapter_rows;
    float av[XPT];
    const float* a = adapter + (size_t)(mk ? srow : 0) * D;
#pragma unroll
    for (int j = 0; j < XPT; j++) av[j] = (mk && tid + 256 * j < D) ? a[tid + 256 * j] : 0.f;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < n; i += 256) {
        const float v = pv[i];
        const int id = pi[i];
        if (v > bv || (v == bv && id < bi)) { bv = v; bi = id; }
    }
    // max value, lowest id among ties (voxtral.c argmax: strict >), by shuffles in the wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float v = __shfl_xor(bv, o, 64);
        const int id = __shfl_xor(bi, o, 64);
        if (v > bv || (v == bv && id < bi)) { bv = v; bi = id; }
    }
    if (lane == 0) {
        sv[wave] = bv;
        si[wave] = bi;
    }
    __syncthreads();
    float best = sv[0];
    int besti = si[0];
#pragma unroll
    for (int w = 1; w < 4; w++)
        if (sv[w] > best || (sv[w] == best && si[w] < besti)) { best = sv[w]; besti = si[w]; }
    const int tok = besti == 0x7fffffff ? 0 : besti;
    if (tid == 0) {
        // the token log is a ring of tokens_cap entries (the host drains it every <= 16 steps)
        if (tokens) tokens[step % tokens_cap] = tok;
        state[0] = st0 + 1;
        state[1] = srow;
        state[2] = tok;
        state[3] = step + 1;
    }
    if (mk) {
        // next step's input x = adapter[row] + tok_emb[token] (voxtral.c:1106-1113)
#pragma unroll
        for (int j = 0; j < XPT; j++)
            if (tid + 256 * j < D) x[tid + 256 * j] = av[j] + emb_at(emb, esc, tok, D, tid + 256 * j);
    }
    if (alts) alt_merge(part_alt, n, tok, best, step % tokens_cap, alts);
}

// ============================================================================
// Batched decode step (C4): row i of the batch belongs to stream i.
// ============================================================================
// next inputs of every slot (voxtral.c:1106-1113): x_i = adapter_i[state[1]] +
// tok_emb[state[2]] while the slot is live, 0 otherwise (a stopped row stays finite)
__global__ __launch_bounds__(256) void k_embed_batch(const BatchSlot* __restrict__ slots, const void* __restrict__ emb,
                                                     const float* __restrict__ esc, int D, float* __restrict__ x) {
    const int i = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
    const BatchSlot& sl = slots[i];
    if (j >= D) return;
    float v = 0.f;
    if (sl.live) {
        const int row = sl.state[1], tok = sl.state[2];
        v = sl.adapter[(size_t)row * D + j] + emb_at(emb, esc, tok, D, j);
    }
    x[(size_t)i * D + j] = v;
}

// argmax over row i's logits, first max wins (voxtral_decoder.c:771-779): ARGB slices.  In a
// batched step (slots) stopped rows are skipped, and rows whose slot keeps alternatives also
// leave the slice's stream_fill_alts partial {max, sum, top-4 text values, their ids} in palt.
__global__ __launch_bounds__(256) void k_argmax_rows(const float* __restrict__ logits, int V, float* __restrict__ pval,
                                                     int* __restrict__ pidx, const BatchSlot* __restrict__ slots,
                                                     float* __restrict__ palt) {
    __shared__ float sv[256];
    __shared__ int si[256];
    const int i = blockIdx.y, b = blockIdx.x;
    if (slots && !slots[i].live) return;
    const bool alt = slots && slots[i].alts;
    const int per = (V + ARGB - 1) / ARGB;
    const int lo = b * per, hi = min(V, lo + per);
    const float* lg = logits + (size_t)i * V;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    float am = -INFINITY, as = 0.f, tv[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int ti[4] = {-1, -1, -1, -1};
    for (int j = lo + threadIdx.x; j < hi; j += 256) {
        const float v = lg[j];
        if (v > bv) { bv = v; bi = j; }  // j ascends per thread
        if (alt) alt_row(v, j, am, as, tv, ti);
    }
    sv[threadIdx.x] = bv;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) {
            const float v = sv[threadIdx.x + h];
            const int id = si[threadIdx.x + h];
            if (v > sv[threadIdx.x] || (v == sv[threadIdx.x] && id < si[threadIdx.x])) {
                sv[threadIdx.x] = v;
                si[threadIdx.x] = id;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        pval[i * ARGB + b] = sv[0];
        pidx[i * ARGB + b] = si[0];
    }
    if (alt) {
        alt_tree(am, as, tv, ti);
        if (threadIdx.x == 0) {
            float* pa = palt + ((size_t)i * ARGB + b) * ALT_PART;
            pa[0] = am;
            pa[1] = as;
            for (int k = 0; k < 4; k++) {
                pa[2 + k] = tv[k];
                pa[6 + k] = __int_as_float(ti[k]);
            }
        }
    }
}

// per live slot: final argmax, the stream's token ring and state, the batch's token log, the
// slot's bookkeeping (stop at stop_tok, after `left` steps or past its last adapter row), and
// the next input row x_i = adapter_i[row] + tok_emb[token] (voxtral.c:1106-1113), 0 once the
// slot stopped; then the step's alternatives record when the slot keeps them
__global__ __launch_bounds__(256) void k_argmax_batch_final(const float* __restrict__ pval, const int* __restrict__ pidx,
                                                            const float* __restrict__ palt, BatchSlot* __restrict__ slots,
                                                            int tokens_cap, int* __restrict__ toklog,
                                                            const void* __restrict__ emb, const float* __restrict__ esc,
                                                            int D, float* __restrict__ x) {
    __shared__ int stok, srow, slive, sstep;
    __shared__ float sbest;
    const int i = blockIdx.x;
    BatchSlot* sl = slots + i;
    float* xr = x + (size_t)i * D;
    const int live = sl->live;
    __syncthreads();  // every wave has read the slot before thread 0 advances it
    if (!live) {
        for (int j = threadIdx.x; j < D; j += 256) xr[j] = 0.f;
        return;
    }
    if (threadIdx.x < 64) {
        float bv = pval[i * ARGB + threadIdx.x];
        int bi = pidx[i * ARGB + threadIdx.x];
        for (int off = 32; off > 0; off >>= 1) {
            const float v = __shfl_xor(bv, off, 64);
            const int id = __shfl_xor(bi, off, 64);
            if (v > bv || (v == bv && id < bi)) { bv = v; bi = id; }
        }
        if (threadIdx.x == 0) {
            const int tok = bi == 0x7fffffff ? 0 : bi;
            int* st = sl->state;
            const int step = st[3], row = st[1] + 1, pos = st[0] + 1;
            sl->tokens[step % tokens_cap] = tok;  // ring, as k_argmax_final
            const int k = sl->produced;
            toklog[i * BATCH_TOKLOG + k % BATCH_TOKLOG] = tok;
            st[0] = pos;
            st[1] = row;
            st[2] = tok;
            st[3] = step + 1;
            const int left = sl->left - 1;
            const int live = left > 0 && tok != sl->stop_tok && row < sl->adapter_rows;
            sl->pos = pos;
            sl->produced = k + 1;
            sl->left = left;
            sl->live = live;
            stok = tok;
            srow = row;
            slive = live;
            sstep = step;
            sbest = bv;
        }
    }
    __syncthreads();
    const float* a = sl->adapter + (size_t)srow * D;
    for (int j = threadIdx.x; j < D; j += 256) xr[j] = slive ? a[j] + emb_at(emb, esc, stok, D, j) : 0.f;
    if (sl->alts) alt_merge(palt + (size_t)i * ARGB * ALT_PART, ARGB, stok, sbest, sstep % tokens_cap, sl->alts);
}

// ============================================================================
// Batched decode (M <= 16 rows: the streams of a batched step).  Each f32 row is held as
// three bf16 planes hi/mid/lo (hi + mid + lo = the row exactly) so that MFMA products with
// bf16 / int8 weights are exact.
// ============================================================================

// ============================================================================
// Fragment-major skinny GEMM (batched decode, M <= 16 rows).  The batched path keeps its own
// copy of every decoder matrix and the LM head in MFMA fragment order, so that each 1 KiB a
// wave loads is one A operand: for 16-row group g and 64-k block b,
//   bf16: two 1-KiB halves t = 0, 1; lane l's 16 B = W[16g + (l&15)][64b + 16(l>>4) + 8t .. +7]
//   int8: one 1-KiB block;           lane l's 16 B = W[16g + (l&15)][64b + 16(l>>4) .. +15]
//         (its first 8 bytes feed half 0, the last 8 half 1, converted to bf16 exactly).
// The k order inside a block is permuted the same way for the x planes (B operand), so the
// sum over k is unchanged:
//   plane p, chunk (b, t) of 1 KiB: lane l's 16 B = x_p[row l&15][64b + 16(l>>4) + 8t .. +7].
// Weight and plane loads are then contiguous 1 KiB per wave-instruction (the row-major
// fragment loads touched 16 rows x 64 B each and cost twice the address-unit time).
// ============================================================================

// one thread per 16 B of the packed copy
template <int WQ8>
__global__ __launch_bounds__(256) void k_frag_pack(const uint8_t* __restrict__ src, int K, size_t n16,
                                                   uint8_t* __restrict__ dst) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n16) return;
    const int lane = (int)(i & 63);
    const size_t chunk = i >> 6;
    const int KB = K >> 6;
    const int t = WQ8 ? 0 : (int)(chunk & 1);
    const size_t gb = WQ8 ? chunk : chunk >> 1;
    const size_t g = gb / KB;
    const int b = (int)(gb % KB);
    const size_t row = g * 16 + (lane & 15);
    const int col = b * 64 + (lane >> 4) * 16 + t * 8;
    const size_t esz = WQ8 ? 1 : 2;
    *reinterpret_cast<uint4*>(dst + i * 16) = *reinterpret_cast<const uint4*>(src + (row * K + col) * esz);
}

// residual of a split projection: x[j][n] += sum of its S slabs (k_skl), one element per thread
__global__ __launch_bounds__(256) void k_resid_slabs(float* __restrict__ x, int D, const float* __restrict__ part,
                                                     int S, const float* __restrict__ bias) {
    const int j = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
    if (n < D) x[(size_t)j * D + n] += bias ? psum(part, S, D, j, n) + bias[n] : psum(part, S, D, j, n);
}

// QKV slabs of row blockIdx.x summed in split order (+ bias), RoPE of q and k, K/V append at
// ring slot (pos0 + i) % cap: k_slabs_rows + k_rope_kv in one pass with the same operations
// in the same order (voxtral_encoder.c:570-607).  rope: the row of position pos0.
__global__ __launch_bounds__(256) void k_slabs_rope_kv(const float* __restrict__ part, int S,
                                                       const float* __restrict__ bias, int qd, int kvd, int hd,
                                                       const float* __restrict__ rope, int pos0,
                                                       float* __restrict__ q, float* __restrict__ Kc,
                                                       float* __restrict__ Vc, int cap) {
    // one column pair per thread: q / k pairs (roped), then v pairs; grid (pairs / 256, rows)
    const int i = blockIdx.y, N = qd + 2 * kvd;
    const int p = blockIdx.x * 256 + threadIdx.x, n = 2 * p;
    if (n >= N) return;
    const int slot = (pos0 + i) % cap;
    // bias and rope first: independent of the slabs, in flight with them
    const float2 bb = bias ? *reinterpret_cast<const float2*>(bias + n) : make_float2(0.f, 0.f);
    const float2 cs = n < qd + kvd ? *reinterpret_cast<const float2*>(rope + (size_t)i * hd + 2 * (n % hd / 2))
                                   : make_float2(1.f, 0.f);
    const float2 xx = psum2(part, S, N, i, n);
    float x0 = xx.x, x1 = xx.y;
    if (bias) {
        x0 += bb.x;
        x1 += bb.y;
    }
    if (n >= qd + kvd) {
        float* vr = Vc + (size_t)slot * kvd + (n - qd - kvd);
        vr[0] = x0;
        vr[1] = x1;
        return;
    }
    const float c = cs.x, s = cs.y;  // qd is a multiple of hd: the pair's rope index n % hd / 2
    float* dst = n < qd ? q + (size_t)i * qd + n : Kc + (size_t)slot * kvd + (n - qd);
    dst[0] = x0 * c - x1 * s;
    dst[1] = x0 * s + x1 * c;
}

// out[j][n] = the S slabs of row j + bias[n] (row-major result of a skinny projection)
__global__ __launch_bounds__(256) void k_slabs_rows(const float* __restrict__ part, int S, int N,
                                                    const float* __restrict__ bias, float* __restrict__ out, int ldo) {
    const int j = blockIdx.y, n = blockIdx.x * 256 + threadIdx.x;
    if (n < N) out[(size_t)j * ldo + n] = bias ? psum(part, S, N, j, n) + bias[n] : psum(part, S, N, j, n);
}

// RMSNorm (+ ada) of row blockIdx.y into fragment-major planes, columns chunk blockIdx.x of
// 512 (every block sums the squares of the whole row: 12 KB from L2); a thread owns 8
// consecutive columns: one 16-B piece of each plane
__global__ __launch_bounds__(64) void k_rmsnorm_fplanes(const float* __restrict__ x, int D,
                                                        const float* __restrict__ w,
                                                        const float* __restrict__ ada, float eps,
                                                        uint16_t* __restrict__ xs) {
    const int j = blockIdx.y, tid = threadIdx.x;
    const float* xr = x + (size_t)j * D;
    float ss = 0.f;
    for (int i = tid * 4; i < D; i += 64 * 4) {
        const float4 v = *reinterpret_cast<const float4*>(xr + i);
        ss = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, fmaf(v.w, v.w, ss))));
    }
    ss = wave_sum(ss);
    const float inv = 1.0f / sqrtf(ss / (float)D + eps);
    const size_t P = (size_t)SK_ROWS * D;
    const int c = blockIdx.x * 64 + tid;
    if (c >= D / 8) return;
    const int k = c * 8;
    uint32_t hp[4], mp[4], lp[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
        uint16_t h0, m0, l0, h1, m1, l1;
        float v0 = xr[k + e] * inv * w[k + e], v1 = xr[k + e + 1] * inv * w[k + e + 1];
        if (ada) {
            v0 *= (1.0f + ada[k + e]);
            v1 *= (1.0f + ada[k + e + 1]);
        }
        split3(v0, h0, m0, l0);
        split3(v1, h1, m1, l1);
        hp[e / 2] = h0 | ((uint32_t)h1 << 16);
        mp[e / 2] = m0 | ((uint32_t)m1 << 16);
        lp[e / 2] = l0 | ((uint32_t)l1 << 16);
    }
    const size_t o = frag_off(j, k);
    *reinterpret_cast<uint4*>(xs + o) = make_uint4(hp[0], hp[1], hp[2], hp[3]);
    *reinterpret_cast<uint4*>(xs + P + o) = make_uint4(mp[0], mp[1], mp[2], mp[3]);
    *reinterpret_cast<uint4*>(xs + 2 * P + o) = make_uint4(lp[0], lp[1], lp[2], lp[3]);
}

// Residual + RMSNorm (+ ada) of row blockIdx.x in one pass: x += the S slabs of the previous
// projection (k_skl, summed in split order as k_resid_slabs), the updated row written back,
// its sum of squares reduced in the block, the normalised row stored as fragment-major
// planes.  A thread owns 8 consecutive columns (D <= 8 * 512).
// EPT consecutive elements per thread (4: D <= 2048, 8: D <= 4096); every load of a thread
// (row, slabs in chunks, bias, norm weight, ada) goes out before the first wait
template <int EPT>
__global__ __launch_bounds__(512) void k_resid_rmsnorm_fplanes(float* __restrict__ x, int D,
                                                               const float* __restrict__ part, int S,
                                                               const float* __restrict__ bias,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ ada, float eps,
                                                               uint16_t* __restrict__ xs) {
    constexpr int NV = EPT / 4;               // float4 per thread
    constexpr int CH = EPT == 4 ? 16 : 8;     // slabs per load round
    __shared__ float sred[8];
    const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int k = tid * EPT;
    const bool own = k < D;
    float v[EPT], wv[EPT], av[EPT], bv[EPT];
    float ss = 0.f;
    if (own) {
        float* xr = x + (size_t)j * D + k;
#pragma unroll
        for (int u = 0; u < NV; u++) {
            const float4 a = *reinterpret_cast<const float4*>(xr + 4 * u);
            const float4 ww = *reinterpret_cast<const float4*>(w + k + 4 * u);
            const float4 aa = ada ? *reinterpret_cast<const float4*>(ada + k + 4 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 bb = bias ? *reinterpret_cast<const float4*>(bias + k + 4 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
            v[4 * u] = a.x; v[4 * u + 1] = a.y; v[4 * u + 2] = a.z; v[4 * u + 3] = a.w;
            wv[4 * u] = ww.x; wv[4 * u + 1] = ww.y; wv[4 * u + 2] = ww.z; wv[4 * u + 3] = ww.w;
            av[4 * u] = aa.x; av[4 * u + 1] = aa.y; av[4 * u + 2] = aa.z; av[4 * u + 3] = aa.w;
            bv[4 * u] = bb.x; bv[4 * u + 1] = bb.y; bv[4 * u + 2] = bb.z; bv[4 * u + 3] = bb.w;
        }
        if (S > 0) {
            float r[EPT];
            const float* pb = part + (size_t)(j >> 4) * S * SK_ROWS * D + (size_t)(j & 15) * D + k;
            for (int s0 = 0; s0 < S; s0 += CH) {
                float4 t[CH][NV];
#pragma unroll
                for (int c = 0; c < CH; c++)
#pragma unroll
                    for (int u = 0; u < NV; u++)
                        t[c][u] = s0 + c < S ? *reinterpret_cast<const float4*>(pb + (size_t)(s0 + c) * SK_ROWS * D + 4 * u)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int c = 0; c < CH; c++)
                    if (s0 + c < S)
#pragma unroll
                        for (int u = 0; u < NV; u++) {
                            const float tt[4] = {t[c][u].x, t[c][u].y, t[c][u].z, t[c][u].w};
#pragma unroll
                            for (int e = 0; e < 4; e++) r[4 * u + e] = (s0 + c) ? r[4 * u + e] + tt[e] : tt[e];
                        }
            }
            if (bias) {
#pragma unroll
                for (int e = 0; e < EPT; e++) r[e] += bv[e];
            }
#pragma unroll
            for (int e = 0; e < EPT; e++) v[e] += r[e];
#pragma unroll
            for (int u = 0; u < NV; u++)
                *reinterpret_cast<float4*>(xr + 4 * u) = make_float4(v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
        }
#pragma unroll
        for (int e = 0; e < EPT; e++) ss = fmaf(v[e], v[e], ss);
    }
    ss = wave_sum(ss);
    if (lane == 0) sred[wave] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) tot += sred[i];
    if (!own) return;
    const float inv = 1.0f / sqrtf(tot / (float)D + eps);
    uint32_t hp[EPT / 2], mp[EPT / 2], lq[EPT / 2];
#pragma unroll
    for (int e = 0; e < EPT; e += 2) {
        float v0 = v[e] * inv * wv[e], v1 = v[e + 1] * inv * wv[e + 1];
        if (ada) {
            v0 *= (1.0f + av[e]);
            v1 *= (1.0f + av[e + 1]);
        }
        uint16_t h0, m0, l0, h1, m1, l1;
        split3(v0, h0, m0, l0);
        split3(v1, h1, m1, l1);
        hp[e / 2] = h0 | ((uint32_t)h1 << 16);
        mp[e / 2] = m0 | ((uint32_t)m1 << 16);
        lq[e / 2] = l0 | ((uint32_t)l1 << 16);
    }
    if (EPT == 8) {
        *reinterpret_cast<uint4*>(xs + frag_at(j, D, 0, k)) = make_uint4(hp[0], hp[1], hp[2 % (EPT / 2)], hp[3 % (EPT / 2)]);
        *reinterpret_cast<uint4*>(xs + frag_at(j, D, 1, k)) = make_uint4(mp[0], mp[1], mp[2 % (EPT / 2)], mp[3 % (EPT / 2)]);
        *reinterpret_cast<uint4*>(xs + frag_at(j, D, 2, k)) = make_uint4(lq[0], lq[1], lq[2 % (EPT / 2)], lq[3 % (EPT / 2)]);
    } else {
        // 4 consecutive elements share one 8-B run of the fragment layout (frag_off)
        *reinterpret_cast<uint2*>(xs + frag_at(j, D, 0, k)) = make_uint2(hp[0], hp[1]);
        *reinterpret_cast<uint2*>(xs + frag_at(j, D, 1, k)) = make_uint2(mp[0], mp[1]);
        *reinterpret_cast<uint2*>(xs + frag_at(j, D, 2, k)) = make_uint2(lq[0], lq[1]);
    }
}

// rows of x (f32) into fragment-major planes
__global__ __launch_bounds__(256) void k_split_fplanes(const float* __restrict__ x, int K, uint16_t* __restrict__ xs) {
    const int j = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= K / 8) return;
    const int k = c * 8;
    const float* xr = x + (size_t)j * K + k;
    const float4 a = *reinterpret_cast<const float4*>(xr), b = *reinterpret_cast<const float4*>(xr + 4);
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t hp[4], mp[4], lp[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
        uint16_t h0, m0, l0, h1, m1, l1;
        split3(v[e], h0, m0, l0);
        split3(v[e + 1], h1, m1, l1);
        hp[e / 2] = h0 | ((uint32_t)h1 << 16);
        mp[e / 2] = m0 | ((uint32_t)m1 << 16);
        lp[e / 2] = l0 | ((uint32_t)l1 << 16);
    }
    *reinterpret_cast<uint4*>(xs + frag_at(j, K, 0, k)) = make_uint4(hp[0], hp[1], hp[2], hp[3]);
    *reinterpret_cast<uint4*>(xs + frag_at(j, K, 1, k)) = make_uint4(mp[0], mp[1], mp[2], mp[3]);
    *reinterpret_cast<uint4*>(xs + frag_at(j, K, 2, k)) = make_uint4(lp[0], lp[1], lp[2], lp[3]);
}

__device__ __forceinline__ bf16x8 i8x8_bf16(uint32_t lo, uint32_t hi) {
    uint32_t h[8];
#pragma unroll
    for (int b = 0; b < 4; b++) {
        h[b] = __float_as_uint(i8f(lo, b)) >> 16;
        h[4 + b] = __float_as_uint(i8f(hi, b)) >> 16;
    }
    return __builtin_bit_cast(bf16x8, make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16)));
}

// one 64-k block of R row groups (A halves) and of the three planes (B halves) of Z 16-row
// blocks of streams
template <int WQ8, int R, int Z = 1>
struct SkfRegs {
    u32x4 a[R][WQ8 ? 1 : 2];
    uint4 x[Z][3][2];
};

// block b of the wave's range; past the range the loads go through zero-length descriptors
// (they return 0 and move no bytes, so the ring below needs no branches)
template <int WQ8, int R, int Z>
__device__ __forceinline__ void skf_load(SkfRegs<WQ8, R, Z>& s, __amdgpu_buffer_rsrc_t W, __amdgpu_buffer_rsrc_t X,
                                         int kbytes, int b, int pbytes) {
    constexpr int FB = WQ8 ? 1024 : 2048;
    const int lo = (threadIdx.x & 63) * 16;
#pragma unroll
    for (int z = 0; z < Z; z++)
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(X, lo + t * 1024, (z * 3 + p) * pbytes + b * 2048, 0);
                s.x[z][p][t] = make_uint4(v.x, v.y, v.z, v.w);
            }
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int t = 0; t < (WQ8 ? 1 : 2); t++)
            s.a[r][t] = __builtin_amdgcn_raw_buffer_load_b128(W, lo + t * 1024, r * kbytes + b * FB, 2);
}

template <int WQ8, int R, int Z>
__device__ __forceinline__ void skf_mma(const SkfRegs<WQ8, R, Z>& s, f32x4 (&acc)[Z][R]) {
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
        for (int r = 0; r < R; r++) {
            bf16x8 af;
            if (WQ8) {
                const u32x4 q = s.a[r][0];
                af = t ? i8x8_bf16(q.z, q.w) : i8x8_bf16(q.x, q.y);
            } else {
                const u32x4 q = s.a[r][t];
                af = __builtin_bit_cast(bf16x8, make_uint4(q.x, q.y, q.z, q.w));
            }
#pragma unroll
            for (int z = 0; z < Z; z++)
#pragma unroll
                for (int p = 0; p < 3; p++)
                    acc[z][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8, s.x[z][p][t]), acc[z][r], 0, 0, 0);
        }
}

// Block = R row groups (16R rows) x all of K, K split over NW waves in 64-k blocks; the
// wave partials meet in LDS and the block stores its 16R x 16Z outputs C[j][row] (the LM head:
// its planes fit no LDS, and at 8192 row groups the per-block plane re-reads are amortised
// over R = 4 groups).  Z = 2: both 16-row blocks of a 32-stream step against each weight
// fragment the wave loads, so the 805 MB of embeddings cross the load path once per step
// instead of once per row block (the planes of a row block z follow block z - 1's three).
template <int WQ8, int R, int NW, int D, int Z = 1>
__global__ __launch_bounds__(NW * 64) void k_skf(const uint16_t* __restrict__ xs, int K,
                                                 const uint8_t* __restrict__ W, const float* __restrict__ wscale,
                                                 int N, int nb, float* __restrict__ C, int ldc) {
    __shared__ float red[NW][Z * R][4][64];
    constexpr int FB = WQ8 ? 1024 : 2048;
    // wave index through readfirstlane: a provably uniform block range keeps the buffer
    // loads' soffset in an SGPR (else every load becomes a waterfall loop)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int KB = K >> 6;
    const int b0 = KB * wave / NW, b1 = KB * (wave + 1) / NW;
    const int g0 = blockIdx.x * R;
    const int kbytes = KB * FB;  // bytes of one row group
    const __amdgpu_buffer_rsrc_t Wd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(W) + (size_t)g0 * kbytes, 0, R * kbytes, 0x00020000);
    const int pbytes = SK_ROWS * K * 2;  // one plane
    const __amdgpu_buffer_rsrc_t Xd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(xs), 0, Z * 3 * pbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t Wz = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(W), 0, 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t Xz = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(xs), 0, 0, 0x00020000);
    f32x4 acc[Z][R];
#pragma unroll
    for (int z = 0; z < Z; z++)
#pragma unroll
        for (int r = 0; r < R; r++) acc[z][r] = f32x4{0.f, 0.f, 0.f, 0.f};
    // register ring of D blocks: block b + D - 1 is requested before block b's MFMAs, so a
    // wave keeps D - 1 blocks of weights and planes in flight
    SkfRegs<WQ8, R, Z> s[D];
#define SKF_LOAD(slot, blk)                                                                  \
    do {                                                                                     \
        const int bb__ = (blk);                                                              \
        const bool in__ = bb__ < b1;                                                         \
        skf_load<WQ8, R, Z>(s[slot], in__ ? Wd : Wz, in__ ? Xd : Xz, kbytes, in__ ? bb__ : 0, pbytes); \
    } while (0)
#pragma unroll
    for (int i = 0; i < D - 1; i++) SKF_LOAD(i, b0 + i);
    for (int b = b0; b < b1; b += D) {
#pragma unroll
        for (int i = 0; i < D; i++) {
            SKF_LOAD((i + D - 1) % D, b + i + D - 1);
            __builtin_amdgcn_sched_barrier(0);
            skf_mma<WQ8, R, Z>(s[i], acc);  // zeros past the range: acc + 0
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#undef SKF_LOAD
#pragma unroll
    for (int z = 0; z < Z; z++)
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int i = 0; i < 4; i++) red[wave][z * R + r][i][lane] = acc[z][r][i];
    __syncthreads();
    // output o: row block z = o / (256 R), group r = (o >> 8) % R, row rr = (o >> 4) & 15,
    // stream j = o & 15 of the row block; D layout: col = lane&15, row = (lane>>4)*4 + i
    for (int o = tid; o < Z * R * 256; o += NW * 64) {
        const int zr = o >> 8, z = zr / R, r = zr % R, rr = (o >> 4) & 15, j = o & 15;
        if (z * 16 + j >= nb) continue;
        const int ln = ((rr >> 2) << 4) + j, i = rr & 3;
        const int row = (g0 + r) * 16 + rr;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < NW; w++) v += red[w][zr][i][ln];
        C[(size_t)(z * 16 + j) * ldc + row] = WQ8 ? v * wscale[row] : v;
    }
}

// ============================================================================
// LDS-planes skinny GEMM (batched decode projections): block (chunk c, k-split s) stages the
// planes of its KS 64-k blocks in LDS once (KS x 6 KiB, shared by its waves), each wave
// streams one 16-row group's KS weight blocks -- all issued before the first wait -- and
// writes its 16 x 16 partial sums to part[s][16][N] (scaled for Q8).  The consumer sums the
// splits in order (k_rope_kv_batch, k_rmsnorm_fplanes, k_swiglu_fplanes), so no reduction
// kernel runs and the result does not depend on timing.  Re-reading the planes from L2 per
// 16-row group (k_skf at R = 1) moved 3x the weight bytes through the load path.
// ============================================================================
// ssq != null: the planes hold x * w (* (1 + ada)) of an RMSNorm (k_resid_xw_fplanes) and
// every result of stream row j is multiplied by 1 / sqrt(sum_t ssq[z][t][j] / K + eps), the
// row's sum of squares from its nsl column slices added in slice order.
template <int WQ8, int NW, int KS, int SC = 0>
__global__ __launch_bounds__(NW * 64) void k_skl(const uint16_t* __restrict__ xs, int K,
                                                 const uint8_t* __restrict__ W, const float* __restrict__ wscale,
                                                 int N, int nb, float* __restrict__ part,
                                                 const float* __restrict__ ssq = nullptr, int nsl = 0, float eps = 0.f) {
    __shared__ uint4 xb[KS * 6 * 64];  // [block][plane][half][lane]
    __shared__ float s_sq[SC ? SK_ROWS * SKL_MAX_SLICES : 1];
    constexpr int FB = WQ8 ? 1024 : 2048, NH = WQ8 ? 1 : 2;
    constexpr int NF = KS * 6 / NW;  // 16-B plane pieces per thread
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int KB = K >> 6, S = KB / KS, X = N / (16 * NW);
    // 1-D grid.  Z > 1 row blocks (more than 16 rows): the Z blocks that stream the same weight
    // slice u = 8q + r for row blocks z = 0..Z-1 are ids (qZ + z) * 8 + r, i.e. the same XCD
    // under round-robin placement and dispatched together, so the repeat reads of each weight
    // byte hit that XCD's L2 instead of HBM (placement is a speed matter only, never correctness)
    int u = blockIdx.x, z = 0;
    const int Z = (nb + SK_ROWS - 1) / SK_ROWS;
    if (Z > 1) {
        const int t = u >> 3;
        z = t % Z;
        u = (t / Z) * 8 + (u & 7);
        if (u >= X * S) return;
    }
    const int s = u / X, kb0 = s * KS;
    const int g = (u % X) * NW + wave;
    const size_t P = (size_t)SK_ROWS * K;
    // row block z: its planes and slabs ([rb][3][16][K], [rb][S][16][N])
    xs += (size_t)z * 3 * P;
    part += (size_t)z * S * SK_ROWS * N;
    nb -= z * SK_ROWS;
    // planes first: vmcnt retires in issue order, so the weights issued after them stay in
    // flight while the plane pieces are written to LDS
    uint4 f[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        const int idx = tid + i * NW * 64;
        const int blk = idx / 384, rem = idx % 384;
        const int p = rem >> 7, t = (rem >> 6) & 1, l = rem & 63;
        f[i] = *reinterpret_cast<const uint4*>(xs + p * P + (size_t)((kb0 + blk) * 2 + t) * 512 + l * 8);
    }
    // SC: the slice sums of squares ssq[z][t][j] travel with the planes (one value per
    // thread into LDS), the epilogue adds them up per row
    float sqv = 0.f;
    if (SC) sqv = ssq[(size_t)z * nsl * SK_ROWS + min(tid, nsl * SK_ROWS - 1)];
    const __amdgpu_buffer_rsrc_t Wd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(W) + (size_t)g * KB * FB, 0, KB * FB, 0x00020000);
    u32x4 a[KS][NH];
#pragma unroll
    for (int kb = 0; kb < KS; kb++)
#pragma unroll
        for (int t = 0; t < NH; t++) a[kb][t] = __builtin_amdgcn_raw_buffer_load_b128(Wd, lane * 16 + t * 1024, (kb0 + kb) * FB, 2);
#pragma unroll
    for (int i = 0; i < NF; i++) xb[tid + i * NW * 64] = f[i];
    if (SC && tid < nsl * SK_ROWS) s_sq[tid] = sqv;
    __syncthreads();
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KS; kb++)
#pragma unroll
        for (int t = 0; t < 2; t++) {
            bf16x8 af;
            if (WQ8) {
                const u32x4 q = a[kb][0];
                af = t ? i8x8_bf16(q.z, q.w) : i8x8_bf16(q.x, q.y);
            } else {
                const u32x4 q = a[kb][t];
                af = __builtin_bit_cast(bf16x8, make_uint4(q.x, q.y, q.z, q.w));
            }
#pragma unroll
            for (int p = 0; p < 3; p++)
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8, xb[((kb * 3 + p) * 2 + t) * 64 + lane]),
                                                             acc, 0, 0, 0);
        }
    const int j = lane & 15;
    if (SC) {
        // all reads out together (one LDS latency), then added in slice order
        float sv[SKL_MAX_SLICES];
#pragma unroll
        for (int t = 0; t < SKL_MAX_SLICES; t++) sv[t] = s_sq[min(t, nsl - 1) * SK_ROWS + j];
        float ss = 0.f;
#pragma unroll
        for (int t = 0; t < SKL_MAX_SLICES; t++)
            if (t < nsl) ss += sv[t];
        const float inv = 1.0f / sqrtf(ss / (float)K + eps);
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] *= inv;
    }
    if (j < nb) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int row = g * 16 + (lane >> 4) * 4 + i;
            part[((size_t)s * SK_ROWS + j) * N + row] = WQ8 ? acc[i] * wscale[row] : acc[i];
        }
    }
}

// k_skl for 17..32 rows (two row blocks of 16) in one block: the planes of both row blocks'
// K-slice sit in LDS (2 x KS x 6 KiB) and each weight fragment a wave loads feeds the MFMAs of
// both, so a weight byte crosses the CU's load path once per step instead of once per row
// block (k_skl's Z > 1 grid streams each slice twice, the second time from L2).  Same splits,
// per-output summation order and slab layout [rb][s][16][N] as k_skl: the same bits.
template <int WQ8, int NW, int KS, int SC = 0>
__global__ __launch_bounds__(NW * 64) void k_skl2(const uint16_t* __restrict__ xs, int K,
                                                  const uint8_t* __restrict__ W, const float* __restrict__ wscale,
                                                  int N, int nb, float* __restrict__ part,
                                                  const float* __restrict__ ssq = nullptr, int nsl = 0, float eps = 0.f) {
    __shared__ uint4 xb[2][KS * 6 * 64];  // [row block][block][plane][half][lane]
    __shared__ float s_sq[SC ? 2 * SK_ROWS * SKL_MAX_SLICES : 1];
    constexpr int FB = WQ8 ? 1024 : 2048, NH = WQ8 ? 1 : 2;
    constexpr int NF = KS * 6 / NW;  // 16-B plane pieces per thread and row block
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int KB = K >> 6, S = KB / KS, X = N / (16 * NW);
    const int u = blockIdx.x;
    const int s = u / X, kb0 = s * KS;
    const int g = (u % X) * NW + wave;
    const size_t P = (size_t)SK_ROWS * K;
    uint4 f[2][NF];
#pragma unroll
    for (int z = 0; z < 2; z++)
#pragma unroll
        for (int i = 0; i < NF; i++) {
            const int idx = tid + i * NW * 64;
            const int blk = idx / 384, rem = idx % 384;
            const int p = rem >> 7, t = (rem >> 6) & 1, l = rem & 63;
            f[z][i] = *reinterpret_cast<const uint4*>(xs + (size_t)z * 3 * P + p * P + (size_t)((kb0 + blk) * 2 + t) * 512 + l * 8);
        }
    constexpr int NSQ = SC ? (2 * SK_ROWS * SKL_MAX_SLICES + NW * 64 - 1) / (NW * 64) : 1;
    float sqv[NSQ];
    if (SC) {
#pragma unroll
        for (int i = 0; i < NSQ; i++) {
            const int e = tid + i * NW * 64;  // (z, t, j) = ssq[z][t][j], z = e / (nsl * 16)
            sqv[i] = e < 2 * nsl * SK_ROWS ? ssq[e] : 0.f;
        }
    }
    const __amdgpu_buffer_rsrc_t Wd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(W) + (size_t)g * KB * FB, 0, KB * FB, 0x00020000);
    u32x4 a[KS][NH];
#pragma unroll
    for (int kb = 0; kb < KS; kb++)
#pragma unroll
        for (int t = 0; t < NH; t++) a[kb][t] = __builtin_amdgcn_raw_buffer_load_b128(Wd, lane * 16 + t * 1024, (kb0 + kb) * FB, 2);
#pragma unroll
    for (int z = 0; z < 2; z++)
#pragma unroll
        for (int i = 0; i < NF; i++) xb[z][tid + i * NW * 64] = f[z][i];
    if (SC) {
#pragma unroll
        for (int i = 0; i < NSQ; i++)
            if (tid + i * NW * 64 < 2 * nsl * SK_ROWS) s_sq[tid + i * NW * 64] = sqv[i];
    }
    __syncthreads();
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kb = 0; kb < KS; kb++)
#pragma unroll
        for (int t = 0; t < 2; t++) {
            bf16x8 af;
            if (WQ8) {
                const u32x4 q = a[kb][0];
                af = t ? i8x8_bf16(q.z, q.w) : i8x8_bf16(q.x, q.y);
            } else {
                const u32x4 q = a[kb][t];
                af = __builtin_bit_cast(bf16x8, make_uint4(q.x, q.y, q.z, q.w));
            }
#pragma unroll
            for (int z = 0; z < 2; z++)
#pragma unroll
                for (int p = 0; p < 3; p++)
                    acc[z] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        af, __builtin_bit_cast(bf16x8, xb[z][((kb * 3 + p) * 2 + t) * 64 + lane]), acc[z], 0, 0, 0);
        }
    const int j = lane & 15;
#pragma unroll
    for (int z = 0; z < 2; z++) {
        if (SC) {
            float sv[SKL_MAX_SLICES];
#pragma unroll
            for (int t = 0; t < SKL_MAX_SLICES; t++) sv[t] = s_sq[(z * nsl + min(t, nsl - 1)) * SK_ROWS + j];
            float ss = 0.f;
#pragma unroll
            for (int t = 0; t < SKL_MAX_SLICES; t++)
                if (t < nsl) ss += sv[t];
            const float inv = 1.0f / sqrtf(ss / (float)K + eps);
#pragma unroll
            for (int i = 0; i < 4; i++) acc[z][i] *= inv;
        }
        if (z * SK_ROWS + j < nb) {
            float* pz = part + (size_t)z * S * SK_ROWS * N;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int row = g * 16 + (lane >> 4) * 4 + i;
                pz[((size_t)s * SK_ROWS + j) * N + row] = WQ8 ? acc[z][i] * wscale[row] : acc[z][i];
            }
        }
    }
}

// Residual + the planes of an RMSNorm without its row reduction: x += the S slabs of the
// previous projection (+ bias, summed in split order as k_resid_rmsnorm_fplanes), the row
// written back, the planes of x * w (* (1 + ada)) -- the inverse RMS is applied by the next
// projection (k_skl ssq) -- and the sum of squares of this block's column slice to
// ssq[row block][slice][row % 16].  One wave per (256-column slice, row): a row's slab bytes spread over
// D / 256 CUs instead of one (the batched step's rows are latency-bound at 16 blocks).
__global__ __launch_bounds__(64) void k_resid_xw_fplanes(float* __restrict__ x, int D,
                                                         const float* __restrict__ part, int S,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ ada,
                                                         uint16_t* __restrict__ xs, float* __restrict__ ssq) {
    // slabs per load round: 24 covers the batched step's wo (8 splits) and W2 (18) in one
    // round of loads instead of 1 and 3 dependent ones
    constexpr int CH = 24;
    const int sl = blockIdx.x, j = blockIdx.y, lane = threadIdx.x;
    const int k = sl * 256 + lane * 4;
    float* xr = x + (size_t)j * D + k;
    float4 v = *reinterpret_cast<const float4*>(xr);
    const float4 ww = *reinterpret_cast<const float4*>(w + k);
    const float4 aa = ada ? *reinterpret_cast<const float4*>(ada + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 bb = bias ? *reinterpret_cast<const float4*>(bias + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (S > 0) {
        const float* pb = part + (size_t)(j >> 4) * S * SK_ROWS * D + (size_t)(j & 15) * D + k;
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s0 = 0; s0 < S; s0 += CH) {
            float4 t[CH];
#pragma unroll
            for (int c = 0; c < CH; c++)
                t[c] = s0 + c < S ? *reinterpret_cast<const float4*>(pb + (size_t)(s0 + c) * SK_ROWS * D)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int c = 0; c < CH; c++)
                if (s0 + c < S) {
                    if (s0 + c) {
                        r.x += t[c].x; r.y += t[c].y; r.z += t[c].z; r.w += t[c].w;
                    } else {
                        r = t[c];
                    }
                }
        }
        if (bias) {
            r.x += bb.x; r.y += bb.y; r.z += bb.z; r.w += bb.w;
        }
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        *reinterpret_cast<float4*>(xr) = v;
    }
    float ss = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, v.w * v.w)));
    ss = wave_sum(ss);
    if (lane == 0) ssq[((size_t)(j >> 4) * gridDim.x + sl) * SK_ROWS + (j & 15)] = ss;
    const float e[4] = {v.x * ww.x, v.y * ww.y, v.z * ww.z, v.w * ww.w};
    const float ad[4] = {aa.x, aa.y, aa.z, aa.w};
    uint32_t hp[2], mp[2], lq[2];
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
        float v0 = e[i], v1 = e[i + 1];
        if (ada) {
            v0 *= (1.0f + ad[i]);
            v1 *= (1.0f + ad[i + 1]);
        }
        uint16_t h0, m0, l0, h1, m1, l1;
        split3(v0, h0, m0, l0);
        split3(v1, h1, m1, l1);
        hp[i / 2] = h0 | ((uint32_t)h1 << 16);
        mp[i / 2] = m0 | ((uint32_t)m1 << 16);
        lq[i / 2] = l0 | ((uint32_t)l1 << 16);
    }
    *reinterpret_cast<uint2*>(xs + frag_at(j, D, 0, k)) = make_uint2(hp[0], hp[1]);
    *reinterpret_cast<uint2*>(xs + frag_at(j, D, 1, k)) = make_uint2(mp[0], mp[1]);
    *reinterpret_cast<uint2*>(xs + frag_at(j, D, 2, k)) = make_uint2(lq[0], lq[1]);
}

// silu(W1 x) * (W3 x) of the split W1|W3 result (16-row interleave, upload_w13) into the
// fragment-major planes of the w2 input; a thread owns 2 consecutive hidden units
__global__ __launch_bounds__(256) void k_swiglu_fplanes(const float* __restrict__ part, int S, int H,
                                                        uint16_t* __restrict__ xs) {
    const int j = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= H / 2) return;
    const int h0 = c * 2, N = 2 * H;
    const int rg = (h0 >> 4) * 32 + (h0 & 15);  // W1 row of unit h0; its W3 row is rg + 16
    uint16_t hh[2], mm[2], ll[2];
    const float2 g2 = psum2(part, S, N, j, rg), u2 = psum2(part, S, N, j, rg + 16);
    split3(silu(g2.x) * u2.x, hh[0], mm[0], ll[0]);
    split3(silu(g2.y) * u2.y, hh[1], mm[1], ll[1]);
    // h0 even: one 4-B piece per plane
    *reinterpret_cast<uint32_t*>(xs + frag_at(j, H, 0, h0)) = hh[0] | ((uint32_t)hh[1] << 16);
    *reinterpret_cast<uint32_t*>(xs + frag_at(j, H, 1, h0)) = mm[0] | ((uint32_t)mm[1] << 16);
    *reinterpret_cast<uint32_t*>(xs + frag_at(j, H, 2, h0)) = ll[0] | ((uint32_t)ll[1] << 16);
}

// ============================================================================
// k_sklx: k_skl (above) with its neighbouring row kernels folded in, for the streaming
// encoder's ~25-row chunks where those kernels (5 us each, latency only) cost as much as the
// projections.  Same grid, planes and MFMA loop as k_skl (bf16 weights); see SklFused.
// ============================================================================
template <int NW, int KS, int PRO, int EPI>
__global__ __launch_bounds__(NW * 64) void k_sklx(const uint16_t* __restrict__ xs, int K,
                                                  const uint8_t* __restrict__ W, int N, int nb, const SklFused f) {
    __shared__ uint4 xb[KS * 6 * 64];  // [block][plane][half][lane]
    __shared__ float s_ss[PRO == SKX_PRO_SCALE ? 2 * NW * 64 : 1];
    __shared__ int s_fin;
    constexpr int FB = 2048;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int KB = K >> 6, S = KB / KS, X = N / (16 * NW);
    // 1-D grid, row blocks of one weight slice on one XCD (k_skl)
    int u = blockIdx.x, z = 0;
    const int Z = (nb + SK_ROWS - 1) / SK_ROWS;
    if (Z > 1) {
        const int t = u >> 3;
        z = t % Z;
        u = (t / Z) * 8 + (u & 7);
        if (u >= X * S) return;
    }
    const int s = u / X, xi = u % X, kb0 = s * KS;
    const int g = xi * NW + wave;
    const int nbz = min(nb - z * SK_ROWS, SK_ROWS);  // rows of this row block
    const __amdgpu_buffer_rsrc_t Wd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(W) + (size_t)g * KB * FB, 0, KB * FB, 0x00020000);
    u32x4 a[KS][2];
    constexpr int NF = KS * 6 / NW;
    const size_t P = (size_t)SK_ROWS * K;
    const uint16_t* xz = xs + (size_t)z * 3 * P;
    uint4 fp[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        const int idx = tid + i * NW * 64;
        const int blk = idx / 384, rem = idx % 384;
        const int p = rem >> 7, t = (rem >> 6) & 1, l = rem & 63;
        fp[i] = *reinterpret_cast<const uint4*>(xz + p * P + (size_t)((kb0 + blk) * 2 + t) * 512 + l * 8);
    }
    // SKX_PRO_SCALE: the producer's per-slice row sums of squares, all in flight at once
    const int nss = PRO == SKX_PRO_SCALE ? f.nsl * SK_ROWS : 0;
    const float* sp = f.ssq_in + (size_t)z * nss;
    float ss0 = 0.f, ss1 = 0.f;
    if (PRO == SKX_PRO_SCALE) {
        if (tid < nss) ss0 = sp[tid];
        if (tid + NW * 64 < nss) ss1 = sp[tid + NW * 64];
    }
#pragma unroll
    for (int kb = 0; kb < KS; kb++)
#pragma unroll
        for (int t = 0; t < 2; t++)
            a[kb][t] = __builtin_amdgcn_raw_buffer_load_b128(Wd, lane * 16 + t * 1024, (kb0 + kb) * FB, 2);
#pragma unroll
    for (int i = 0; i < NF; i++) xb[tid + i * NW * 64] = fp[i];
    if (PRO == SKX_PRO_SCALE) {
        if (tid < nss) s_ss[tid] = ss0;
        if (tid + NW * 64 < nss) s_ss[tid + NW * 64] = ss1;
    }
    __syncthreads();
    // the inverse RMS of this lane's row j = lane & 15 (slices summed in order, every thread alike)
    float inv = 1.f;
    if (PRO == SKX_PRO_SCALE) {
        float ss = 0.f;
        for (int q = 0; q < f.nsl; q++) ss += s_ss[q * SK_ROWS + (lane & 15)];
        inv = 1.0f / sqrtf(ss / (float)K + f.eps);
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KS; kb++)
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const u32x4 q = a[kb][t];
            const bf16x8 af = __builtin_bit_cast(bf16x8, make_uint4(q.x, q.y, q.z, q.w));
#pragma unroll
            for (int p = 0; p < 3; p++)
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8, xb[((kb * 3 + p) * 2 + t) * 64 + lane]),
                                                             acc, 0, 0, 0);
        }
    if (PRO == SKX_PRO_SCALE) {
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] *= inv;
    }
    // slab [z][s][16][N] out write-through (sc1), then the slice's ticket
    const size_t zbase = (size_t)z * S * SK_ROWS * N;
    const __amdgpu_buffer_rsrc_t Pd = __builtin_amdgcn_make_buffer_rsrc(f.part + zbase, 0, S * SK_ROWS * N * 4, 0x00020000);
    {
        const int j = lane & 15;
        if (j < nbz)
            __builtin_amdgcn_raw_buffer_store_b128(
                u32x4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])}, Pd,
                (((s * SK_ROWS + j) * N) + g * 16 + (lane >> 4) * 4) * 4, 0, 16);
    }
    // Publication order (MI355X_MICROARCH.md "handoff-flag": sc1 payload -> vmcnt(0) -> flag):
    // the slab stores above are write-through (sc1), so once vmcnt(0) retires them they sit
    // past every XCD's L2; the finisher reads them with sc1 loads, which miss its own L2.  No
    // dirty line is involved on either side, so no agent-scope release / acquire fence (an L2
    // write-back / invalidate per block) is needed; the ticket itself is a relaxed agent-scope
    // add, issued by one lane after the whole block has drained.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* tk = f.ticket + z * X + xi;
    if (tid == 0) s_fin = S == 1 || __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
    __syncthreads();
    if (!s_fin) return;
    if (tid == 0 && S > 1) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- this block completes slice xi: columns [c0, c0 + 16 NW) of rows z * 16 + j ----
    const int c0 = xi * NW * 16;
    auto slab2 = [&](int j, int n) -> float2 {  // psum2 over write-through slabs (sc1 loads)
        float2 v = make_float2(0.f, 0.f);
        for (int s0 = 0; s0 < S; s0 += 8) {
            u32x2 t[8];
#pragma unroll
            for (int c = 0; c < 8; c++)
                if (s0 + c < S)
                    t[c] = __builtin_amdgcn_raw_buffer_load_b64(Pd, (((s0 + c) * SK_ROWS + j) * N + n) * 4, 0, 16);
#pragma unroll
            for (int c = 0; c < 8; c++)
                if (s0 + c < S) {
                    v.x = (s0 + c) ? v.x + __uint_as_float(t[c].x) : __uint_as_float(t[c].x);
                    v.y = (s0 + c) ? v.y + __uint_as_float(t[c].y) : __uint_as_float(t[c].y);
                }
        }
        return v;
    };
    if (EPI == SKX_EPI_RESID) {
        // thread: row j, 4 consecutive columns; x += (slabs + bias); row sums of squares
        constexpr int TPR = NW * 4;  // threads per row (16 or 32, inside one wave)
        const int j = tid / TPR, n = c0 + 4 * (tid % TPR);
        float ss = 0.f;
        if (j < nbz) {
            float* xr = f.x + (size_t)(z * SK_ROWS + j) * N + n;
            const float4 xo = *reinterpret_cast<const float4*>(xr);
            const float4 bb = f.bias ? *reinterpret_cast<const float4*>(f.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float2 r0 = slab2(j, n), r1 = slab2(j, n + 2);
            float r[4] = {r0.x, r0.y, r1.x, r1.y};
            if (f.bias) {
                r[0] += bb.x;
                r[1] += bb.y;
                r[2] += bb.z;
                r[3] += bb.w;
            }
            const float4 v = make_float4(xo.x + r[0], xo.y + r[1], xo.z + r[2], xo.w + r[3]);
            *reinterpret_cast<float4*>(xr) = v;
            ss = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, v.w * v.w)));
            if (f.planes) {
                // the next projection's planes: x * w (* (1 + ada)); its inverse RMS is applied
                // to its MFMA results (SKX_PRO_SCALE)
                const float4 ww = *reinterpret_cast<const float4*>(f.nw + n);
                const float4 aa = f.ada ? *reinterpret_cast<const float4*>(f.ada + n) : make_float4(0.f, 0.f, 0.f, 0.f);
                const float ve[4] = {v.x, v.y, v.z, v.w}, we[4] = {ww.x, ww.y, ww.z, ww.w}, ae[4] = {aa.x, aa.y, aa.z, aa.w};
                uint16_t hh[4], mm[4], ll[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    float y = ve[e] * we[e];
                    if (f.ada) y *= (1.0f + ae[e]);
                    split3(y, hh[e], mm[e], ll[e]);
                }
                const int jj = z * SK_ROWS + j;
                *reinterpret_cast<uint2*>(f.planes + frag_at(jj, N, 0, n)) =
                    make_uint2(hh[0] | ((uint32_t)hh[1] << 16), hh[2] | ((uint32_t)hh[3] << 16));
                *reinterpret_cast<uint2*>(f.planes + frag_at(jj, N, 1, n)) =
                    make_uint2(mm[0] | ((uint32_t)mm[1] << 16), mm[2] | ((uint32_t)mm[3] << 16));
                *reinterpret_cast<uint2*>(f.planes + frag_at(jj, N, 2, n)) =
                    make_uint2(ll[0] | ((uint32_t)ll[1] << 16), ll[2] | ((uint32_t)ll[3] << 16));
            }
        }
#pragma unroll
        for (int o = 1; o < TPR; o <<= 1) ss += __shfl_xor(ss, o, 64);
        if (tid % TPR == 0) f.ssq_out[((size_t)z * X + xi) * SK_ROWS + j] = ss;
    } else if (EPI == SKX_EPI_SWIGLU) {
        // thread: row j, hidden units h0, h0 + 1 (W1 row rg, W3 row rg + 16: upload_w13)
        constexpr int TPR = NW * 4;
        const int j = tid / TPR, pp = tid % TPR;
        if (j < nbz) {
            const int H = N / 2, h0 = xi * NW * 8 + 2 * pp;
            const int rg = (h0 >> 4) * 32 + (h0 & 15);
            const float2 g2 = slab2(j, rg), u2 = slab2(j, rg + 16);
            uint16_t hh[2], mm[2], ll[2];
            split3(silu(g2.x) * u2.x, hh[0], mm[0], ll[0]);
            split3(silu(g2.y) * u2.y, hh[1], mm[1], ll[1]);
            const int jj = z * SK_ROWS + j;
            *reinterpret_cast<uint32_t*>(f.planes + frag_at(jj, H, 0, h0)) = hh[0] | ((uint32_t)hh[1] << 16);
            *reinterpret_cast<uint32_t*>(f.planes + frag_at(jj, H, 1, h0)) = mm[0] | ((uint32_t)mm[1] << 16);
            *reinterpret_cast<uint32_t*>(f.planes + frag_at(jj, H, 2, h0)) = ll[0] | ((uint32_t)ll[1] << 16);
        }
    } else {
        // SKX_EPI_QKV: column pairs (n, n + 1), two per thread (k_slabs_rope_kv)
        constexpr int PPR = NW * 8;  // pairs per row
#pragma unroll
        for (int it = 0; it < 2; it++) {
            const int item = tid + it * NW * 64;
            const int j = item / PPR, n = c0 + 2 * (item % PPR);
            if (j >= nbz) continue;
            const int i = z * SK_ROWS + j;
            const int slot = (f.pos0 + i) % f.cap;
            const float2 bb = f.bias ? *reinterpret_cast<const float2*>(f.bias + n) : make_float2(0.f, 0.f);
            const float2 cs = n < f.qd + f.kvd
                                  ? *reinterpret_cast<const float2*>(f.rope + (size_t)i * f.hd + 2 * (n % f.hd / 2))
                                  : make_float2(1.f, 0.f);
            const float2 xx = slab2(j, n);
            float x0 = xx.x, x1 = xx.y;
            if (f.bias) {
                x0 += bb.x;
                x1 += bb.y;
            }
            if (n >= f.qd + f.kvd) {
                float* vr = f.Vc + (size_t)slot * f.kvd + (n - f.qd - f.kvd);
                vr[0] = x0;
                vr[1] = x1;
                continue;
            }
            float* dst = n < f.qd ? f.q + (size_t)i * f.qd + n : f.Kc + (size_t)slot * f.kvd + (n - f.qd);
            dst[0] = x0 * cs.x - x1 * cs.y;
            dst[1] = x0 * cs.y + x1 * cs.x;
        }
    }
}

// im2col for the causal conv stem (voxtral_kernels.c:430-447):
// A[t][ic*3 + k] = src[(stride*t + off + k) * C + ic]
__global__ __launch_bounds__(256) void k_im2col3(const float* __restrict__ src, int C, int T,
                                                 int stride, int off, float* __restrict__ A) {
    const int t = blockIdx.x;
    const int KK = C * 3;
    for (int e = threadIdx.x; e < KK; e += 256) {
        int ic = e / 3, k = e % 3;
        A[(size_t)t * KK + e] = src[(size_t)(stride * t + off + k) * C + ic];
    }
}

// mel tail update with the reference's quirk for 1-frame chunks (voxtral.c:637-643):
// tail = last two frames, or [0, only] when the chunk had a single frame.
__global__ void k_mel_tail(const float* __restrict__ melp, int n_new, int MB, float* __restrict__ tail) {
    // melp points at the [tail(2) + new] buffer; tail is its first two rows
    for (int b = threadIdx.x; b < MB; b += blockDim.x) {
        float t0, t1;
        if (n_new >= 2) {
            t0 = melp[(size_t)(2 + n_new - 2) * MB + b];
            t1 = melp[(size_t)(2 + n_new - 1) * MB + b];
        } else {
            t0 = 0.f;
            t1 = melp[(size_t)(2 + n_new - 1) * MB + b];
        }
        tail[b] = t0;
        tail[MB + b] = t1;
    }
}

// ============================================================================
// Incremental log-mel on the device (voxtral_audio.c:454-513, one block per frame).
// Frame f reads samples[start0 + 160 f .. + 400): Hann-windowed, direct 201 x 400 DFT with
// the reference's float tables (cos/sin of 2 pi k n / 400 in float, transposed [n][k] so
// the threads' k are consecutive), power re^2 + im^2, 128 Slaney filters ([k][b] order),
// log10 clamped at LOG_MEL_MAX - 8, (v + 4) / 4.  Every product and sum is a separately
// rounded f32 operation in the reference's order (n ascending, then k ascending): no FMA
// contraction (#pragma below), so only log10f's last bit can differ from the CPU path.
// ============================================================================
constexpr int MELK_FFT = 400, MELK_FREQ = 201, MELK_HOP = 160, MELK_BINS = 128;

// F frames per block: every table element a thread loads serves F frames (the tables are
// 2 x 321 KB, read from L2 by every block: one frame per block spent most of its time on
// them); each frame's products and sums are the same operations in the same order as with
// one frame per block, so the bits do not depend on F
template <int F>
__global__ __launch_bounds__(256) void k_mel_frames(const float* __restrict__ samples, long long start0, int nframes,
                                                    const float* __restrict__ window,
                                                    const float* __restrict__ dcosT,
                                                    const float* __restrict__ dsinT,
                                                    const float* __restrict__ filtT, float log_min,
                                                    float* __restrict__ mel) {
    // hipcc contracts a * b + c into an FMA by default; the reference rounds the product
    // first, which moves low-power bins by up to 1e-4 relative
#pragma clang fp contract(off)
    __shared__ float win[F][MELK_FFT];
    __shared__ float pw[F][MELK_FREQ];
    const int tid = threadIdx.x;
    const int f0 = blockIdx.x * F, nf = min(F, nframes - f0);
    for (int i = tid; i < F * MELK_FFT; i += 256) {
        const int f = i / MELK_FFT, n = i % MELK_FFT;
        win[f][n] = f < nf ? samples[start0 + (long long)(f0 + f) * MELK_HOP + n] * window[n] : 0.f;
    }
    __syncthreads();
    // one frame per block: the table entries are loaded 40 (67) at a time ahead of their use
    // (the loop-carried sums keep the reference's order; with one load pair per iteration the
    // L2 latency of every iteration was exposed: 50 frames 20.4 -> 13.0 us; 100 at a time 15.8);
    // several frames per block keep one load pair per iteration (their frames' arithmetic
    // covers it: 3,000 frames at 4 per block 43.4 us, against 53.4 with the batched loads)
    constexpr int UN = F == 1 ? 40 : 1, UK = F == 1 ? 67 : 1;  // 400 = 10 x 40, 201 = 3 x 67
    if (tid < MELK_FREQ) {
        float re[F], im[F];
#pragma unroll
        for (int f = 0; f < F; f++) re[f] = im[f] = 0.f;
        for (int n0 = 0; n0 < MELK_FFT; n0 += UN) {
            float cc[UN], sv[UN];
#pragma unroll
            for (int u = 0; u < UN; u++) {
                cc[u] = dcosT[(n0 + u) * MELK_FREQ + tid];
                sv[u] = dsinT[(n0 + u) * MELK_FREQ + tid];
            }
#pragma unroll
            for (int u = 0; u < UN; u++)
#pragma unroll
                for (int f = 0; f < F; f++) {
                    const float w = win[f][n0 + u];
                    re[f] = re[f] + w * cc[u];
                    im[f] = im[f] + w * sv[u];
                }
        }
#pragma unroll
        for (int f = 0; f < F; f++) pw[f][tid] = re[f] * re[f] + im[f] * im[f];
    }
    __syncthreads();
    if (tid < MELK_BINS) {
        float sum[F];
#pragma unroll
        for (int f = 0; f < F; f++) sum[f] = 0.f;
        for (int k0 = 0; k0 < MELK_FREQ; k0 += UK) {
            float fw[UK];
#pragma unroll
            for (int u = 0; u < UK; u++) fw[u] = filtT[(k0 + u) * MELK_BINS + tid];
#pragma unroll
            for (int u = 0; u < UK; u++)
#pragma unroll
                for (int f = 0; f < F; f++) sum[f] = sum[f] + fw[u] * pw[f][k0 + u];
        }
#pragma unroll
        for (int f = 0; f < F; f++) {
            if (f >= nf) break;
            float v = sum[f];
            if (v < 1e-10f) v = 1e-10f;
            v = log10f(v);
            if (v < log_min) v = log_min;
            mel[(size_t)(f0 + f) * MELK_BINS + tid] = (v + 4.0f) / 4.0f;
        }
    }
}

// vox_mel_finish's right reflect (voxtral_audio.c:615-623): dst[i] = buf[real_end - 2 - i]
__global__ void k_mel_reflect(float* __restrict__ buf, long long n, long long real_end, int len) {
    for (int i = threadIdx.x; i < len; i += blockDim.x) {
        const long long src = real_end - 2 - i;
        buf[n + i] = src >= 0 ? buf[src] : 0.f;
    }
}

// ============================================================================
// Host-side launchers
// ============================================================================
#define LAUNCH_CHECK() \
    do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return e__; } while (0)

hipError_t launch_rmsnorm_rows(const float* x, int ldx, float* y, int ldy, const float* w,
                               const float* ada, int M, int D, float eps, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rmsnorm_rows, dim3(M), dim3(256), 0, st, x, ldx, y, ldy, w, ada, D, eps);
    LAUNCH_CHECK();
    return hipSuccess;
}

// k_gemm2 split count: two 128x128 blocks per CU (LDS), so a launch of T tiles x S slices
// runs ceil(T S / 512) rounds of K/(64 S) stages (~1.3 us each, two blocks sharing a CU);
// a split adds the partial tiles' round trip (2 S M N 4 B at ~5 TB/s) and the reduce.
static int gemm2_ksplit(int M, int N, int K, size_t ws_elems, int tn = G2_N) {
    // tn = 256 (WN = 4): half the tiles, each with twice the MFMA work per stage
    const int tiles = (N / tn) * ((M + G2_M - 1) / G2_M);
    const double tstage = tn == G2_N ? 1.3 : 2.6;
    int best = 1;
    double best_t = 1e30;
    for (int s = 1; s <= 32; s *= 2) {
        if (K % (s * G2_K) || (s > 1 && ((size_t)s * M * N > ws_elems || K / s < 2 * G2_K))) break;
        const double rounds = (double)((tiles * s + 511) / 512);
        double t = rounds * (K / s / G2_K) * tstage;
        if (s > 1) t += 4.0 + 2.0 * s * (double)M * N * 4 / 5e6;
        if (t < best_t) { best_t = t; best = s; }
    }
    return best;
}

template <int E, int Q, int NP, int WN>
static hipError_t gemm2_launch_np(dim3 grid, hipStream_t st, const float* A, int lda, const void* W, int K,
                                  int M, int N, const float* wscale, const float* bias, float* C, int ldc) {
    static bool attr = false;  // opt in to > 64 KB of dynamic LDS once per instance
    const size_t lds = ((size_t)NP * G2_M + 64 * WN) * G2_LDS * 2;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm2<E, Q, NP, WN>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL((k_gemm2<E, Q, NP, WN>), grid, dim3(128 * WN), lds, st, A, lda, W, K, M, N, wscale, bias, C,
                       ldc);
    return hipGetLastError();
}

int g_gemm_wide = -1;  // tools/kbench knob: 128 x 256 tiles where they apply (-1: VOX_HIP_GEMM_WIDE, default on)
static bool gemm_wide(int M, int N, const float* wscale) {
    if (g_gemm_wide < 0) {
        const char* e = getenv("VOX_HIP_GEMM_WIDE");
        g_gemm_wide = (e && atoi(e) == 0) ? 0 : 1;
    }
    if (!g_gemm_wide || wscale || gemm_planes() != 2 || N % 256) return false;
    // wide tiles where they still fill the GPU, or where both widths need split-K anyway
    // (tools/kbench at M = 677: W1|W3 61.9 -> 53.3, wo 27.8 -> 25.9, w2 45.6 -> 40.2 us; the
    // QKV's 288 narrow tiles would drop to 144 wide ones: 51.4 -> 62.5, kept narrow)
    const int mt = (M + G2_M - 1) / G2_M;
    return (N / 256) * mt >= 192 || (N / G2_N) * mt < 128;
}

template <int E, int Q>
static hipError_t gemm2_launch(dim3 grid, hipStream_t st, const float* A, int lda, const void* W, int K,
                               int M, int N, const float* wscale, const float* bias, float* C, int ldc) {
    if (!Q && gemm_wide(M, N, wscale)) {
        grid.x = N / 256;
        return gemm2_launch_np<E, 0, 2, 4>(grid, st, A, lda, W, K, M, N, wscale, bias, C, ldc);
    }
    return gemm_planes() == 2 ? gemm2_launch_np<E, Q, 2, 2>(grid, st, A, lda, W, K, M, N, wscale, bias, C, ldc)
                              : gemm2_launch_np<E, Q, 3, 2>(grid, st, A, lda, W, K, M, N, wscale, bias, C, ldc);
}

template <int EPI>
static hipError_t gemm_t(const float* A, int lda, const void* W, const float* wscale, int K, int M,
                         int N, const float* bias, float* C, int ldc, hipStream_t st, float* ws,
                         size_t ws_elems) {
    const int S = ws ? gemm2_ksplit(M, N, K, ws_elems, gemm_wide(M, N, wscale) ? 256 : G2_N) : 1;
    if (S > 1) {
        dim3 grid(N / G2_N, (M + G2_M - 1) / G2_M, S);
        hipError_t e = wscale ? gemm2_launch<EPI_PARTIAL, 1>(grid, st, A, lda, W, K, M, N, wscale, nullptr, ws, N)
                              : gemm2_launch<EPI_PARTIAL, 0>(grid, st, A, lda, W, K, M, N, wscale, nullptr, ws, N);
        if (e != hipSuccess) return e;
        const size_t outs = (size_t)M * (EPI == EPI_SWIGLU ? N / 2 : N);
        hipLaunchKernelGGL(k_splitk_reduce<EPI>, dim3((unsigned)((outs + 255) / 256)), dim3(256), 0, st, ws, S, M,
                           N, wscale, bias, C, ldc);
        LAUNCH_CHECK();
        return hipSuccess;
    }
    dim3 grid(N / G2_N, (M + G2_M - 1) / G2_M, 1);
    return wscale ? gemm2_launch<EPI, 1>(grid, st, A, lda, W, K, M, N, wscale, bias, C, ldc)
                  : gemm2_launch<EPI, 0>(grid, st, A, lda, W, K, M, N, wscale, bias, C, ldc);
}

hipError_t launch_gemm(int epi, int nsplit, const float* A, int lda, const void* W,
                       const float* wscale, int K, int M, int N, const float* bias, float* C,
                       int ldc, hipStream_t st, float* ws, size_t ws_elems) {
    if (M <= 0) return hipSuccess;
    // nsplit: the activation split of the reference-boundary callers; the planes are set by
    // vox_hip_set_gemm_planes (2 or 3), shapes are padded by the callers to 128 / 64
    if (nsplit != 3 || N % G2_N || K % G2_K || lda % 4) return hipErrorInvalidValue;
#define GEMM_CASE(E) \
    if (epi == E) return gemm_t<E>(A, lda, W, wscale, K, M, N, bias, C, ldc, st, ws, ws_elems);
    GEMM_CASE(EPI_STORE) GEMM_CASE(EPI_RESID) GEMM_CASE(EPI_GELU) GEMM_CASE(EPI_GELU_ERF) GEMM_CASE(EPI_SWIGLU)
#undef GEMM_CASE
    return hipErrorInvalidValue;
}

hipError_t launch_rope_kv(const float* qkv, int M, int qd, int kvd, int hd, const float* rope,
                          int pos0, float* q, float* Kc, float* Vc, int cap, hipStream_t st, int kv16) {
    if (M <= 0) return hipSuccess;
    if (kvd % 2) return hipErrorInvalidValue;
    if (kv16)
        hipLaunchKernelGGL(k_rope_kv<kvh_t>, dim3(M), dim3(256), 0, st, qkv, M, qd, kvd, hd, rope, pos0, q, Kc, Vc, cap);
    else
        hipLaunchKernelGGL(k_rope_kv<float>, dim3(M), dim3(256), 0, st, qkv, M, qd, kvd, hd, rope, pos0, q, Kc, Vc, cap);
    LAUNCH_CHECK();
    return hipSuccess;
}

VOX_KB_KNOB(g_attn_blocks, 0);  // tools/kbench knob: target grid size of the key-range split (0 = 512)

hipError_t launch_rope_kv_rows(const float* qkv, int N, int qd, int kvd, int hd, const float* rope_table,
                               const EncRows& er, float* q, int cap, hipStream_t st) {
    if (N <= 0) return hipSuccess;
    if (er.B < 1 || er.B > VOX_MAX_BATCH) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_rope_kv_rows, dim3(N), dim3(256), 0, st, qkv, qd, kvd, hd, rope_table, er, q, cap);
    LAUNCH_CHECK();
    return hipSuccess;
}

// VOX_HIP_ATT_PLANES=0: the attention writes f32 rows and k_split_fplanes makes the wo planes
// (the round-5 path) instead of the attention writing the planes itself
static int g_att_planes = -1;
static bool att_planes() {
    if (g_att_planes < 0) {
        const char* e = getenv("VOX_HIP_ATT_PLANES");
        g_att_planes = (e && atoi(e) == 0) ? 0 : 1;
    }
    return g_att_planes == 1;
}

hipError_t launch_attn_rows(int hd, const float* Q, const EncRows& er, int N, int cap, float* O, int H, int KVH,
                            int window, float scale, float* ws, size_t ws_elems, hipStream_t st, uint16_t* xs) {
    if (N <= 0) return hipSuccess;
    if (er.B < 1 || er.B > VOX_MAX_BATCH || (hd != 64 && hd != 128)) return hipErrorInvalidValue;
    if (xs && N > PLANE_MAX_ROWS) return hipErrorInvalidValue;
    int qbm = 0, keys = 0;
    for (int b = 0; b < er.B; b++) {
        qbm = std::max(qbm, (er.nr[b] + 15) / 16);
        const int ks = std::max(er.pos0[b] - window + 1, 0);
        keys = std::max(keys, er.pos0[b] + er.nr[b] - ks);
    }
    if (qbm == 0) return hipSuccess;
    // key splits as launch_attn_rows_mf picks them, over every stream's (head, query block)s
    int ns = 1;
    int nblk = 0;
    for (int b = 0; b < er.B; b++) nblk += H * ((er.nr[b] + 15) / 16);
    if (ws && nblk < 256) {
        ns = std::min((keys + 63) / 64, std::max(1, 256 / nblk));
        while (ns > 1 && (size_t)H * N * ns * (hd + 2) > ws_elems) ns--;
    }
    dim3 grid(H, qbm, ns * er.B);
    // xs: the output rows as the wo input's planes (by the attention itself, or by the combine)
    uint16_t* kxs = ns == 1 && att_planes() ? xs : nullptr;
    if (hd == 64)
        hipLaunchKernelGGL((k_attn_mf<64, float, 1>), grid, dim3(256), 0, st, Q, H * hd, nullptr, nullptr, cap, O, H * hd,
                           N, H, KVH, 0, 0, window, scale, ns, ws, er, kxs);
    else
        hipLaunchKernelGGL((k_attn_mf<128, float, 1>), grid, dim3(256), 0, st, Q, H * hd, nullptr, nullptr, cap, O,
                           H * hd, N, H, KVH, 0, 0, window, scale, ns, ws, er, kxs);
    LAUNCH_CHECK();
    if (ns > 1) {
        if (hd == 64)
            hipLaunchKernelGGL(k_attn_tiled_combine<64>, dim3(H, N), dim3(64), 0, st, ws, ns, N, O, H * hd, xs);
        else
            hipLaunchKernelGGL(k_attn_tiled_combine<128>, dim3(H, N), dim3(128), 0, st, ws, ns, N, O, H * hd, xs);
        LAUNCH_CHECK();
    } else if (xs && !kxs) {
        return launch_split_fplanes(O, N, H * hd, xs, st);
    }
    return hipSuccess;
}

hipError_t launch_attn_rows_mf(int hd, const float* Q, int ldq, const float* Kc, const float* Vc,
                             int cap, float* O, int ldo, int M, int H, int KVH, int q_pos0,
                             int k_first, int window, float scale, hipStream_t st, float* ws, size_t ws_elems,
                             uint16_t* xs, int kv16) {
    if (M <= 0) return hipSuccess;
    if (hd != 64 && hd != 128) return hipErrorInvalidValue;
    if (xs && (M > PLANE_MAX_ROWS || ldo != H * hd)) return hipErrorInvalidValue;
    // 16 queries per block: 32 (each K/V tile of a 25-row streaming chunk read once per head
    // instead of twice) measured slower, 15.7 vs 14.6 us (tools/kbench, round 1)
    const int QT = 16;
    const int qb = (M + QT - 1) / QT;
    // key-range splits when the (head, query block) grid cannot fill the chip: at least 64
    // keys per split, about 256 blocks in all (a 25-row streaming chunk over ~775 keys: 4)
    int ks = q_pos0 - window + 1;
    if (ks < k_first) ks = k_first;
    const int keys = q_pos0 + M - ks;
    int ns = 1;
    if (ws && H * qb < 256) {
        // (k_attn_mf, 25 rows x 775 keys: 256 blocks 10.4 us, 512 11.8, 128 13.9, 1024 12.0)
        const int target = g_attn_blocks ? g_attn_blocks : 256;
        ns = std::min((keys + 63) / 64, std::max(1, target / (H * qb)));
        while (ns > 1 && (size_t)H * M * ns * (hd + 2) > ws_elems) ns--;
    }
    dim3 grid(H, qb, ns);
    if (kv16) {
        // the 16-bit decoder ring (prefill)
        if (hd != 128) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_attn_mf<128, kvh_t>), grid, dim3(256), 0, st, Q, ldq, Kc, Vc, cap, O, ldo, M, H, KVH,
                           q_pos0, k_first, window, scale, ns, ws);
    } else if (hd == 64) {
        hipLaunchKernelGGL(k_attn_mf<64>, grid, dim3(256), 0, st, Q, ldq, Kc, Vc, cap, O, ldo, M, H, KVH, q_pos0,
                           k_first, window, scale, ns, ws, EncRows{}, ns == 1 && att_planes() ? xs : nullptr);
    } else {
        hipLaunchKernelGGL(k_attn_mf<128>, grid, dim3(256), 0, st, Q, ldq, Kc, Vc, cap, O, ldo, M, H, KVH, q_pos0,
                           k_first, window, scale, ns, ws, EncRows{}, ns == 1 && att_planes() ? xs : nullptr);
    }
    LAUNCH_CHECK();
    if (ns > 1) {
        // with xs the combine writes the wo planes itself
        if (hd == 64)
            hipLaunchKernelGGL(k_attn_tiled_combine<64>, dim3(H, M), dim3(64), 0, st, ws, ns, M, O, ldo, xs);
        else
            hipLaunchKernelGGL(k_attn_tiled_combine<128>, dim3(H, M), dim3(128), 0, st, ws, ns, M, O, ldo, xs);
        LAUNCH_CHECK();
    } else if (xs && (kv16 || !att_planes())) {
        return launch_split_fplanes(O, M, H * hd, xs, st);
    }
    return hipSuccess;
}

hipError_t launch_slabs_rope_kv(const float* part, int S, int M, const float* bias, int qd, int kvd, int hd,
                                const float* rope, int pos0, float* q, float* Kc, float* Vc, int cap, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    if (M > SK_MAX_ROWS || S < 1 || qd % hd || kvd % hd || hd % 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_slabs_rope_kv, dim3((qd / 2 + kvd + 255) / 256, M), dim3(256), 0, st, part, S, bias, qd, kvd,
                       hd, rope, pos0, q, Kc, Vc, cap);
    LAUNCH_CHECK();
    return hipSuccess;
}

#ifdef VOX_GEMV_STAMPS
// diagnostic build only (tools/kbench_stamps): where k_gemv's per-block stamps go (null: off)
hipError_t gemv_set_stamps(unsigned long long* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_gemv_stamps), &p, sizeof p); }
#endif
VOX_KB_KNOB(g_gemv_rb, 0);  // tools/kbench knob: force 4- or 8-row groups (0 = automatic)
// Rows per group: each block should stream at least two groups, so that the next group's
// loads overlap this group's reduction and epilogue (one group per block left every block
// idle at its tail).  tools/kbench, bf16 / 768 blocks: QKV 10.2 -> 8.5 us with 4-row
// groups, W1|W3 20.5 -> 20.0, W2 12.1 -> 11.4 and wo 6.7 -> 6.4 with 2-row groups; the LM
// head (16 groups per block at 8 rows) keeps 8.
static int gemv_rb(int rows) {
    if (g_gemv_rb && rows % g_gemv_rb == 0) return g_gemv_rb;
    if (rows >= 65536 && rows % 8 == 0) return 8;
    if (rows >= 6144 && rows % 4 == 0) return 4;
    return 2;
}

VOX_KB_KNOB(g_gemv_maxb, 0);  // tools/kbench knob: grid cap other than GEMV_MAX_BLOCKS (no LM head)
int gemv_grid(int rows) {
    // the largest divisor of the group count that fits 4 blocks per CU: every block then
    // runs the same number of groups (no tail); tools/kbench VOX_KB_ONLY=grid: 1536-2304
    // blocks were slower on every decode shape, bf16 and Q8 (profiles/r3_kbench_gemv_grid.txt)
    const int ng = rows / gemv_rb(rows), maxb = g_gemv_maxb ? g_gemv_maxb : GEMV_MAX_BLOCKS;
    int best = 1;
    for (int gsz = 1; gsz <= maxb && gsz <= ng; gsz++)
        if (ng % gsz == 0) best = gsz;
    if (best < 256 && ng > maxb) best = maxb;  // no good divisor: accept a tail
    return best;
}

template <int P, int E, int RB, int Q8>
static const void* gemv_fn(int kq) {
    switch (kq) {
        case 1: return reinterpret_cast<const void*>(&k_gemv<P, E, RB, 1, Q8>);
        case 2: return reinterpret_cast<const void*>(&k_gemv<P, E, RB, 2, Q8>);
        case 3: return reinterpret_cast<const void*>(&k_gemv<P, E, RB, 3, Q8>);
        case 4: return reinterpret_cast<const void*>(&k_gemv<P, E, RB, 4, Q8>);
        case 5: return reinterpret_cast<const void*>(&k_gemv<P, E, RB, 5, Q8>);
        default: return nullptr;
    }
}

int gemv_occupancy(const void* fn) {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, 0) != hipSuccess) occ = 0;
    return occ;
}

template <int P, int E, int RB, int Q8>
static hipError_t gemv_k(const GemvArgs& a, int grid, hipStream_t st) {
    const int kq = ((Q8 ? a.K >> 4 : a.K >> 3) + 255) / 256;
    switch (kq) {
#define KQ_CASE(Q) case Q: hipLaunchKernelGGL((k_gemv<P, E, RB, Q, Q8>), dim3(grid), dim3(256), 0, st, a); break;
        KQ_CASE(1) KQ_CASE(2) KQ_CASE(3) KQ_CASE(4) KQ_CASE(5)
#undef KQ_CASE
        default: return hipErrorInvalidValue;
    }
    LAUNCH_CHECK();
    return hipSuccess;
}

// kernel instance launch_gemv would use (tools, occupancy queries)
const void* gemv_kernel(int pro, int epi, const GemvArgs& a) {
    const int rb = gemv_rb(a.rows);
    const int kq = ((a.wscale ? a.K >> 4 : a.K >> 3) + 255) / 256;
#define GEMV_FN(P, E)                                                                     \
    if (pro == P && epi == E)                                                             \
        return rb == 8 ? (a.wscale ? gemv_fn<P, E, 8, 1>(kq) : gemv_fn<P, E, 8, 0>(kq))   \
             : rb == 2 ? (a.wscale ? gemv_fn<P, E, 2, 1>(kq) : gemv_fn<P, E, 2, 0>(kq))   \
                       : (a.wscale ? gemv_fn<P, E, 4, 1>(kq) : gemv_fn<P, E, 4, 0>(kq));
    GEMV_FN(PRO_NONE, EPI_STORE) GEMV_FN(PRO_NONE, EPI_RESID) GEMV_FN(PRO_NORM, EPI_QKV)
    GEMV_FN(PRO_NORM_ADA, EPI_SWIGLU) GEMV_FN(PRO_NORM, EPI_LOGITS) GEMV_FN(PRO_NORM, EPI_LOGITS_ALT)
    GEMV_FN(PRO_NORM, EPI_QKV_BIAS) GEMV_FN(PRO_NORM, EPI_SWIGLU)
#undef GEMV_FN
    return nullptr;
}

template <int P, int E, int RB>
static hipError_t gemv_q(const GemvArgs& a, int grid, hipStream_t st) {
    return a.wscale ? gemv_k<P, E, RB, 1>(a, grid, st) : gemv_k<P, E, RB, 0>(a, grid, st);
}

// The same launch with HIP events recorded by the kernel's own dispatch packet
// (hipExtLaunchKernel): they bracket the kernel itself, not the marker packets an
// event-record node adds.  Eager launches only (not capturable into a graph).
hipError_t launch_gemv_timed(int pro, int epi, const GemvArgs& a, hipEvent_t start, hipEvent_t stop,
                             hipStream_t st) {
    const void* fn = gemv_kernel(pro, epi, a);
    if (!fn) return hipErrorInvalidValue;
    GemvArgs args = a;
    void* kargs[] = {&args};
    return hipExtLaunchKernel(fn, dim3(gemv_grid(a.rows)), dim3(256), kargs, 0, st, start, stop, 0);
}

// the shapes launch_gemv accepts: whole 16-B chunks per row, whole row groups, and at most
// 5 rounds of 256 chunks per row (the instantiated KQ)
bool gemv_ok(int rows, int K, int q8) {
    const int kc = q8 ? K >> 4 : K >> 3;
    return rows > 0 && K > 0 && K % (q8 ? 16 : 8) == 0 && rows % gemv_rb(rows) == 0 && (kc + 255) / 256 <= 5;
}

hipError_t launch_gemv(int pro, int epi, const GemvArgs& a, hipStream_t st) {
    const int rb = gemv_rb(a.rows);
    if (!gemv_ok(a.rows, a.K, a.wscale != nullptr)) return hipErrorInvalidValue;
    if (epi == EPI_QKV_BIAS && !a.bias) return hipErrorInvalidValue;
    const int grid = gemv_grid(a.rows);
#define GEMV_CASE(P, E) \
    if (pro == P && epi == E)                                                            \
        return rb == 8 ? gemv_q<P, E, 8>(a, grid, st) : rb == 2 ? gemv_q<P, E, 2>(a, grid, st) : gemv_q<P, E, 4>(a, grid, st);
    GEMV_CASE(PRO_NONE, EPI_STORE) GEMV_CASE(PRO_NONE, EPI_RESID) GEMV_CASE(PRO_NORM, EPI_QKV)
    GEMV_CASE(PRO_NORM_ADA, EPI_SWIGLU) GEMV_CASE(PRO_NORM, EPI_LOGITS) GEMV_CASE(PRO_NORM, EPI_LOGITS_ALT)
    // the encoder's single-row chunks (run_encoder_rows_gemv)
    GEMV_CASE(PRO_NORM, EPI_QKV_BIAS) GEMV_CASE(PRO_NORM, EPI_SWIGLU)
#undef GEMV_CASE
    return hipErrorInvalidValue;
}

// partial slots per head (at least 4)
int attn_maxch(int window) { return std::max(4, (window + ATT_MIN_BK - 1) / ATT_MIN_BK); }
int attn_maxsplits(int window) { return (window + ATT_BK - 1) / ATT_BK; }
VOX_KB_KNOB(g_attn_lw, 0);  // tools/kbench knob: waves per long-context block (2 or 4; 0 = ATT_LWAVES)
VOX_KB_KNOB(g_attn_kvfast, 1);  // long-context grid with the kv heads of a key range adjacent (tools/kbench: 0 = off)
// batched step, <= 256 keys: 128-key blocks when (stream, kv head) blocks < 256 (16 streams
// 6582 -> 6695 tok/s, 8 streams 3556 -> 3632; VOX_HIP_ATT_BSPLIT=0: off)
int g_attn_bsplit = -1;

// past 256 keys: blocks of NWV x 16 keys per (kv head, key range); the last block of a kv
// head merges the partials
// (kv heads of one key range on neighbouring blocks, kvfast: L = 8192 f32 over 26 layers'
// rings 27.4 -> 22.9 us per layer, tools/kbench VOX_KB_ONLY=attn)
template <int HD, int NWV, class KT>
static void attn_long(const AttnPtrs& p, int nb, int cap, int pos_host, int window, float scale, int H, int KVH,
                      int splits, int maxs, hipStream_t st) {
    const int nsb = splits * (ATT_BK / (NWV * ATT_CH));  // key-range blocks per kv head
    if (g_attn_kvfast)
        hipLaunchKernelGGL((k_attn_decode<HD, 4, 0, 0, NWV, KT>), dim3(nsb * KVH, 1, nb), dim3(NWV * 64), 0, st, p,
                           cap, pos_host, window, scale, H, KVH, maxs, AttnFuse{}, 1);
    else
        hipLaunchKernelGGL((k_attn_decode<HD, 4, 0, 0, NWV, KT>), dim3(nsb, KVH, nb), dim3(NWV * 64), 0, st, p, cap,
                           pos_host, window, scale, H, KVH, maxs);
}

// splits = 256-key spans provided per head group (>= the context's ceil(L / 256) for every
// step the launch serves).  1: 1024-thread blocks of 256 keys, no combine kernel.  > 1:
// 512-thread blocks of 128 keys per (kv head, span half) and k_attn_combine -- a 256-key
// block per CU had read K/V at the per-CU rate (L = 1000: 32 blocks, 12.3 us; now 10.0).
template <class KT>
static hipError_t attn_launch(int hd, const AttnPtrs& p, int nb, int cap, int pos_host, int window, float scale,
                              int H, int KVH, int splits, hipStream_t st) {
    const int maxs = attn_maxch(window);
    if (H % KVH || H / KVH > 4 || maxs > ATT_MAX_PARTS || splits < 1 || splits > attn_maxsplits(window) || nb < 1 ||
        nb > VOX_MAX_BATCH)
        return hipErrorInvalidValue;
    // batches of >= 4 streams: one block per (stream, kv head), K/V read once for its query
    // heads (16 streams: 15.8 -> ~10 us per layer); a single stream needs the 32 blocks
#define VOX_ATT(HD)                                                                                        \
    if (splits == 1 && nb >= 4) {                                                                         \
        hipLaunchKernelGGL((k_attn_decode<HD, 4, 0, 0, ATT_WAVES, KT>), dim3(1, KVH, nb), dim3(1024), 0, st, p, \
                           cap, pos_host, window, scale, H, KVH, maxs);                                    \
    } else if (splits == 1) {                                                                              \
        hipLaunchKernelGGL((k_attn_decode<HD, 1, 0, 0, ATT_WAVES, KT>), dim3(1, H, nb), dim3(1024), 0, st, p,   \
                           cap, pos_host, window, scale, H, KVH, maxs);                                    \
    } else if (g_attn_lw == 4 || (g_attn_lw == 2 && splits * 8 <= maxs)) {                                \
        if (g_attn_lw == 4) attn_long<HD, 4, KT>(p, nb, cap, pos_host, window, scale, H, KVH, splits, maxs, st); \
        else attn_long<HD, 2, KT>(p, nb, cap, pos_host, window, scale, H, KVH, splits, maxs, st);          \
    } else if (g_attn_lw == 16) {                                                                          \
        attn_long<HD, 16, KT>(p, nb, cap, pos_host, window, scale, H, KVH, splits, maxs, st);              \
    } else {                                                                                               \
        attn_long<HD, ATT_LWAVES, KT>(p, nb, cap, pos_host, window, scale, H, KVH, splits, maxs, st);      \
    }
    if (hd == 128) {
        VOX_ATT(128)
    } else if (hd == 64 && sizeof(KT) == 4) {
        VOX_ATT(64)
    } else {
        return hipErrorInvalidValue;
    }
#undef VOX_ATT
    LAUNCH_CHECK();
    return hipSuccess;
}

// splits = key blocks provided per head group (>= the context's ceil(L / 256) for every
// step the launch serves); 1 -> one block per query head, no combine kernel.
int g_attn_short = -1;  // k_attn_short for one stream's contexts <= 256 keys (VOX_HIP_ATT_SHORT=0: off)
// k_attn_short's keys 64..255 are loaded after the position read (waves 4..15): C2 on one
// box, all 256 speculative 655.3 / 655.4 / 655.7 tok/s, from wave 8 663.7 / 667.7 / 666.7; on
// another, from wave 8 672.3 / 670.7 / 673.2, from wave 4 676.6 / 676.7 / 676.2, from wave 2
// within noise of wave 4 (profiles/r4_attn_short_late_ab.txt, r4_attn_short_late2_ab.txt)
hipError_t launch_attn_decode(int hd, const float* q, const float* Kc, const float* Vc, int cap,
                              const int* state, int pos_host, int window, float scale, int H,
                              int KVH, float* part, float* out, int splits, hipStream_t st, int kv16) {
    if (g_attn_short < 0) {
        const char* e = getenv("VOX_HIP_ATT_SHORT");
        g_attn_short = (e && atoi(e) == 0) ? 0 : 1;
    }
    if (g_attn_short && splits == 1 && hd == 128 && window > ATT_BK && cap >= ATT_BK && H % KVH == 0) {
        // contexts of <= 256 keys (splits == 1) with a window of > 256: nothing has left the
        // window (lp < 256 < window) and the ring has not wrapped, so keys = slots 0..lp (a
        // window of exactly 256 would reach L = 256 again at lp >= 256 with wrapped slots)
        if (kv16)
            hipLaunchKernelGGL((k_attn_short<128, kvh_t, 4>), dim3(H), dim3(1024), 0, st, q,
                               reinterpret_cast<const kvh_t*>(Kc), reinterpret_cast<const kvh_t*>(Vc), state, pos_host,
                               scale, H, KVH, out);
        else
            hipLaunchKernelGGL((k_attn_short<128, float, 4>), dim3(H), dim3(1024), 0, st, q, Kc, Vc, state, pos_host,
                               scale, H, KVH, out);
        LAUNCH_CHECK();
        return hipSuccess;
    }
    AttnPtrs p;
    memset(&p, 0, sizeof p);
    p.q[0] = q; p.Kc[0] = Kc; p.Vc[0] = Vc; p.state[0] = state; p.part[0] = part; p.out[0] = out;
    return kv16 ? attn_launch<kvh_t>(hd, p, 1, cap, pos_host, window, scale, H, KVH, splits, st)
                : attn_launch<float>(hd, p, 1, cap, pos_host, window, scale, H, KVH, splits, st);
}

hipError_t launch_attn_decode_batch(int hd, const AttnPtrs& p, int nb, int cap, int window, float scale,
                                    int H, int KVH, int splits, hipStream_t st, int kv16) {
    return kv16 ? attn_launch<kvh_t>(hd, p, nb, cap, 0, window, scale, H, KVH, splits, st)
                : attn_launch<float>(hd, p, nb, cap, 0, window, scale, H, KVH, splits, st);
}

template <class KT>
static hipError_t attn_batch_fused(const AttnPtrs& p, const AttnFuse& f, int nb, int cap, int window, float scale,
                                   int H, int KVH, int splits, int maxs, hipStream_t st) {
    if (g_attn_bsplit < 0) {
        const char* e = getenv("VOX_HIP_ATT_BSPLIT");
        g_attn_bsplit = e ? std::max(0, std::min(2, atoi(e))) : 1;
    }
    // contexts <= 256 keys: one 1024-thread block per (stream, kv head) -- unless those blocks
    // cannot fill the chip (16 streams x 8 kv heads = 128 blocks on 256 CUs): then the 128-key
    // blocks of the long path (two per (stream, kv head), last arriver merges);
    // VOX_HIP_ATT_BSPLIT=2: the 128-key blocks at any row count
    if (splits == 1 && (!g_attn_bsplit || (g_attn_bsplit == 1 && nb * KVH >= 256))) {
        hipLaunchKernelGGL((k_attn_decode<128, 4, 0, 1, ATT_WAVES, KT>), dim3(1, KVH, nb), dim3(1024), 0, st, p, cap, 0,
                           window, scale, H, KVH, maxs, f);
        LAUNCH_CHECK();
        return hipSuccess;
    }
    hipLaunchKernelGGL((k_attn_decode<128, 4, 0, 1, ATT_LWAVES, KT>), dim3(splits * (ATT_BK / ATT_LBK) * KVH, 1, nb),
                       dim3(ATT_LWAVES * 64), 0, st, p, cap, 0, window, scale, H, KVH, maxs, f, 1);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_attn_batch_fused(int hd, const AttnPtrs& p, const AttnFuse& f, int nb, int cap, int window,
                                   float scale, int H, int KVH, int splits, hipStream_t st, int kv16) {
    const int maxs = attn_maxch(window);
    if (hd != 128 || H % KVH || H / KVH > 4 || maxs > ATT_MAX_PARTS || splits < 1 || splits > attn_maxsplits(window) ||
        nb < 1 || nb > VOX_MAX_BATCH || !f.qkv || !f.rope || !f.xs || f.S < 1 || f.N != (H + 2 * KVH) * hd)
        return hipErrorInvalidValue;
    return kv16 ? attn_batch_fused<kvh_t>(p, f, nb, cap, window, scale, H, KVH, splits, maxs, st)
                : attn_batch_fused<float>(p, f, nb, cap, window, scale, H, KVH, splits, maxs, st);
}
// diagnostic variants for tools/kbench (not used by the engine)
// the batched fused attention (128-key blocks, the bsplit grid) with per-wave phase stamps
// to p.out[0] (10 u64 per wave: DBG 4 in k_attn_decode)
hipError_t launch_attn_batch_dbg(const AttnPtrs& p, const AttnFuse& f, int nb, int cap, int window, float scale, int H,
                                 int KVH, int splits, hipStream_t st) {
    const int maxs = attn_maxch(window);
    if (!p.out[0] || nb < 1 || nb > VOX_MAX_BATCH || H % KVH || H / KVH > 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_attn_decode<128, 4, 4, 1, ATT_LWAVES, float>), dim3(splits * (ATT_BK / ATT_LBK) * KVH, 1, nb),
                       dim3(ATT_LWAVES * 64), 0, st, p, cap, 0, window, scale, H, KVH, maxs, f, 1);
    LAUNCH_CHECK();
    return hipSuccess;
}
hipError_t launch_attn_dbg(int dbg, const float* q, const float* Kc, const float* Vc, int cap,
                           const int* state, float* part, float* out, hipStream_t st) {
    dim3 grid(1, 32);
    AttnPtrs p;
    memset(&p, 0, sizeof p);
    p.q[0] = q; p.Kc[0] = Kc; p.Vc[0] = Vc; p.state[0] = state; p.part[0] = part; p.out[0] = out;
    if (dbg == 1) hipLaunchKernelGGL((k_attn_decode<128, 1, 1>), grid, dim3(1024), 0, st, p, cap, 0, 8192, 0.088f, 32, 8, 32);
    if (dbg == 3) hipLaunchKernelGGL((k_attn_decode<128, 1, 3>), grid, dim3(1024), 0, st, p, cap, 0, 8192, 0.088f, 32, 8, 32);
    if (dbg == 4) hipLaunchKernelGGL((k_attn_decode<128, 1, 4>), grid, dim3(1024), 0, st, p, cap, 0, 8192, 0.088f, 32, 8, 32);
    return hipGetLastError();
}

hipError_t launch_embed_step(const float* adapter, const void* emb, const float* esc, const int* state,
                             int D, float* x, hipStream_t st) {
    hipLaunchKernelGGL(k_embed_step, dim3((D + 255) / 256), dim3(256), 0, st, adapter, emb, esc, state, D, x);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_embed_rows(const float* adapter, const void* emb, const float* esc, int row0, int n,
                             int first_tok, int rest_tok, int D, float* x, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_embed_rows, dim3(n), dim3(256), 0, st, adapter, emb, esc, row0, first_tok, rest_tok, D, x);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_argmax_final(const float* pv, const int* pi, int n, int* state, int* tokens,
                               int cap, const float* adapter, int adapter_rows,
                               const void* emb, const float* esc, int D, float* x,
                               const float* part_alt, float* alts, hipStream_t st) {
    if (adapter && D > 16 * 256) return hipErrorInvalidValue;  // k_argmax_final: 16 next-input elements per thread
    hipLaunchKernelGGL(k_argmax_final, dim3(1), dim3(256), 0, st, pv, pi, n, state, tokens, cap,
                       adapter, adapter_rows, emb, esc, D, x, part_alt, alts);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_embed_batch(const BatchSlot* slots, int nb, const void* emb, const float* esc, int D, float* x,
                              hipStream_t st) {
    if (nb < 1 || nb > VOX_MAX_BATCH || !slots) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_embed_batch, dim3((D + 255) / 256, nb), dim3(256), 0, st, slots, emb, esc, D, x);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_argmax_batch(const float* logits, int nb, int V, float* pval, int* pidx, float* palt,
                               BatchSlot* slots, int tokens_cap, int* toklog, const void* emb, const float* esc, int D,
                               float* x, hipStream_t st) {
    if (nb < 1 || nb > VOX_MAX_BATCH || !slots || !palt || !toklog) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_argmax_rows, dim3(ARGB, nb), dim3(256), 0, st, logits, V, pval, pidx, slots, palt);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_argmax_batch_final, dim3(nb), dim3(256), 0, st, pval, pidx, palt, slots, tokens_cap, toklog,
                       emb, esc, D, x);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_frag_pack(const void* src, int N, int K, int q8, void* dst, hipStream_t st) {
    if (N % 16 || K % 64) return hipErrorInvalidValue;
    const size_t n16 = (size_t)N * K * (q8 ? 1 : 2) / 16;
    const dim3 grid((unsigned)((n16 + 255) / 256));
    if (q8)
        hipLaunchKernelGGL(k_frag_pack<1>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(src), K, n16,
                           static_cast<uint8_t*>(dst));
    else
        hipLaunchKernelGGL(k_frag_pack<0>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(src), K, n16,
                           static_cast<uint8_t*>(dst));
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_rmsnorm_fplanes(float* x, int nb, int D, const float* w, const float* ada, float eps,
                                  uint16_t* xs, const float* part, int S, hipStream_t st, const float* bias) {
    // slabs (S > 0) come from k_skl launches of <= SK_MAX_ROWS rows; plain rows: any row set
    if (nb < 1 || nb > (S > 0 ? SK_MAX_ROWS : PLANE_MAX_ROWS) || D % 64) return hipErrorInvalidValue;
    if (D <= 4 * 512 && D % 4 == 0) {
        hipLaunchKernelGGL(k_resid_rmsnorm_fplanes<4>, dim3(nb), dim3(512), 0, st, x, D, part, S, bias, w, ada, eps, xs);
        LAUNCH_CHECK();
        return hipSuccess;
    }
    if (D <= 8 * 512) {
        hipLaunchKernelGGL(k_resid_rmsnorm_fplanes<8>, dim3(nb), dim3(512), 0, st, x, D, part, S, bias, w, ada, eps, xs);
        LAUNCH_CHECK();
        return hipSuccess;
    }
    if (nb > SK_ROWS) return hipErrorInvalidValue;
    if (S > 0) {
        hipLaunchKernelGGL(k_resid_slabs, dim3((D + 255) / 256, nb), dim3(256), 0, st, x, D, part, S, bias);
        LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_rmsnorm_fplanes, dim3((D / 8 + 63) / 64, nb), dim3(64), 0, st, x, D, w, ada, eps, xs);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_resid_slabs(float* x, int nb, int D, const float* part, int S, const float* bias, hipStream_t st) {
    if (nb < 1 || nb > SK_MAX_ROWS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_resid_slabs, dim3((D + 255) / 256, nb), dim3(256), 0, st, x, D, part, S, bias);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_slabs_rows(const float* part, int S, int nb, int N, const float* bias, float* out, int ldo,
                             hipStream_t st) {
    if (nb < 1 || nb > SK_MAX_ROWS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_slabs_rows, dim3((N + 255) / 256, nb), dim3(256), 0, st, part, S, N, bias, out, ldo);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_split_fplanes(const float* x, int nb, int K, uint16_t* xs, hipStream_t st) {
    if (nb < 1 || nb > PLANE_MAX_ROWS || K % 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_split_fplanes, dim3((K / 8 + 255) / 256, nb), dim3(256), 0, st, x, K, xs);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_swiglu_fplanes(const float* part, int S, int H, int nb, uint16_t* xs, hipStream_t st) {
    if (nb < 1 || nb > SK_MAX_ROWS || H % 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_swiglu_fplanes, dim3((H / 2 + 255) / 256, nb), dim3(256), 0, st, part, S, H, xs);
    LAUNCH_CHECK();
    return hipSuccess;
}

// tuning knobs (tools/kbench; 0 = automatic): k_skf row groups per block, waves per block,
// ring depth; k_skl waves per block
VOX_KB_KNOB(g_skf_r, 0);
VOX_KB_KNOB(g_skf_nw, 0);
VOX_KB_KNOB(g_skf_d, 0);
VOX_KB_KNOB(g_skl_nw, 0);

template <int Q, int R, int NW, int D, int Z = 1>
static hipError_t skf_launch(const uint16_t* xs, int K, const void* W, const float* wscale, int N, int nb,
                             float* C, int ldc, hipStream_t st) {
    hipLaunchKernelGGL((k_skf<Q, R, NW, D, Z>), dim3(N / (16 * R)), dim3(NW * 64), 0, st, xs, K,
                       static_cast<const uint8_t*>(W), wscale, N, nb, C, ldc);
    return hipGetLastError();
}

// the configurations built (1024-thread blocks cap a wave at 128 VGPRs: shallower rings)
#define SKF_CONFIGS(X) \
    X(1, 4, 2) X(1, 8, 2) X(2, 4, 2) X(2, 4, 3) X(2, 8, 2) X(4, 4, 2) X(4, 8, 2)

template <int Q>
static hipError_t skf_cfg(const uint16_t* xs, int K, const void* W, const float* wscale, int N, int nb, float* C,
                          int ldc, hipStream_t st) {
    const int groups = N / 16;
    const int r = g_skf_r ? g_skf_r : (groups >= 2048 ? 4 : groups >= 512 ? 2 : 1);
    if (groups % r) return hipErrorInvalidValue;
    const int nw = g_skf_nw ? g_skf_nw : 4, d = g_skf_d ? g_skf_d : 2;
#define SKF_X(RR, NWW, DD) \
    if (r == RR && nw == NWW && d == DD) return skf_launch<Q, RR, NWW, DD>(xs, K, W, wscale, N, nb, C, ldc, st);
    SKF_CONFIGS(SKF_X)
#undef SKF_X
    return hipErrorInvalidValue;
}

hipError_t launch_gemm_skf(const uint16_t* xs, int K, const void* Wf, const float* wscale, int N, int nb, float* C,
                           int ldc, hipStream_t st) {
    if (nb < 1 || nb > SK_ROWS || N % 64 || K % 64 || !C) return hipErrorInvalidValue;
    return wscale ? skf_cfg<1>(xs, K, Wf, wscale, N, nb, C, ldc, st) : skf_cfg<0>(xs, K, Wf, wscale, N, nb, C, ldc, st);
}

// 17..32 rows (two 16-row blocks of planes, block 1's after block 0's three) in one launch
// reading every weight once: R = 4 row groups per block, 4 waves, 2-deep ring.  tools/kbench
// (profiles/r6_kbench_skf2.txt), the LM head at 32 rows: two 16-row launches 250.0 us, one
// launch at R = 1 / 2 / 4 328.1 / 192.1 / 149.3 us, the same bits
VOX_KB_KNOB(g_skf2_r, 4);
hipError_t launch_gemm_skf2(const uint16_t* xs, int K, const void* Wf, const float* wscale, int N, int nb, float* C,
                            int ldc, hipStream_t st) {
    if (nb <= SK_ROWS || nb > 2 * SK_ROWS || N % 64 || K % 64 || !C) return hipErrorInvalidValue;
    const int r = g_skf2_r;
    if ((N / 16) % r) return hipErrorInvalidValue;
    if (r == 1) return wscale ? skf_launch<1, 1, 4, 2, 2>(xs, K, Wf, wscale, N, nb, C, ldc, st)
                              : skf_launch<0, 1, 4, 2, 2>(xs, K, Wf, wscale, N, nb, C, ldc, st);
    if (r == 4) return wscale ? skf_launch<1, 4, 4, 2, 2>(xs, K, Wf, wscale, N, nb, C, ldc, st)
                              : skf_launch<0, 4, 4, 2, 2>(xs, K, Wf, wscale, N, nb, C, ldc, st);
    return wscale ? skf_launch<1, 2, 4, 2, 2>(xs, K, Wf, wscale, N, nb, C, ldc, st)
                  : skf_launch<0, 2, 4, 2, 2>(xs, K, Wf, wscale, N, nb, C, ldc, st);
}

template <int Q, int NW, int KS>
static hipError_t skl_launch(const uint16_t* xs, int K, const void* W, const float* wscale, int N, int nb,
                             float* part, hipStream_t st, const float* ssq, int nsl, float eps) {
    const int units = (N / (16 * NW)) * (K / (64 * KS));
    const int Z = (nb + SK_ROWS - 1) / SK_ROWS;
    const int grid = Z > 1 ? (units + 7) / 8 * 8 * Z : units;
    if (ssq)
        hipLaunchKernelGGL((k_skl<Q, NW, KS, 1>), dim3(grid), dim3(NW * 64), 0, st, xs, K, static_cast<const uint8_t*>(W),
                           wscale, N, nb, part, ssq, nsl, eps);
    else
        hipLaunchKernelGGL((k_skl<Q, NW, KS, 0>), dim3(grid), dim3(NW * 64), 0, st, xs, K, static_cast<const uint8_t*>(W),
                           wscale, N, nb, part, nullptr, 0, 0.f);
    return hipGetLastError();
}

hipError_t launch_resid_xw_fplanes(float* x, int nb, int D, const float* w, const float* ada, uint16_t* xs,
                                   const float* part, int S, const float* bias, float* ssq, hipStream_t st) {
    if (nb < 1 || nb > SK_MAX_ROWS || D % 256 || D / 256 > SKL_MAX_SLICES || !ssq) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_resid_xw_fplanes, dim3(D / 256, nb), dim3(64), 0, st, x, D, part, S, bias, w, ada, xs, ssq);
    LAUNCH_CHECK();
    return hipSuccess;
}

// waves (row groups) per block of k_skl at S splits, by the 8-wave grid size (N / 128) * S:
// narrow outputs take 8 from 128 blocks (decoder wo 3072 x 4096: 7.8 -> 7.1 us at 16 rows; the
// encoder's wo / w2 at 40 / 100 blocks stay at 4), wide ones from 384 (decoder QKV 6144 x 3072
// at 288: 11.4 -> 10.2 us with 4; encoder W1|W3 at 400 keeps 8)
static int skl_nw_for(int N, int S) {
    const int nb8 = (N / 128) * S;
    int nw = g_skl_nw ? g_skl_nw : (N % 128 == 0 && nb8 >= (N <= 4096 ? 128 : 384) ? 8 : 4);
    if (N % (16 * nw)) nw = 4;
    return nw;
}

// k_skl split count.  K / 512 splits (8 64-k blocks each) by default; with N given, 6-block
// splits on 4 waves where they spread the weight bytes more evenly over the CUs in one
// residency round: the most bytes any CU streams is ceil(blocks / CUs) x the block's bytes
// (decoder QKV 6144 x 3072: 576 blocks of 64 KiB, up to 3 per CU, against 768 of 48 KiB, 3
// per CU -- kbench 10.46 -> 9.26 us at 16 rows, profiles/r4_kbench_skl_sweep.txt; the other
// decoder and encoder shapes keep 8 or have no 6-block split)
int skl_splits(int K, int N) {
    const int KB = K / 64;
    const int S8 = KB % 8 == 0 ? KB / 8 : KB % 4 == 0 ? KB / 4 : 0;
    if (N <= 0 || !S8 || KB % 8 || KB % 6 || N % 64 || g_skl_nw) return S8;
    const int cus = 256;
    const int nw8 = skl_nw_for(N, S8);
    const long long b8 = (long long)(N / (16 * nw8)) * S8, b6 = (long long)(N / 64) * (KB / 6);
    if (b6 > 3LL * cus) return S8;
    const long long c8 = (b8 + cus - 1) / cus * 8 * nw8, c6 = (b6 + cus - 1) / cus * 6 * 4;
    return c6 < c8 ? KB / 6 : S8;
}

template <int Q, int NW, int KS>
static hipError_t skl2_launch(const uint16_t* xs, int K, const void* W, const float* wscale, int N, int nb,
                              float* part, hipStream_t st, const float* ssq, int nsl, float eps) {
    const int grid = (N / (16 * NW)) * (K / (64 * KS));
    if (ssq)
        hipLaunchKernelGGL((k_skl2<Q, NW, KS, 1>), dim3(grid), dim3(NW * 64), 0, st, xs, K, static_cast<const uint8_t*>(W),
                           wscale, N, nb, part, ssq, nsl, eps);
    else
        hipLaunchKernelGGL((k_skl2<Q, NW, KS, 0>), dim3(grid), dim3(NW * 64), 0, st, xs, K, static_cast<const uint8_t*>(W),
                           wscale, N, nb, part, nullptr, 0, 0.f);
    return hipGetLastError();
}

#define SKL2_CONFIGS(X) X(4, 4) X(8, 4) X(4, 6) X(4, 8) X(8, 8)
static hipError_t skl2_cfg(int nw, int ks, const uint16_t* xs, int K, const void* Wf, const float* wscale, int N,
                           int nb, float* part, hipStream_t st, const float* ssq, int nsl, float eps) {
    if (nb <= SK_ROWS || nb > 2 * SK_ROWS || K % 64 || (K / 64) % ks || N % (16 * nw) || (ks * 6) % nw ||
        (ssq && (nsl < 1 || nsl > SKL_MAX_SLICES)))
        return hipErrorInvalidValue;
#define SKL2_X(NWW, KSS)                                                                                      \
    if (nw == NWW && ks == KSS)                                                                               \
        return wscale ? skl2_launch<1, NWW, KSS>(xs, K, Wf, wscale, N, nb, part, st, ssq, nsl, eps)           \
                      : skl2_launch<0, NWW, KSS>(xs, K, Wf, wscale, N, nb, part, st, ssq, nsl, eps);
    SKL2_CONFIGS(SKL2_X)
#undef SKL2_X
    return hipErrorInvalidValue;
}

// tools/kbench: k_skl2 (17..32 rows) at a given waves-per-block / 64-k blocks per split
hipError_t launch_gemm_skl2_cfg(int nw, int ks, const uint16_t* xs, int K, const void* Wf, int N, int nb, float* part,
                                hipStream_t st) {
    return skl2_cfg(nw, ks, xs, K, Wf, nullptr, N, nb, part, st, nullptr, 0, 0.f);
}

hipError_t launch_gemm_skl(const uint16_t* xs, int K, const void* Wf, const float* wscale, int N, int nb,
                           float* part, hipStream_t st, const float* ssq, int nsl, float eps, int pair) {
    const int S = skl_splits(K, N);
    // ssq: each row block's nsl x 16 sums ride with its planes (nsl * 16 <= the block's threads)
    if (nb < 1 || nb > SK_MAX_ROWS || K % 64 || !S || (ssq && (nsl < 1 || nsl > SKL_MAX_SLICES)))
        return hipErrorInvalidValue;
    const int ks = K / 64 / S;
    const int nw = ks == 6 ? 4 : skl_nw_for(N, S);
    if (N % (16 * nw)) return hipErrorInvalidValue;
    // pair (the batched step's 17..32 rows): both row blocks in one k_skl2 block at the same
    // waves and splits -- the same bits, each weight fragment loaded once (QKV 12.7 -> 11.4,
    // wo 9.8 -> 8.7, W2 17.7 -> 16.7 us at 32 rows, profiles/r6_kbench_skl2.txt)
    if (pair && nb > SK_ROWS && nb <= 2 * SK_ROWS) {
        const hipError_t e = skl2_cfg(nw, ks, xs, K, Wf, wscale, N, nb, part, st, ssq, nsl, eps);
        if (e != hipErrorInvalidValue) return e;
    }
#define SKL_X(Q, NWW, KSS) \
    if ((wscale != nullptr) == Q && nw == NWW && ks == KSS) return skl_launch<Q, NWW, KSS>(xs, K, Wf, wscale, N, nb, part, st, ssq, nsl, eps);
    SKL_X(0, 4, 8) SKL_X(0, 8, 8) SKL_X(0, 4, 4) SKL_X(0, 8, 4) SKL_X(0, 4, 6)
    SKL_X(1, 4, 8) SKL_X(1, 8, 8) SKL_X(1, 4, 4) SKL_X(1, 8, 4) SKL_X(1, 4, 6)
#undef SKL_X
    return hipErrorInvalidValue;
}


// tools/kbench: k_skl (bf16, 16 rows) at a given waves-per-block / 64-k blocks per split
hipError_t launch_gemm_skl_cfg(int nw, int ks, const uint16_t* xs, int K, const void* Wf, int N, int nb, float* part,
                               hipStream_t st) {
    if (nb < 1 || nb > SK_ROWS || K % 64 || (K / 64) % ks || N % (16 * nw) || (ks * 6) % nw) return hipErrorInvalidValue;
#define SKC_X(NWW, KSS) \
    if (nw == NWW && ks == KSS) return skl_launch<0, NWW, KSS>(xs, K, Wf, nullptr, N, nb, part, st, nullptr, 0, 0.f);
    SKC_X(4, 4) SKC_X(8, 4) SKC_X(4, 6) SKC_X(4, 8) SKC_X(8, 8) SKC_X(4, 12) SKC_X(8, 12) SKC_X(4, 16) SKC_X(8, 16)
#undef SKC_X
    return hipErrorInvalidValue;
}

static int sklx_nw(int N, int K) {
    // waves per block as launch_gemm_skl picks them at K / 512 splits
    return skl_nw_for(N, skl_splits(K));
}

int sklx_slices(int N, int K) { return N / (16 * sklx_nw(N, K)); }

template <int NW, int KS, int PRO, int EPI>
static hipError_t sklx_launch(const uint16_t* xs, int K, const void* W, int N, int nb, const SklFused& f,
                              hipStream_t st) {
    const int units = (N / (16 * NW)) * (K / (64 * KS));
    const int Z = (nb + SK_ROWS - 1) / SK_ROWS;
    const int grid = Z > 1 ? (units + 7) / 8 * 8 * Z : units;
    hipLaunchKernelGGL((k_sklx<NW, KS, PRO, EPI>), dim3(grid), dim3(NW * 64), 0, st, xs, K,
                       static_cast<const uint8_t*>(W), N, nb, f);
    return hipGetLastError();
}

hipError_t launch_gemm_sklx(int pro, int epi, const uint16_t* xs, int K, const void* Wf, int N, int nb,
                            const SklFused& f, hipStream_t st) {
    const int S = skl_splits(K);
    if (nb < 1 || nb > SK_MAX_ROWS || K % 64 || !S || !f.part || !f.ticket) return hipErrorInvalidValue;
    const int ks = K / 64 / S, nw = sklx_nw(N, K);
    if (N % (16 * nw) || (N / (16 * nw)) * ((nb + SK_ROWS - 1) / SK_ROWS) > SKX_TICKETS) return hipErrorInvalidValue;
    if (!xs || (pro == SKX_PRO_SCALE && (!f.ssq_in || f.nsl < 1 || f.nsl * SK_ROWS > 2 * nw * 64)))
        return hipErrorInvalidValue;
    if (epi == SKX_EPI_RESID && f.planes && !f.nw) return hipErrorInvalidValue;
    if (epi == SKX_EPI_RESID && (!f.x || !f.ssq_out)) return hipErrorInvalidValue;
    if (epi == SKX_EPI_SWIGLU && (!f.planes || N % 64)) return hipErrorInvalidValue;
    if (epi == SKX_EPI_QKV && (!f.q || !f.Kc || !f.Vc || !f.rope || f.hd % 2 || f.qd % f.hd || f.cap < 1 ||
                               N != f.qd + 2 * f.kvd))
        return hipErrorInvalidValue;
#define SKX_X(NWW, KSS, PP, EE) \
    if (nw == NWW && ks == KSS && pro == PP && epi == EE) return sklx_launch<NWW, KSS, PP, EE>(xs, K, Wf, N, nb, f, st);
#define SKX_CFG(PP, EE) SKX_X(4, 4, PP, EE) SKX_X(4, 8, PP, EE) SKX_X(8, 4, PP, EE) SKX_X(8, 8, PP, EE)
    SKX_CFG(SKX_PRO_PLANES, SKX_EPI_QKV)
    SKX_CFG(SKX_PRO_SCALE, SKX_EPI_QKV)
    SKX_CFG(SKX_PRO_PLANES, SKX_EPI_RESID)
    SKX_CFG(SKX_PRO_SCALE, SKX_EPI_SWIGLU)
#undef SKX_CFG
#undef SKX_X
    return hipErrorInvalidValue;
}

hipError_t launch_im2col3(const float* src, int C, int T, int stride, int off, float* A,
                          hipStream_t st) {
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_im2col3, dim3(T), dim3(256), 0, st, src, C, T, stride, off, A);
    LAUNCH_CHECK();
    return hipSuccess;
}

VOX_KB_KNOB(g_mel_fpb, 0);  // tools/kbench knob: frames per k_mel_frames block (0 = by count)
hipError_t launch_mel_frames(const float* samples, long long start0, int nframes, const float* window,
                             const float* dcosT, const float* dsinT, const float* filtT, float log_min, float* mel,
                             hipStream_t st) {
    if (nframes <= 0) return hipSuccess;
    // frames per block: one for a streaming feed (50 frames: 20.4 us against 38.3 with 4, the
    // block's serial DFT sets the time), 4 from 512 frames on (a clip's mel: 3000 frames 109.9
    // -> 43.4 us); tools/kbench VOX_KB_ONLY=mel, profiles/r6_kbench_mel.txt
    const int F = g_mel_fpb ? g_mel_fpb : nframes >= 512 ? 4 : 1;
#define MEL_F(FF)                                                                                              \
    if (F == FF) hipLaunchKernelGGL(k_mel_frames<FF>, dim3((nframes + FF - 1) / FF), dim3(256), 0, st, samples, \
                                    start0, nframes, window, dcosT, dsinT, filtT, log_min, mel);
    MEL_F(1) MEL_F(2) MEL_F(4) MEL_F(8)
#undef MEL_F
    if (F != 1 && F != 2 && F != 4 && F != 8) return hipErrorInvalidValue;
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_mel_reflect(float* buf, long long n, long long real_end, int len, hipStream_t st) {
    hipLaunchKernelGGL(k_mel_reflect, dim3(1), dim3(256), 0, st, buf, n, real_end, len);
    LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_mel_tail(const float* melp, int n_new, int MB, float* tail, hipStream_t st) {
    hipLaunchKernelGGL(k_mel_tail, dim3(1), dim3(128), 0, st, melp, n_new, MB, tail);
    LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace vox
