#include <algorithm>
// kbench.hip -- isolated timing of the decode-step kernels (HIP events, back-to-back
// launches on one stream).  Build: make -C tools; run: tools/kbench [iters]
// Shapes: Voxtral-4B decoder (voxtral.h:37-48).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../voxtral.c_amd/csrc/vox_hip_internal.h"
#include "../voxtral.c_amd/csrc/vox_hip_dev.h"

using namespace vox;
namespace vox { extern int g_skf_r, g_skf_nw, g_skf_d, g_skl_nw, g_gemv_rb, g_attn_lw, g_attn_blocks, g_attn_short, g_gemmf_rb, g_gemmf_minu, g_gemmf_wr, g_gemmf_order, g_mel_fpb, g_skf2_r, g_attn_kvfast, g_attn_bsplit, g_gemv_maxb; }
#ifdef VOX_GEMV_STAMPS
namespace vox { hipError_t gemv_set_stamps(unsigned long long* p); }
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static void* dmalloc(size_t bytes, int fill) {
    void* p;
    CK(hipMalloc(&p, bytes));
    // a small constant bf16 pair (finite as f32 too); values do not matter for timing
    CK(hipMemsetD32(p, fill ? 0x3c003c01u : 0u, bytes / 4));
    return p;
}

template <class F>
static double timeit(F f, int iters, hipStream_t st) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    CK(hipEventRecord(a, st));
    for (int i = 0; i < iters; i++) f();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.0 / iters;
}

// prefetch probe (VOX_KB_ONLY=pf): block h reads the first row group of block h of the GEMV
// that follows (rows as gemv_rows maps them), so that group sits in the L2 of the XCD block h
// of the GEMV will run on
__global__ __launch_bounds__(256) void k_touch_rows(const uint16_t* __restrict__ W, int rowbytes, int rb, int swiglu,
                                                    int* __restrict__ sink) {
    const int h = blockIdx.x;
    unsigned acc = 0;
    for (int i = 0; i < rb; i++) {
        int row;
        if (swiglu) {
            const int u = h * (rb / 2) + (i >> 1);
            row = ((u >> 4) << 5) + (u & 15) + ((i & 1) << 4);
        } else {
            row = h * rb + i;
        }
        const uint4* rp = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(W) + (size_t)row * rowbytes);
        for (int c = threadIdx.x; c < rowbytes / 16; c += 256) {
            const uint4 v = rp[c];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9e3779b9u) sink[0] = (int)acc;
}

// VOX_KB_ONLY=bar: what a launch boundary between dependent weight streams costs.  One decode
// layer's four weight reads (QKV, wo, W1|W3, W2 sizes) as (A) four launches of a plain streaming
// kernel in a graph, (B) one launch whose 768 blocks meet at a grid barrier between the reads
// (a relaxed agent-scope arrival counter, reset by a memset node per replay; 3 blocks per CU,
// all resident), (C) as B with each block's first loads of the next read issued before it
// waits at the barrier.
constexpr int BAR_U = 4;  // 16-B loads per thread in flight per iteration
typedef unsigned int bar_v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 bar_ld(const uint4* p) {
    const bar_v4 t = __builtin_nontemporal_load(reinterpret_cast<const bar_v4*>(p));
    return make_uint4(t.x, t.y, t.z, t.w);
}
struct BarStreams {
    const uint4* w[4];
    size_t n16[4];
};
__device__ __forceinline__ void bar_first(const uint4* W, size_t n16, int b, int G, uint4 (&v)[BAR_U]) {
    const size_t per = (n16 + G - 1) / G, s0 = (size_t)b * per, e = min(n16, s0 + per);
#pragma unroll
    for (int k = 0; k < BAR_U; k++) {
        const size_t i = s0 + threadIdx.x + (size_t)k * 256;
        v[k] = i < e ? bar_ld(W + i) : make_uint4(0, 0, 0, 0);
    }
}
__device__ __forceinline__ unsigned bar_rest(const uint4* W, size_t n16, int b, int G, const uint4 (&v0)[BAR_U]) {
    const size_t per = (n16 + G - 1) / G, s0 = (size_t)b * per, e = min(n16, s0 + per);
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < BAR_U; k++) acc ^= v0[k].x ^ v0[k].y ^ v0[k].z ^ v0[k].w;
    for (size_t i0 = s0 + BAR_U * 256; i0 < e; i0 += BAR_U * 256) {
        uint4 v[BAR_U];
#pragma unroll
        for (int k = 0; k < BAR_U; k++) {
            const size_t i = i0 + threadIdx.x + (size_t)k * 256;
            v[k] = i < e ? bar_ld(W + i) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < BAR_U; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    return acc;
}
__global__ __launch_bounds__(256) void k_bar_one(const uint4* W, size_t n16, int* sink) {
    uint4 v[BAR_U];
    bar_first(W, n16, blockIdx.x, gridDim.x, v);
    const unsigned acc = bar_rest(W, n16, blockIdx.x, gridDim.x, v);
    if (acc == 0x9e3779b9u) sink[0] = (int)acc;
}
// HIER: arrivals counted per XCD group (block b % 8, 64-B apart) and only each group's last
// arrival bumps the global phase counter ctr[0] (8 adds per barrier instead of G)
template <int PF, int HIER = 0>
__global__ __launch_bounds__(256) void k_bar_chain(const BarStreams S, int* ctr, int* sink) {
    const int G = gridDim.x, b = blockIdx.x;
    unsigned acc = 0;
    uint4 v[BAR_U];
    bar_first(S.w[0], S.n16[0], b, G, v);
    for (int j = 0; j < 4; j++) {
        acc ^= bar_rest(S.w[j], S.n16[j], b, G, v);
        if (j == 3) break;
        if (PF) bar_first(S.w[j + 1], S.n16[j + 1], b, G, v);
        __syncthreads();
        if (threadIdx.x == 0) {
            int target = (j + 1) * G;
            if (HIER) {
                const int grp = b & 7, gn = G / 8;  // G % 8 == 0
                if (__hip_atomic_fetch_add(ctr + 16 * (1 + grp), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (j + 1) * gn - 1)
                    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                target = (j + 1) * 8;
            } else {
                __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            long long spins = 0;
            while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++spins < (1 << 22))
                __builtin_amdgcn_s_sleep(1);
            if (spins >= (1 << 22)) sink[1] = 1;  // bounded: a missing block is reported, not waited for
        }
        __syncthreads();
        if (!PF) bar_first(S.w[j + 1], S.n16[j + 1], b, G, v);
    }
    if (acc == 0x9e3779b9u) sink[0] = (int)acc;
}

// VOX_KB_ONLY=gw: a wave-independent decode GEMV prototype (STORE epilogue only).  Each wave
// owns RB whole rows per group (no cross-wave reduction, no per-group block barrier), x sits
// in LDS (one barrier at the start), and the wave's next U rounds of 16-B weight chunks are in
// flight while it computes the current ones (flattened group x round-block steps).
template <int RB, int WQ8, int U>
__global__ __launch_bounds__(256) void k_gemv_wave(const void* __restrict__ W, const float* __restrict__ x, int K, int rows,
                                                   float* __restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) float sx[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rowbytes = WQ8 ? K : 2 * K, NC = rowbytes / 16, NR = (NC + 63) / 64, NB = (NR + U - 1) / U;
    const int WS = gridDim.x * 4, ngroups = rows / RB;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W), 0, rows * rowbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wz = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W), 0, 0, 0x00020000);
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    auto issue = [&](int g, int rb, uint4 (&wv)[U][RB]) {
        const bool ok = g < ngroups;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int c = (rb * U + u) * 64 + lane;
            const int cc = c < NC ? c : 0;
#pragma unroll
            for (int i = 0; i < RB; i++) {
                const v4u v = __builtin_amdgcn_raw_buffer_load_b128(ok ? wr : wz, cc * 16, (ok ? g * RB + i : 0) * rowbytes, 2);
                wv[u][i] = make_uint4(v.x, v.y, v.z, v.w);
            }
        }
    };
    float acc[RB];
#pragma unroll
    for (int i = 0; i < RB; i++) acc[i] = 0.f;
    auto compute = [&](int rb, const uint4 (&wv)[U][RB]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int c = (rb * U + u) * 64 + lane;
            const bool in = c < NC;
            if (WQ8) {
                float4 xv[4];
#pragma unroll
                for (int h = 0; h < 4; h++) xv[h] = in ? reinterpret_cast<const float4*>(sx)[c * 4 + h] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int i = 0; i < RB; i++) acc[i] = dot16q(wv[u][i], xv, acc[i]);
            } else {
                const float4 x0 = in ? reinterpret_cast<const float4*>(sx)[c * 2] : make_float4(0.f, 0.f, 0.f, 0.f);
                const float4 x1 = in ? reinterpret_cast<const float4*>(sx)[c * 2 + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int i = 0; i < RB; i++) acc[i] = dot8(wv[u][i], x0, x1, acc[i]);
            }
        }
    };
    int g = blockIdx.x * 4 + wave, rb = 0;
    uint4 A[U][RB], B[U][RB];
    issue(g, 0, A);
    for (int i = threadIdx.x; i < K / 4; i += 256) reinterpret_cast<float4*>(sx)[i] = reinterpret_cast<const float4*>(x)[i];
    __syncthreads();
    auto step = [&](const uint4 (&cur)[U][RB], uint4 (&nxt)[U][RB]) {
        int gn = g, rn = rb + 1;
        if (rn == NB) { rn = 0; gn += WS; }
        issue(gn, rn, nxt);
        compute(rb, cur);
        if (rb == NB - 1) {
#pragma unroll
            for (int i = 0; i < RB; i++) {
                const float v = wave_sum(acc[i]);
                if (lane == 0) y[g * RB + i] = v;
                acc[i] = 0.f;
            }
        }
        g = gn;
        rb = rn;
    };
    while (g < ngroups) {
        step(A, B);
        if (g >= ngroups) break;
        step(B, A);
    }
}

int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 200;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int D = 3072, DQ = 4096, DKV = 1024, DH = 9216, V = 131072, HD = 128, H = 32, KVH = 8;
    // distinct weight buffers per launch so every launch streams from HBM (26 layers)
    const int NL = 26;
    std::vector<uint16_t*> wqkv(NL), wo(NL), w13(NL), w2(NL);
    for (int l = 0; l < NL; l++) {
        wqkv[l] = (uint16_t*)dmalloc((size_t)(DQ + 2 * DKV) * D * 2, 1);
        wo[l] = (uint16_t*)dmalloc((size_t)D * DQ * 2, 1);
        w13[l] = (uint16_t*)dmalloc((size_t)2 * DH * D * 2, 1);
        w2[l] = (uint16_t*)dmalloc((size_t)D * DH * 2, 1);
    }
    uint16_t* emb = (uint16_t*)dmalloc((size_t)V * D * 2, 1);
    float* x = (float*)dmalloc(DH * 4, 1);
    float* y = (float*)dmalloc(V * 4, 0);
    float* normw = (float*)dmalloc(DH * 4, 1);
    float* ada = (float*)dmalloc(DH * 4, 1);
    const int cap = 8192 + 64;
    float* Kc = (float*)dmalloc((size_t)cap * DKV * 4, 1);
    float* Vc = (float*)dmalloc((size_t)cap * DKV * 4, 1);
    float* rope = (float*)dmalloc((size_t)16384 * HD * 4, 1);
    float* part = (float*)dmalloc((size_t)H * 128 * (HD + 2) * 4 + 4096, 0);  // + arrival counts
    float* pv = (float*)dmalloc(4096 * 4, 0);
    int* pi = (int*)dmalloc(4096 * 4, 0);
    int* state;
    CK(hipMalloc(&state, 16));

    {
        hipDeviceProp_t prop;
        CK(hipGetDeviceProperties(&prop, 0));
        printf("device %s: %d CUs, clock %d MHz, L2 %d KB\n", prop.name, prop.multiProcessorCount, prop.clockRate / 1000, prop.l2CacheSize / 1024);
        struct O { const char* n; int pro, epi, K, rows; int q8; };
        for (O o : {O{"qkv", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, 0}, O{"wo", PRO_NONE, EPI_RESID, DQ, D, 0},
                    O{"w13", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, 0}, O{"w2", PRO_NONE, EPI_RESID, DH, D, 0},
                    O{"lm", PRO_NORM, EPI_LOGITS, D, V, 0}, O{"qkv q8", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, 1},
                    O{"wo q8", PRO_NONE, EPI_RESID, DQ, D, 1}, O{"w13 q8", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, 1},
                    O{"w2 q8", PRO_NONE, EPI_RESID, DH, D, 1}}) {
            GemvArgs a;
            memset(&a, 0, sizeof a);
            a.K = o.K; a.rows = o.rows; a.wscale = o.q8 ? (const float*)1 : nullptr;
            printf("occupancy %-7s %d blocks/CU, grid %d\n", o.n, gemv_occupancy(gemv_kernel(o.pro, o.epi, a)), gemv_grid(o.rows));
        }
    }
    int layer = 0;
    float* wsc = (float*)dmalloc((size_t)V * 4, 1);  // Q8 row scales (any finite values)
    const float* qs = nullptr;  // set: the weight buffers are read as int8 rows
    auto gemv = [&](int pro, int epi, const uint16_t* W, int K, int rows) {
        GemvArgs a;
        memset(&a, 0, sizeof a);
        a.x = x; a.K = K; a.W = W; a.wscale = qs; a.rows = rows; a.norm_w = normw; a.ada = ada; a.eps = 1e-5f;
        a.y = y; a.qd = DQ; a.kvd = DKV; a.hd = HD; a.rope = rope; a.state = state; a.Kc = Kc; a.Vc = Vc;
        a.cap = cap; a.part_val = pv; a.part_idx = pi;
        CK(launch_gemv(pro, epi, a, st));
    };
    struct R { const char* name; double us; double bytes; };
    std::vector<R> res;
    auto add = [&](const char* n, double us, double bytes) {
        res.push_back({n, us, bytes});
        printf("%-34s %9.2f us  %8.1f GB/s\n", n, us, bytes / us / 1e3);
        fflush(stdout);
    };
    const bool only_gemmf = getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "gemmf");
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "mel")) {
        // k_mel_frames: frames per block 1 / 2 / 4 / 8 at a 0.5 s feed (50 frames) and a 30 s
        // clip (3000), outputs compared bit for bit with one frame per block
        const int NS = 500000;
        float* smp = (float*)dmalloc((size_t)NS * 4, 1);
        float* win = (float*)dmalloc(400 * 4, 1);
        float* dc = (float*)dmalloc(400 * 201 * 4, 1);
        float* ds = (float*)dmalloc(400 * 201 * 4, 1);
        float* ft = (float*)dmalloc(201 * 128 * 4, 1);
        float* mo = (float*)dmalloc((size_t)3000 * 128 * 4, 0);
        std::vector<float> r1((size_t)3000 * 128), rx((size_t)3000 * 128);
        for (int nf : {50, 3000})
            for (int F : {1, 2, 4, 8}) {
                g_mel_fpb = F;
                CK(launch_mel_frames(smp, 0, nf, win, dc, ds, ft, -8.0f, mo, st));
                CK(hipStreamSynchronize(st));
                CK(hipMemcpy((F == 1 ? r1 : rx).data(), mo, (size_t)nf * 128 * 4, hipMemcpyDeviceToHost));
                const bool same = F == 1 || !memcmp(r1.data(), rx.data(), (size_t)nf * 128 * 4);
                const double us = timeit([&] { CK(launch_mel_frames(smp, 0, nf, win, dc, ds, ft, -8.0f, mo, st)); }, 50, st);
                printf("mel frames %5d  %d per block  %8.2f us  %s\n", nf, F, us, same ? "same bits" : "BITS DIFFER");
                fflush(stdout);
            }
        g_mel_fpb = 0;
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "gpe")) {
        // where the fused prologue / epilogue cost of the W1|W3 and QKV GEMVs sits: each
        // prologue x epilogue combination of the same weights, bf16 and Q8
        for (int q8 = 0; q8 < 2; q8++) {
            qs = q8 ? wsc : nullptr;
            struct C { const char* n; int pro, epi, K, rows, which; };
            // (the instantiated pairs: NONE with STORE / RESID, NORM with SWIGLU / QKV, NORM_ADA with SWIGLU)
            for (C cc : {C{"w13 none/store", PRO_NONE, EPI_STORE, D, 2 * DH, 2}, C{"w13 norm/swiglu", PRO_NORM, EPI_SWIGLU, D, 2 * DH, 2},
                         C{"w13 norm_ada/swiglu", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, 2},
                         C{"qkv none/store", PRO_NONE, EPI_STORE, D, DQ + 2 * DKV, 0}, C{"qkv none/resid", PRO_NONE, EPI_RESID, D, DQ + 2 * DKV, 0},
                         C{"qkv norm/qkv", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, 0}}) {
                char n[96];
                snprintf(n, sizeof n, "gemv %s%s", cc.n, q8 ? " q8" : "");
                add(n, timeit([&] { gemv(cc.pro, cc.epi, cc.which == 2 ? w13[layer++ % NL] : wqkv[layer++ % NL], cc.K, cc.rows); }, iters, st),
                    (double)cc.rows * cc.K * (q8 ? 1 : 2));
            }
        }
        qs = nullptr;
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "gw")) {
        // the current k_gemv (PRO_NONE / EPI_STORE) against the wave-independent prototype,
        // bf16 and Q8, the four decode shapes, 26 rotating layers; results compared
        float* y2 = (float*)dmalloc(V * 4, 0);
        struct S { const char* n; int K, rows; int which; };
        std::vector<float> h1(2 * DH), h2(2 * DH);
        for (int q8 = 0; q8 < 2; q8++) {
            qs = q8 ? wsc : nullptr;
            for (S sh : {S{"qkv", D, DQ + 2 * DKV, 0}, S{"wo", DQ, D, 1}, S{"w13", D, 2 * DH, 2}, S{"w2", DH, D, 3}}) {
                auto wl = [&](int l) -> const uint16_t* { return sh.which == 0 ? wqkv[l] : sh.which == 1 ? wo[l] : sh.which == 2 ? w13[l] : w2[l]; };
                char n[96];
                const double bytes = (double)sh.rows * sh.K * (q8 ? 1 : 2);
                snprintf(n, sizeof n, "gemv %s%s k_gemv", sh.n, q8 ? " q8" : "");
                add(n, timeit([&] { gemv(PRO_NONE, EPI_STORE, wl(layer++ % NL), sh.K, sh.rows); }, iters, st), bytes);
                gemv(PRO_NONE, EPI_STORE, wl(0), sh.K, sh.rows);
                CK(hipStreamSynchronize(st));
                CK(hipMemcpy(h1.data(), y, sh.rows * 4, hipMemcpyDeviceToHost));
                for (int G : {768, 512}) {
                    for (int v = 0; v < 3; v++) {
                        auto launch = [&](const void* Wp) {
                            const size_t lds = (size_t)sh.K * 4;
                            if (q8) {
                                if (v == 0) hipLaunchKernelGGL((k_gemv_wave<4, 1, 2>), dim3(G), dim3(256), lds, st, Wp, x, sh.K, sh.rows, y2);
                                else if (v == 1) hipLaunchKernelGGL((k_gemv_wave<2, 1, 4>), dim3(G), dim3(256), lds, st, Wp, x, sh.K, sh.rows, y2);
                                else hipLaunchKernelGGL((k_gemv_wave<4, 1, 1>), dim3(G), dim3(256), lds, st, Wp, x, sh.K, sh.rows, y2);
                            } else {
                                if (v == 0) hipLaunchKernelGGL((k_gemv_wave<4, 0, 2>), dim3(G), dim3(256), lds, st, Wp, x, sh.K, sh.rows, y2);
                                else if (v == 1) hipLaunchKernelGGL((k_gemv_wave<2, 0, 4>), dim3(G), dim3(256), lds, st, Wp, x, sh.K, sh.rows, y2);
                                else hipLaunchKernelGGL((k_gemv_wave<4, 0, 1>), dim3(G), dim3(256), lds, st, Wp, x, sh.K, sh.rows, y2);
                            }
                        };
                        static const char* vn[3] = {"RB4 U2", "RB2 U4", "RB4 U1"};
                        snprintf(n, sizeof n, "gemv %s%s wave-indep G=%d %s", sh.n, q8 ? " q8" : "", G, vn[v]);
                        add(n, timeit([&] { launch(wl(layer++ % NL)); }, iters, st), bytes);
                        launch(wl(0));
                        CK(hipStreamSynchronize(st));
                        CK(hipMemcpy(h2.data(), y2, sh.rows * 4, hipMemcpyDeviceToHost));
                        double md = 0, mx = 0;
                        for (int r = 0; r < sh.rows; r++) {
                            md = std::max(md, (double)fabsf(h1[r] - h2[r]));
                            mx = std::max(mx, (double)fabsf(h1[r]));
                        }
                        printf("   max |diff| %.3g of max |y| %.3g\n", md, mx);
                    }
                }
            }
        }
        qs = nullptr;
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "bar")) {
        int* ctr = (int*)dmalloc(16 * 9 * 4, 0);
        int* sink = (int*)dmalloc(64, 0);
        const size_t nb[4] = {(size_t)(DQ + 2 * DKV) * D * 2 / 16, (size_t)D * DQ * 2 / 16, (size_t)2 * DH * D * 2 / 16,
                              (size_t)D * DH * 2 / 16};
        const double bytes = 16.0 * (nb[0] + nb[1] + nb[2] + nb[3]);
        for (int G : {768, 512}) {
            std::vector<hipGraphExec_t> ga(NL), gb(NL), gc(NL), gd(NL);
            for (int l = 0; l < NL; l++) {
                const uint4* w[4] = {(const uint4*)wqkv[l], (const uint4*)wo[l], (const uint4*)w13[l], (const uint4*)w2[l]};
                BarStreams S;
                for (int j = 0; j < 4; j++) { S.w[j] = w[j]; S.n16[j] = nb[j]; }
                for (int v = 0; v < 4; v++) {
                    hipGraph_t g;
                    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
                    if (v == 0) {
                        for (int j = 0; j < 4; j++) hipLaunchKernelGGL(k_bar_one, dim3(G), dim3(256), 0, st, w[j], nb[j], sink);
                    } else {
                        CK(hipMemsetAsync(ctr, 0, 16 * 9 * 4, st));
                        if (v == 1) hipLaunchKernelGGL(k_bar_chain<0>, dim3(G), dim3(256), 0, st, S, ctr, sink);
                        else if (v == 2) hipLaunchKernelGGL(k_bar_chain<1>, dim3(G), dim3(256), 0, st, S, ctr, sink);
                        else hipLaunchKernelGGL((k_bar_chain<1, 1>), dim3(G), dim3(256), 0, st, S, ctr, sink);
                    }
                    CK(hipStreamEndCapture(st, &g));
                    CK(hipGraphInstantiate(v == 0 ? &ga[l] : v == 1 ? &gb[l] : v == 2 ? &gc[l] : &gd[l], g, nullptr, nullptr, 0));
                    CK(hipGraphDestroy(g));
                }
            }
            const char* nm[4] = {"4 launches (graph)", "1 launch, grid barriers", "1 launch, barriers + next loads first",
                                 "1 launch, per-XCD barriers + next loads first"};
            for (int rep = 0; rep < 2; rep++)
                for (int v = 0; v < 4; v++) {
                    std::vector<hipGraphExec_t>& gx = v == 0 ? ga : v == 1 ? gb : v == 2 ? gc : gd;
                    char n[96];
                    snprintf(n, sizeof n, "bar G=%d %s", G, nm[v]);
                    add(n, timeit([&] { CK(hipGraphLaunch(gx[layer++ % NL], st)); }, iters, st), bytes);
                }
            int flag[2];
            CK(hipMemcpy(flag, sink, 8, hipMemcpyDeviceToHost));
            printf("barrier timeouts: %d\n", flag[1]);
        }
        // the Q8 layer's bytes (int8 rows: half of each read) and single reads of each size: the
        // floor a streaming kernel with the decode step's launch structure reaches
        for (int G : {768, 512, 384}) {
            std::vector<hipGraphExec_t> gq(NL);
            for (int l = 0; l < NL; l++) {
                const uint4* w[4] = {(const uint4*)wqkv[l], (const uint4*)wo[l], (const uint4*)w13[l], (const uint4*)w2[l]};
                hipGraph_t g;
                CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
                for (int j = 0; j < 4; j++) hipLaunchKernelGGL(k_bar_one, dim3(G), dim3(256), 0, st, w[j], nb[j] / 2, sink);
                CK(hipStreamEndCapture(st, &g));
                CK(hipGraphInstantiate(&gq[l], g, nullptr, nullptr, 0));
                CK(hipGraphDestroy(g));
            }
            char n[96];
            snprintf(n, sizeof n, "bar G=%d Q8 layer bytes, 4 launches", G);
            add(n, timeit([&] { CK(hipGraphLaunch(gq[layer++ % NL], st)); }, iters, st), bytes / 2);
            const char* rn[4] = {"qkv", "wo", "w13", "w2"};
            for (int q8 = 0; q8 < 2; q8++)
                for (int j = 0; j < 4; j++) {
                    const uint4* w[4] = {(const uint4*)wqkv[0], (const uint4*)wo[0], (const uint4*)w13[0], (const uint4*)w2[0]};
                    std::vector<const uint4*> ws(NL);
                    for (int l = 0; l < NL; l++)
                        ws[l] = j == 0 ? (const uint4*)wqkv[l] : j == 1 ? (const uint4*)wo[l] : j == 2 ? (const uint4*)w13[l] : (const uint4*)w2[l];
                    (void)w;
                    snprintf(n, sizeof n, "bar G=%d one read %s%s", G, rn[j], q8 ? " (Q8 bytes)" : "");
                    const size_t m = q8 ? nb[j] / 2 : nb[j];
                    add(n, timeit([&] { hipLaunchKernelGGL(k_bar_one, dim3(G), dim3(256), 0, st, ws[layer++ % NL], m, sink); }, iters, st),
                        16.0 * m);
                }
        }
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "pf")) {
        // does an L2-hot first row group shorten a decode GEMV?  A: GEMV alone (26 rotating
        // layers, cold); B: touch kernel + GEMV; C: touch kernel alone.  GEMV with a hot first
        // group ~ B - C.
        int* sink = (int*)dmalloc(64, 0);
        struct O { const char* n; int pro, epi, K, rows, rb; std::vector<uint16_t*>* w; };
        for (O o : {O{"qkv", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, 4, &wqkv}, O{"wo", PRO_NONE, EPI_RESID, DQ, D, 2, &wo},
                    O{"w13", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, 4, &w13}, O{"w2", PRO_NONE, EPI_RESID, DH, D, 2, &w2}}) {
            const int G = gemv_grid(o.rows);
            const int sw = o.epi == EPI_SWIGLU;
            char nm[96];
            snprintf(nm, sizeof nm, "pf %-4s A gemv cold", o.n);
            add(nm, timeit([&] { gemv(o.pro, o.epi, (*o.w)[layer++ % NL], o.K, o.rows); }, iters, st), (double)o.rows * o.K * 2);
            snprintf(nm, sizeof nm, "pf %-4s B touch + gemv", o.n);
            add(nm, timeit([&] {
                    const uint16_t* W = (*o.w)[layer++ % NL];
                    hipLaunchKernelGGL(k_touch_rows, dim3(G), dim3(256), 0, st, W, o.K * 2, o.rb, sw, sink);
                    gemv(o.pro, o.epi, W, o.K, o.rows);
                }, iters, st), (double)o.rows * o.K * 2);
            snprintf(nm, sizeof nm, "pf %-4s C touch alone (grid %d)", o.n, G);
            add(nm, timeit([&] {
                    hipLaunchKernelGGL(k_touch_rows, dim3(G), dim3(256), 0, st, (*o.w)[layer++ % NL], o.K * 2, o.rb, sw, sink);
                }, iters, st), (double)G * o.rb * o.K * 2);
        }
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "grid")) {
        // decode GEMV grid cap (blocks of 256 threads): 1024 = 4 per CU (default) and larger
        // grids for the Q8 rows, whose waves keep a third of the bf16 bytes in flight
        struct O { const char* n; int pro, epi, K, rows, q8; std::vector<uint16_t*>* w; };
        for (O o : {O{"qkv", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, 0, &wqkv}, O{"wo", PRO_NONE, EPI_RESID, DQ, D, 0, &wo},
                    O{"w13", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, 0, &w13}, O{"w2", PRO_NONE, EPI_RESID, DH, D, 0, &w2},
                    O{"q8 qkv", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, 1, &wqkv}, O{"q8 wo", PRO_NONE, EPI_RESID, DQ, D, 1, &wo},
                    O{"q8 w13", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, 1, &w13}, O{"q8 w2", PRO_NONE, EPI_RESID, DH, D, 1, &w2}})
            for (int mb : {1024, 1536, 2048, 3072}) {
                g_gemv_maxb = mb;
                qs = o.q8 ? wsc : nullptr;
                char nm[96];
                snprintf(nm, sizeof nm, "gemv %-6s cap %4d (grid %4d)", o.n, mb, gemv_grid(o.rows));
                add(nm, timeit([&] { gemv(o.pro, o.epi, (*o.w)[layer++ % NL], o.K, o.rows); }, iters, st),
                    (double)o.rows * o.K * (o.q8 ? 1 : 2));
            }
        g_gemv_maxb = 0;
        qs = nullptr;
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "q8rb")) {
        // Q8 decode GEMVs: rows per group (2 / 4 / 8) x grid cap: with 16 int8 per 16-B chunk a
        // group keeps half the bf16 bytes in flight, so more rows per group (or more groups per
        // CU) should cover the same HBM latency
        struct O { const char* n; int pro, epi, K, rows; std::vector<uint16_t*>* w; };
        for (O o : {O{"q8 qkv", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, &wqkv}, O{"q8 wo", PRO_NONE, EPI_RESID, DQ, D, &wo},
                    O{"q8 w13", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, &w13}, O{"q8 w2", PRO_NONE, EPI_RESID, DH, D, &w2}})
            for (int rb : {4, 8, 2})
                for (int mb : {1024, 2048}) {
                    if (o.epi == EPI_SWIGLU && rb == 2) continue;
                    g_gemv_rb = rb;
                    g_gemv_maxb = mb;
                    qs = wsc;
                    char nm[96];
                    snprintf(nm, sizeof nm, "gemv %-6s rb %d cap %4d (grid %4d)", o.n, rb, mb, gemv_grid(o.rows));
                    add(nm, timeit([&] { gemv(o.pro, o.epi, (*o.w)[layer++ % NL], o.K, o.rows); }, iters, st),
                        (double)o.rows * o.K);
                }
        g_gemv_rb = 0;
        g_gemv_maxb = 0;
        qs = nullptr;
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "sknb")) {
        // batched decode projections at 16 / 32 / 48 rows (1-3 row blocks; the blocks of one
        // weight slice on one XCD): what a step of more than 16 streams costs per GEMM
        uint16_t* xp = (uint16_t*)dmalloc((size_t)3 * 3 * 16 * 9216 * 2, 1);
        float* part = (float*)dmalloc((size_t)3 * 36 * 16 * 18432 * 4, 0);
        float* Cs = (float*)dmalloc((size_t)48 * 131072 * 4, 0);
        struct S { const char* n; int N, K; uint16_t* const* W; double bytes; };
        const S shapes[] = {S{"qkv 6144x3072", DQ + 2 * DKV, D, wqkv.data(), (DQ + 2.0 * DKV) * D * 2},
                            S{"wo  3072x4096", D, DQ, wo.data(), (double)D * DQ * 2},
                            S{"w13 18432x3072", 2 * DH, D, w13.data(), 2.0 * DH * D * 2},
                            S{"w2  3072x9216", D, DH, w2.data(), (double)D * DH * 2}};
        for (const S& g : shapes)
            for (int nb : {16, 32, 48}) {
                char nm[96];
                snprintf(nm, sizeof nm, "skl %s nb%d", g.n, nb);
                add(nm, timeit([&] { CK(launch_gemm_skl(xp, g.K, g.W[layer++ % NL], nullptr, g.N, nb, part, st)); }, iters, st), g.bytes);
            }
        // k_skl2: both row blocks in one block, every (waves, 64-k blocks per split) built
        for (const S& g : shapes)
            for (int nw : {4, 8})
                for (int ks : {4, 6, 8}) {
                    if ((g.K / 64) % ks || (ks * 6) % nw || g.N % (16 * nw)) continue;
                    char nm[96];
                    snprintf(nm, sizeof nm, "skl2 %s nb32 nw%d ks%d (S %d, %d blocks)", g.n, nw, ks, g.K / 64 / ks,
                             g.N / (16 * nw) * (g.K / 64 / ks));
                    const hipError_t e = launch_gemm_skl2_cfg(nw, ks, xp, g.K, g.W[0], g.N, 32, part, st);
                    if (e != hipSuccess) { (void)hipGetLastError(); continue; }
                    add(nm, timeit([&] { CK(launch_gemm_skl2_cfg(nw, ks, xp, g.K, g.W[layer++ % NL], g.N, 32, part, st)); }, iters, st), g.bytes);
                }
        for (int nb : {16}) {
            char nm[96];
            snprintf(nm, sizeof nm, "skf lm 131072x3072 nb%d", nb);
            add(nm, timeit([&] { CK(launch_gemm_skf(xp, D, emb, nullptr, V, nb, Cs, V, st)); }, iters / 4 + 1, st), (double)V * D * 2);
        }
        // the LM head at 32 rows: two launches (one per 16-row block) against one k_skf<Z = 2>
        // launch (R = 1 / 2 / 4 row groups per block); logits compared bit for bit
        {
            add("skf lm nb32 as 2 launches", timeit([&] {
                    CK(launch_gemm_skf(xp, D, emb, nullptr, V, 16, Cs, V, st));
                    CK(launch_gemm_skf(xp + (size_t)3 * 16 * D, D, emb, nullptr, V, 16, Cs + (size_t)16 * V, V, st));
                }, iters / 4 + 1, st), (double)V * D * 2);
            std::vector<float> l0((size_t)32 * V), l1((size_t)32 * V);
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(l0.data(), Cs, l0.size() * 4, hipMemcpyDeviceToHost));
            for (int r : {1, 2, 4}) {
                g_skf2_r = r;
                CK(launch_gemm_skf2(xp, D, emb, nullptr, V, 32, Cs, V, st));
                CK(hipStreamSynchronize(st));
                CK(hipMemcpy(l1.data(), Cs, l1.size() * 4, hipMemcpyDeviceToHost));
                char nm[96];
                snprintf(nm, sizeof nm, "skf2 lm nb32 R%d (%s)", r, memcmp(l0.data(), l1.data(), l0.size() * 4) ? "BITS DIFFER" : "same bits");
                add(nm, timeit([&] { CK(launch_gemm_skf2(xp, D, emb, nullptr, V, 32, Cs, V, st)); }, iters / 4 + 1, st), (double)V * D * 2);
            }
            g_skf2_r = 4;
        }
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "sklks")) {
        // batched decode projections at 16 rows: k_skl waves per block x 64-k blocks per split
        uint16_t* xp = (uint16_t*)dmalloc((size_t)3 * 16 * 9216 * 2, 1);
        float* part = (float*)dmalloc((size_t)36 * 16 * 18432 * 4, 0);
        struct S { const char* n; int N, K; uint16_t* const* W; double bytes; };
        const S shapes[] = {S{"qkv 6144x3072", DQ + 2 * DKV, D, wqkv.data(), (DQ + 2.0 * DKV) * D * 2},
                            S{"wo  3072x4096", D, DQ, wo.data(), (double)D * DQ * 2},
                            S{"w13 18432x3072", 2 * DH, D, w13.data(), 2.0 * DH * D * 2},
                            S{"w2  3072x9216", D, DH, w2.data(), (double)D * DH * 2}};
        for (const S& g : shapes)
            for (int nw : {4, 8})
                for (int ks : {4, 6, 8, 12, 16}) {
                    if ((g.K / 64) % ks || (ks * 6) % nw || g.N % (16 * nw)) continue;
                    char nm[96];
                    snprintf(nm, sizeof nm, "skl %s nw%d ks%d (S %d, %d blocks)", g.n, nw, ks, g.K / 64 / ks,
                             g.N / (16 * nw) * (g.K / 64 / ks));
                    add(nm, timeit([&] { CK(launch_gemm_skl_cfg(nw, ks, xp, g.K, g.W[layer++ % NL], g.N, 16, part, st)); }, iters, st), g.bytes);
                }
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "skb")) {
        // batched decode projections at 16 rows: split-K k_skl (slabs, a row kernel sums them)
        // against whole-K k_skf (final rows: the row kernel's slab sum could go)
        uint16_t* xp = (uint16_t*)dmalloc((size_t)2 * 3 * 16 * 9216 * 2, 1);
        float* Cs = (float*)dmalloc((size_t)16 * 131072 * 4, 0);
        float* part = (float*)dmalloc((size_t)2 * 16 * 18 * 18432 * 4, 0);
        int* sinkb = (int*)dmalloc(64, 0);
        struct S { const char* n; int N, K; uint16_t* const* W; double bytes; };
        const S shapes[] = {S{"qkv 6144x3072", DQ + 2 * DKV, D, wqkv.data(), (DQ + 2.0 * DKV) * D * 2},
                            S{"wo  3072x4096", D, DQ, wo.data(), (double)D * DQ * 2},
                            S{"w13 18432x3072", 2 * DH, D, w13.data(), 2.0 * DH * D * 2},
                            S{"w2  3072x9216", D, DH, w2.data(), (double)D * DH * 2}};
        for (const S& g : shapes) {
            char nm[96];
            snprintf(nm, sizeof nm, "skl %s nb16", g.n);
            add(nm, timeit([&] { CK(launch_gemm_skl(xp, g.K, g.W[layer++ % NL], nullptr, g.N, 16, part, st)); }, iters, st), g.bytes);
            // the same buffer every launch: the weights come from the Infinity Cache (MALL)
            snprintf(nm, sizeof nm, "skl %s nb16 MALL-hot", g.n);
            add(nm, timeit([&] { CK(launch_gemm_skl(xp, g.K, g.W[0], nullptr, g.N, 16, part, st)); }, iters, st), g.bytes);
            // a touch kernel warms the first F bytes (default policy) just before the GEMM:
            // B - C is the GEMM with a warm head
            for (int mb : {16, 32}) {
                const size_t F = std::min((size_t)mb << 20, (size_t)g.bytes);
                const int G = (int)(F / (256 * 16 * 4));
                snprintf(nm, sizeof nm, "skl %s B touch %d MB + gemm", g.n, mb);
                add(nm, timeit([&] {
                        const uint16_t* W = g.W[layer++ % NL];
                        hipLaunchKernelGGL(k_touch_rows, dim3(G), dim3(256), 0, st, W, 256 * 16 * 4, 1, 0, sinkb);
                        CK(launch_gemm_skl(xp, g.K, W, nullptr, g.N, 16, part, st));
                    }, iters, st), g.bytes);
                snprintf(nm, sizeof nm, "skl %s C touch %d MB alone", g.n, mb);
                add(nm, timeit([&] {
                        hipLaunchKernelGGL(k_touch_rows, dim3(G), dim3(256), 0, st, g.W[layer++ % NL], 256 * 16 * 4, 1, 0, sinkb);
                    }, iters, st), (double)F);
            }
            const int Rs[] = {1, 1, 2, 2, 2, 4, 4}, NWs[] = {4, 8, 4, 4, 8, 4, 8}, Ds[] = {2, 2, 2, 3, 2, 2, 2};
            for (int c = 0; c < 7; c++) {
                if ((g.N / 16) % Rs[c]) continue;
                g_skf_r = Rs[c];
                g_skf_nw = NWs[c];
                g_skf_d = Ds[c];
                snprintf(nm, sizeof nm, "skf %s R%d NW%d D%d (%d blocks)", g.n, Rs[c], NWs[c], Ds[c], g.N / 16 / Rs[c]);
                add(nm, timeit([&] { CK(launch_gemm_skf(xp, g.K, g.W[layer++ % NL], nullptr, g.N, 16, Cs, g.N, st)); }, iters, st), g.bytes);
            }
            g_skf_r = g_skf_nw = g_skf_d = 0;
        }
        // the rows between the projections: one 512-thread block per row vs one wave per
        // (256-column slice, row)
        float* xr = (float*)dmalloc((size_t)16 * 9216 * 4, 1);
        float* ssq = (float*)dmalloc(16 * 16 * 4, 0);
        for (int S : {8, 18}) {
            char nm[96];
            snprintf(nm, sizeof nm, "resid(%d)+rmsnorm fplanes 16x3072", S);
            add(nm, timeit([&] { CK(launch_rmsnorm_fplanes(xr, 16, D, xr, xr, 1e-5f, xp, part, S, st)); }, iters, st), 16.0 * D * (10 + 4 * S));
            snprintf(nm, sizeof nm, "resid(%d)+xw fplanes 16x3072 (12 slices)", S);
            add(nm, timeit([&] { CK(launch_resid_xw_fplanes(xr, 16, D, xr, xr, xp, part, S, nullptr, ssq, st)); }, iters, st), 16.0 * D * (10 + 4 * S));
        }
        for (const S& g : {shapes[0], shapes[2]}) {
            char nm[96];
            snprintf(nm, sizeof nm, "skl %s nb16 + rms scale", g.n);
            add(nm, timeit([&] { CK(launch_gemm_skl(xp, g.K, g.W[layer++ % NL], nullptr, g.N, 16, part, st, ssq, 12, 1e-5f)); }, iters, st), g.bytes);
        }
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "attb")) {
        // batched fused decode attention (QKV slabs in, wo planes out) at 16 / 8 streams:
        // each stream its own ring (26 layers rotated so K/V come from HBM)
        const int rcap = 8192 + 64, NLd = 26, S6 = 6, N = DQ + 2 * DKV;
        float* slabs = (float*)dmalloc((size_t)S6 * 16 * N * 4, 1);
        uint16_t* xs = (uint16_t*)dmalloc((size_t)3 * 16 * DQ * 2, 0);
        std::vector<float*> Ks(16 * 2), Vs(16 * 2);
        for (int i = 0; i < 16 * 2; i++) {
            Ks[i] = (float*)dmalloc((size_t)rcap * DKV * 4 * 13, 1);  // 13 layers per buffer
            Vs[i] = (float*)dmalloc((size_t)rcap * DKV * 4 * 13, 1);
        }
        int* states = nullptr;
        CK(hipMalloc(&states, 16 * 16));
        float* parts = (float*)dmalloc((size_t)16 * (H * 128 * (HD + 2) * 4 + 4096), 0);
        BatchSlot* slots = nullptr;
        CK(hipMalloc(&slots, sizeof(BatchSlot) * 16));
        for (int nb : {16, 8})
            for (int L : {64, 128, 190, 256, 512, 1024}) {
                std::vector<int> hs(16 * 4, 0);
                for (int z = 0; z < 16; z++) hs[z * 4] = L - 1;
                CK(hipMemcpy(states, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
                const int need = (L + 255) / 256;
                int splits = 1;
                while (splits < need) splits *= 2;
                {
                    // the engine's form since round 4: rings, position and liveness from the slot
                    // table (layer base + ring_off), the graph's arguments independent of streams
                    std::vector<BatchSlot> hsl(16);
                    memset(hsl.data(), 0, sizeof(BatchSlot) * 16);
                    int l = 0;
                    char nm[96];
                    snprintf(nm, sizeof nm, "attn batch slots nb=%d L=%d splits=%d", nb, L, splits);
                    for (int z = 0; z < 16; z++) {
                        hsl[z].state = states + z * 4;
                        hsl[z].Kc = reinterpret_cast<char*>(Ks[z * 2]);
                        hsl[z].Vc = reinterpret_cast<char*>(Vs[z * 2]);
                        hsl[z].live = z < nb;
                        hsl[z].pos = L - 1;
                    }
                    CK(hipMemcpy(slots, hsl.data(), sizeof(BatchSlot) * 16, hipMemcpyHostToDevice));
                    add(nm, timeit([&] {
                            const int lay = l % 13;  // 13 layers' rings per stream (cold K/V)
                            AttnPtrs p;
                            memset(&p, 0, sizeof p);
                            p.slots = slots;
                            p.ring_off = (size_t)lay * rcap * DKV * 4;
                            for (int z = 0; z < nb; z++) p.part[z] = parts + (size_t)z * (H * 128 * (HD + 2) + 1024);
                            AttnFuse f{slabs, S6, N, rope, xs};
                            CK(launch_attn_batch_fused(HD, p, f, nb, rcap, 8192, 0.088f, H, KVH, splits, st, 0));
                            l++;
                        }, iters, st), (double)nb * L * DKV * 2 * 4);
                }
                if (L > 256) continue;
                for (int bs : {0, 1}) {
                    g_attn_bsplit = bs;
                    int l = 0;
                    char nm[96];
                    snprintf(nm, sizeof nm, "attn batch fused nb=%d L=%d bsplit=%d", nb, L, bs);
                    add(nm, timeit([&] {
                            AttnPtrs p;
                            memset(&p, 0, sizeof p);
                            const int lay = l % NLd;
                            for (int z = 0; z < nb; z++) {
                                p.q[z] = nullptr;
                                p.Kc[z] = Ks[z * 2 + lay / 13] + (size_t)(lay % 13) * rcap * DKV;
                                p.Vc[z] = Vs[z * 2 + lay / 13] + (size_t)(lay % 13) * rcap * DKV;
                                p.state[z] = states + z * 4;
                                p.part[z] = parts + (size_t)z * (H * 128 * (HD + 2) + 1024);
                                p.out[z] = nullptr;
                            }
                            AttnFuse f{slabs, S6, N, rope, xs};
                            CK(launch_attn_batch_fused(HD, p, f, nb, rcap, 8192, 0.088f, H, KVH, 1, st, 0));
                            l++;
                        }, iters, st), (double)nb * L * DKV * 2 * 4);
                }
                {
                    // the same attention without the fused prologue / epilogue (q rows in, rows out)
                    int l = 0;
                    char nm[96];
                    snprintf(nm, sizeof nm, "attn batch plain nb=%d L=%d", nb, L);
                    add(nm, timeit([&] {
                            AttnPtrs p;
                            memset(&p, 0, sizeof p);
                            const int lay = l % NLd;
                            for (int z = 0; z < nb; z++) {
                                p.q[z] = slabs + (size_t)z * DQ;
                                p.Kc[z] = Ks[z * 2 + lay / 13] + (size_t)(lay % 13) * rcap * DKV;
                                p.Vc[z] = Vs[z * 2 + lay / 13] + (size_t)(lay % 13) * rcap * DKV;
                                p.state[z] = states + z * 4;
                                p.part[z] = parts + (size_t)z * (H * 128 * (HD + 2) + 1024);
                                p.out[z] = reinterpret_cast<float*>(xs) + (size_t)z * DQ / 2;
                            }
                            CK(launch_attn_decode_batch(HD, p, nb, rcap, 8192, 0.088f, H, KVH, 1, st, 0));
                            l++;
                        }, iters, st), (double)nb * L * DKV * 2 * 4);
                }
            }
        g_attn_bsplit = -1;
        // phase stamps of the slot-table fused attention (16 streams, 128-key blocks of 8
        // waves): per-wave s_memtime deltas, averaged; the merging block's merge apart
        {
            unsigned long long* stamps = nullptr;
            const int nbs = 16, nblk = 2 * KVH * nbs, nwv = 8;
            CK(hipMalloc(&stamps, (size_t)nblk * nwv * 10 * 8));
            std::vector<BatchSlot> hsl(16);
            for (int L : {64, 128, 190, 256}) {
                memset(hsl.data(), 0, sizeof(BatchSlot) * 16);
                for (int z = 0; z < 16; z++) {
                    hsl[z].state = states + z * 4;
                    hsl[z].Kc = reinterpret_cast<char*>(Ks[z * 2]);
                    hsl[z].Vc = reinterpret_cast<char*>(Vs[z * 2]);
                    hsl[z].live = 1;
                    hsl[z].pos = L - 1;
                }
                CK(hipMemcpy(slots, hsl.data(), sizeof(BatchSlot) * 16, hipMemcpyHostToDevice));
                double acc[8] = {0}, cyc = 0, rt = 0, gstart = 0, gend = 0, n = 0;
                const int nrun = 20;
                for (int r = 0; r < nrun; r++) {
                    AttnPtrs p;
                    memset(&p, 0, sizeof p);
                    p.slots = slots;
                    p.ring_off = (size_t)(r % 13) * rcap * DKV * 4;
                    for (int z = 0; z < nbs; z++) p.part[z] = parts + (size_t)z * (H * 128 * (HD + 2) + 1024);
                    p.out[0] = reinterpret_cast<float*>(stamps);
                    CK(hipMemset(stamps, 0, (size_t)nblk * nwv * 10 * 8));
                    AttnFuse f{slabs, S6, N, rope, xs};
                    CK(launch_attn_batch_dbg(p, f, nbs, rcap, 8192, 0.088f, H, KVH, 1, st));
                    CK(hipStreamSynchronize(st));
                    std::vector<unsigned long long> h((size_t)nblk * nwv * 10);
                    CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
                    unsigned long long g0 = ~0ull, g1 = 0, e1 = 0;
                    for (int b = 0; b < nblk; b++) {
                        const unsigned long long* t0 = &h[(size_t)b * nwv * 10];
                        if (!t0[8]) continue;  // a block with no keys left before its stamps
                        for (int w = 0; w < nwv; w++) {
                            const unsigned long long* t = &h[((size_t)b * nwv + w) * 10];
                            acc[0] += t[6] - t[0];
                            acc[1] += t[7] - t[6];
                            acc[2] += t[1] - t[7];
                            acc[3] += t[2] - t[1];
                            acc[4] += t[3] - t[2];
                            acc[5] += t[4] - t[3];
                            acc[6] += t[5] - t[4];
                            cyc += t[5] - t[0];
                            rt += t[9] - t[8];
                            n += 1;
                            g0 = std::min(g0, t[8]);
                            g1 = std::max(g1, t[8]);
                            e1 = std::max(e1, t[9]);
                        }
                    }
                    gstart += g1 - g0;
                    gend += e1 - g0;
                }
                printf("attn batch stamps nb=16 L=%d per-wave cycles: issue %.0f | loads land %.0f | barrier+new key %.0f | "
                       "QK/sm/PV %.0f | sO+sync %.0f | factors %.0f | out / partial+ticket(+merge) %.0f ; total %.0f cyc = "
                       "%.2f us; block starts spread %.2f us; first start to last end %.2f us\n",
                       L, acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n, acc[6] / n, cyc / n,
                       rt / n / 100.0, gstart / nrun / 100.0, gend / nrun / 100.0);
            }
            CK(hipFree(stamps));
        }
        return 0;
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "attn")) {
        // long-context decode attention as the decode step sees it: 26 layers' rings (f32:
        // 1.76 GB, half: 0.88 GB, far past the 256 MB MALL), one launch per layer in turn
        const int NLd = 26, rcap = 8192 + 64;
        for (int kv16 : {0, 1}) {
            const size_t esz = kv16 ? 2 : 4, per = (size_t)rcap * DKV;
            std::vector<float*> Ks(NLd), Vs(NLd);
            for (int l = 0; l < NLd; l++) {
                Ks[l] = (float*)dmalloc(per * esz, 1);
                Vs[l] = (float*)dmalloc(per * esz, 1);
            }
            for (int L : {1024, 2048, 4096, 8192}) {
                int st4[4] = {L - 1, 0, 0, 0};
                CK(hipMemcpy(state, st4, 16, hipMemcpyHostToDevice));
                int splits = 1;
                while (splits * ATT_BLOCK_KEYS < L) splits *= 2;
                for (int v : {0, 1, 16}) {
                    // v: 0 = key-range-major grid, 1 = kv heads of a key range adjacent (default),
                    // 16 = the same with 256-key blocks of 16 waves
                    g_attn_kvfast = v != 0;
                    g_attn_lw = v == 16 ? 16 : 0;
                    int l = 0;
                    char nm[96];
                    snprintf(nm, sizeof nm, "attn decode L=%d %s 26 layers %d-key blocks%s", L, kv16 ? "half" : "f32",
                             v == 16 ? 256 : 128, g_attn_kvfast ? " kv-fast" : "");
                    add(nm, timeit([&] {
                            CK(launch_attn_decode(HD, x, Ks[l % NLd], Vs[l % NLd], rcap, state, 0, 8192, 0.088f, H, KVH,
                                                  part, y, splits, st, kv16));
                            l++;
                        }, 260, st), (double)L * DKV * 2 * esz);
                }
                g_attn_lw = 0;
                g_attn_kvfast = 1;
            }
            for (int l = 0; l < NLd; l++) {
                CK(hipFree(Ks[l]));
                CK(hipFree(Vs[l]));
            }
        }
        return 0;
    }
    if (!only_gemmf) {
    add("gemv qkv  (6144x3072, norm+rope)", timeit([&] { gemv(PRO_NORM, EPI_QKV, wqkv[layer++ % NL], D, DQ + 2 * DKV); }, iters, st), (DQ + 2.0 * DKV) * D * 2);
    add("gemv wo   (3072x4096, resid)", timeit([&] { gemv(PRO_NONE, EPI_RESID, wo[layer++ % NL], DQ, D); }, iters, st), (double)D * DQ * 2);
    add("gemv w13  (18432x3072, norm+swiglu)", timeit([&] { gemv(PRO_NORM_ADA, EPI_SWIGLU, w13[layer++ % NL], D, 2 * DH); }, iters, st), 2.0 * DH * D * 2);
    add("gemv w2   (3072x9216, resid)", timeit([&] { gemv(PRO_NONE, EPI_RESID, w2[layer++ % NL], DH, D); }, iters, st), (double)D * DH * 2);
    g_gemv_rb = 4;
    add("gemv qkv RB4 (grid 768, 2 groups)", timeit([&] { gemv(PRO_NORM, EPI_QKV, wqkv[layer++ % NL], D, DQ + 2 * DKV); }, iters, st), (DQ + 2.0 * DKV) * D * 2);
    add("gemv w13 RB4", timeit([&] { gemv(PRO_NORM_ADA, EPI_SWIGLU, w13[layer++ % NL], D, 2 * DH); }, iters, st), 2.0 * DH * D * 2);
    g_gemv_rb = 2;
    add("gemv wo RB2 (1536 groups)", timeit([&] { gemv(PRO_NONE, EPI_RESID, wo[layer++ % NL], DQ, D); }, iters, st), (double)D * DQ * 2);
    add("gemv w2 RB2 (1536 groups)", timeit([&] { gemv(PRO_NONE, EPI_RESID, w2[layer++ % NL], DH, D); }, iters, st), (double)D * DH * 2);
    add("gemv qkv RB2", timeit([&] { gemv(PRO_NORM, EPI_QKV, wqkv[layer++ % NL], D, DQ + 2 * DKV); }, iters, st), (DQ + 2.0 * DKV) * D * 2);
    g_gemv_rb = 4;
    add("gemv lm RB4", timeit([&] { gemv(PRO_NORM, EPI_LOGITS, emb, D, V); }, iters / 10 + 1, st), (double)V * D * 2);
    qs = wsc;
    add("q8 gemv qkv RB4", timeit([&] { gemv(PRO_NORM, EPI_QKV, wqkv[layer++ % NL], D, DQ + 2 * DKV); }, iters, st), (DQ + 2.0 * DKV) * D);
    add("q8 gemv w13 RB4", timeit([&] { gemv(PRO_NORM_ADA, EPI_SWIGLU, w13[layer++ % NL], D, 2 * DH); }, iters, st), 2.0 * DH * D);
    g_gemv_rb = 2;
    add("q8 gemv wo RB2", timeit([&] { gemv(PRO_NONE, EPI_RESID, wo[layer++ % NL], DQ, D); }, iters, st), (double)D * DQ);
    add("q8 gemv w2 RB2", timeit([&] { gemv(PRO_NONE, EPI_RESID, w2[layer++ % NL], DH, D); }, iters, st), (double)D * DH);
    g_gemv_rb = 8;
    add("q8 gemv qkv RB8", timeit([&] { gemv(PRO_NORM, EPI_QKV, wqkv[layer++ % NL], D, DQ + 2 * DKV); }, iters, st), (DQ + 2.0 * DKV) * D);
    add("q8 gemv w13 RB8", timeit([&] { gemv(PRO_NORM_ADA, EPI_SWIGLU, w13[layer++ % NL], D, 2 * DH); }, iters, st), 2.0 * DH * D);
    add("q8 gemv lm RB8", timeit([&] { gemv(PRO_NORM, EPI_LOGITS, emb, D, V); }, iters / 10 + 1, st), (double)V * D);
    g_gemv_rb = 4;
    add("q8 gemv wo RB4", timeit([&] { gemv(PRO_NONE, EPI_RESID, wo[layer++ % NL], DQ, D); }, iters, st), (double)D * DQ);
    add("q8 gemv w2 RB4", timeit([&] { gemv(PRO_NONE, EPI_RESID, w2[layer++ % NL], DH, D); }, iters, st), (double)D * DH);
    qs = nullptr;
    g_gemv_rb = 0;
    add("gemv w13 same buffer (MALL-hot)", timeit([&] { gemv(PRO_NORM_ADA, EPI_SWIGLU, w13[0], D, 2 * DH); }, iters, st), 2.0 * DH * D * 2);
    add("gemv wo same buffer (MALL-hot)", timeit([&] { gemv(PRO_NONE, EPI_RESID, wo[0], DQ, D); }, iters, st), (double)D * DQ * 2);
    add("gemv lm   (131072x3072, logits)", timeit([&] { gemv(PRO_NORM, EPI_LOGITS, emb, D, V); }, iters / 10 + 1, st), (double)V * D * 2);
    qs = wsc;
    add("q8 gemv qkv  (6144x3072)", timeit([&] { gemv(PRO_NORM, EPI_QKV, wqkv[layer++ % NL], D, DQ + 2 * DKV); }, iters, st), (DQ + 2.0 * DKV) * D);
    add("q8 gemv wo   (3072x4096)", timeit([&] { gemv(PRO_NONE, EPI_RESID, wo[layer++ % NL], DQ, D); }, iters, st), (double)D * DQ);
    add("q8 gemv w13  (18432x3072)", timeit([&] { gemv(PRO_NORM_ADA, EPI_SWIGLU, w13[layer++ % NL], D, 2 * DH); }, iters, st), 2.0 * DH * D);
    add("q8 gemv w2   (3072x9216)", timeit([&] { gemv(PRO_NONE, EPI_RESID, w2[layer++ % NL], DH, D); }, iters, st), (double)D * DH);
    add("q8 gemv lm   (131072x3072)", timeit([&] { gemv(PRO_NORM, EPI_LOGITS, emb, D, V); }, iters / 10 + 1, st), (double)V * D);
    qs = nullptr;
    }
    if (!only_gemmf)
    {
        // M>1 GEMMs of the encoder / prefill (useful TFLOP/s = 2 M N K / t)
        float* ws = (float*)dmalloc((size_t)8 << 22, 0);
        float* Am = (float*)dmalloc((size_t)1024 * 9216 * 4, 1);
        float* Cm = (float*)dmalloc((size_t)1024 * 131072 * 4, 0);
        struct G { const char* n; int epi, M, N, K; const uint16_t* W; };
        for (G g : {G{"b8  qkv  8x6144x3072", EPI_STORE, 8, 6144, 3072, wqkv[3]},
                    G{"b8  wo   8x3072x4096", EPI_RESID, 8, 3072, 4096, wo[3]},
                    G{"b8  w13  8x18432x3072", EPI_SWIGLU, 8, 18432, 3072, w13[3]},
                    G{"b8  w2   8x3072x9216", EPI_RESID, 8, 3072, 9216, w2[3]},
                    G{"b8  lm   8x131072x3072", EPI_STORE, 8, 131072, 3072, emb},
                    G{"enc qkv  677x6144x1280", EPI_STORE, 677, 6144, 1280, wqkv[1]},
                    G{"enc w13  677x10240x1280", EPI_SWIGLU, 677, 10240, 1280, w13[1]},
                    G{"enc wo   677x1280x2048", EPI_RESID, 677, 1280, 2048, wo[1]},
                    G{"enc w2   677x1280x5120", EPI_RESID, 677, 1280, 5120, w2[1]},
                    G{"pre w2   38x3072x9216", EPI_RESID, 38, 3072, 9216, w2[2]},
                    G{"pre w13  38x18432x3072", EPI_SWIGLU, 38, 18432, 3072, w13[2]}}) {
            const int ldc = g.epi == EPI_SWIGLU ? g.N / 2 : g.N;
            double us = timeit([&] { CK(launch_gemm(g.epi, 3, Am, g.K, g.W, nullptr, g.K, g.M, g.N, nullptr, Cm, ldc, st, ws, (size_t)8 << 20)); }, 20, st);
            char nm[80];
            snprintf(nm, sizeof nm, "gemm %s", g.n);
            printf("%-34s %9.2f us  %8.1f TFLOP/s (useful)\n", nm, us, 2.0 * g.M * g.N * g.K / us / 1e6);
        }
    }
    {
        // k_gemmf (stream-K, planes x fragment-major weights) at the encoder's shapes
        const size_t wsn = 2 * gemmf_ws_floats(gemmf_grid());
        float* gws = (float*)dmalloc(wsn * 4, 0);
        int* gfl = (int*)dmalloc(gemmf_flag_ints() * 4, 0);
        uint16_t* gp = (uint16_t*)dmalloc((size_t)64 * 3 * 16 * 9216 * 2, 1);
        uint16_t* go = (uint16_t*)dmalloc((size_t)64 * 3 * 16 * 9216 * 2, 0);
        float* gc = (float*)dmalloc((size_t)1024 * 18432 * 4, 0);
        int epoch = 0;
        struct G { const char* n; int epi, N, K; const uint16_t* W; };
        for (int M : {256, 400, 512, 677, 1024})
            for (G g : {G{"qkv", EPI_STORE, 6144, 1280, wqkv[1]}, G{"w13", EPI_SWIGLU, 10240, 1280, w13[1]},
                        G{"wo", EPI_RESID, 1280, 2048, wo[1]}, G{"w2", EPI_RESID, 1280, 5120, w2[1]},
                        G{"dqkv", EPI_STORE, 6144, 3072, wqkv[3]}, G{"dw13", EPI_SWIGLU, 18432, 3072, w13[3]}}) {
                if (g.n[0] == 'd' && M != 400 && M != 677) continue;
                for (int v = 0; v < 6; v++) {
                    // np3 (RB4): unit order by shape / column-major / row-major, twice (XCD-grouped
                    // tiles: profiles/r5_kbench_gemmf_xcdgrp.txt);
                    // earlier: profiles/r4_kbench_gemmf*.txt, r5_kbench_gemmf_order*.txt
                    const int np = 3;
                    g_gemmf_order = v % 3;
                    double us = timeit([&] { CK(launch_gemmf(g.epi, np, gp, g.K, M, g.W, g.N, nullptr, gc, g.epi == EPI_SWIGLU ? g.N / 2 : g.N,
                                                             g.epi == EPI_SWIGLU ? go : nullptr, gws, wsn, gfl, ++epoch, st)); }, 20, st);
                    static const char* on[3] = {"auto", "col", "row"};
                    printf("gemmf %-4s M=%4d %dx%d np%d %-6s %9.2f us  %8.1f TFLOP/s (useful)  %6.1f%% of bf16 peak (issued)\n", g.n, M, g.N,
                           g.K, np, on[v % 3], us, 2.0 * M * g.N * g.K / us / 1e6, 100.0 * np * 2.0 * M * g.N * g.K / us / 1e6 / 2500.0);
                    fflush(stdout);
                }
                g_gemmf_order = 0;  // by shape
            }
    }
    if (getenv("VOX_KB_ONLY") && !strcmp(getenv("VOX_KB_ONLY"), "gemmfm")) {
        // k_gemmf at small M (streaming chunks, prefills, the one-shot flush chunk): least
        // stages per block (minu) = half a tile (default) / a quarter / an eighth / 4
        const size_t wsn = 2 * gemmf_ws_floats(gemmf_grid());
        float* gws = (float*)dmalloc(wsn * 4, 0);
        int* gfl = (int*)dmalloc(gemmf_flag_ints() * 4, 0);
        uint16_t* gp = (uint16_t*)dmalloc((size_t)64 * 3 * 16 * 9216 * 2, 1);
        uint16_t* go = (uint16_t*)dmalloc((size_t)64 * 3 * 16 * 9216 * 2, 0);
        float* gc = (float*)dmalloc((size_t)1024 * 18432 * 4, 0);
        int epoch = 0;
        struct G { const char* n; int epi, N, K; const uint16_t* W; };
        for (int M : {25, 38, 70, 400, 677})
            for (G g : {G{"qkv", EPI_STORE, 6144, 1280, wqkv[1]}, G{"w13", EPI_SWIGLU, 10240, 1280, w13[1]},
                        G{"wo", EPI_RESID, 1280, 2048, wo[1]}, G{"w2", EPI_RESID, 1280, 5120, w2[1]},
                        G{"dqkv", EPI_STORE, 6144, 3072, wqkv[3]}, G{"dw13", EPI_SWIGLU, 18432, 3072, w13[3]},
                        G{"dwo", EPI_RESID, 3072, 4096, wo[3]}, G{"dw2", EPI_RESID, 3072, 9216, w2[3]}}) {
                if (g.n[0] == 'd' && M != 38 && M != 677) continue;
                const int S = g.K / 64;
                for (int mu : {0, std::max(4, S / 4), std::max(4, S / 8), 4}) {
                    g_gemmf_minu = mu;
                    double us = timeit([&] { CK(launch_gemmf(g.epi, 3, gp, g.K, M, g.W, g.N, nullptr, gc, g.epi == EPI_SWIGLU ? g.N / 2 : g.N,
                                                             g.epi == EPI_SWIGLU ? go : nullptr, gws, wsn, gfl, ++epoch, st)); }, 20, st);
                    printf("gemmfm %-4s M=%4d %5dx%-4d minu %3d %9.2f us  %7.1f GB/s weights\n", g.n, M, g.N, g.K, mu ? mu : std::max(4, (S + 1) / 2),
                           us, 2.0 * g.N * g.K / us / 1e3);
                    fflush(stdout);
                }
                g_gemmf_minu = 0;
            }
        return 0;
    }
    if (only_gemmf) return 0;
    {
        // batched decode GEMMs (16 streams, fragment-major weights and planes); weights are
        // constant-filled, so the packed layout does not matter for timing
        uint16_t* xp = (uint16_t*)dmalloc((size_t)2 * 3 * 16 * 9216 * 2, 1);
        float* Cs = (float*)dmalloc((size_t)16 * 131072 * 4, 0);
        float* part = (float*)dmalloc((size_t)2 * 16 * 18 * 18432 * 4, 0);
        for (int nw : {0, 4, 8}) {
            g_skl_nw = nw;
            printf("-- skl NW %d (0 = auto)\n", nw);
            struct S { const char* n; int N, K; uint16_t* const* W; double bytes; };
            for (S g : {S{"skl qkv  6144x3072 nb16", DQ + 2 * DKV, D, wqkv.data(), (DQ + 2.0 * DKV) * D * 2},
                        S{"skl wo   3072x4096 nb16", D, DQ, wo.data(), (double)D * DQ * 2},
                        S{"skl w13  18432x3072 nb16", 2 * DH, D, w13.data(), 2.0 * DH * D * 2},
                        S{"skl w2   3072x9216 nb16", D, DH, w2.data(), (double)D * DH * 2}})
                add(g.n, timeit([&] { CK(launch_gemm_skl(xp, g.K, g.W[layer++ % NL], nullptr, g.N, 16, part, st)); }, iters, st), g.bytes);
        }
        g_skl_nw = 0;
        {
            // streaming encoder chunk (-I 0.5, 25 rows = 2 row blocks of 16)
            struct S { const char* n; int N, K; uint16_t* const* W; double bytes; };
            for (S g : {S{"skl enc qkv 6144x1280 nb25", 6144, 1280, wqkv.data(), 6144.0 * 1280 * 2},
                        S{"skl enc wo  1280x2048 nb25", 1280, 2048, wo.data(), 1280.0 * 2048 * 2},
                        S{"skl enc w13 10240x1280 nb25", 10240, 1280, w13.data(), 10240.0 * 1280 * 2},
                        S{"skl enc w2  1280x5120 nb25", 1280, 5120, w2.data(), 1280.0 * 5120 * 2}})
                add(g.n, timeit([&] { CK(launch_gemm_skl(xp, g.K, g.W[layer++ % NL], nullptr, g.N, 25, part, st)); }, iters, st), g.bytes);
        }
        const int Rs[] = {0, 2, 2, 4, 4}, NWs[] = {0, 4, 4, 4, 8}, Ds[] = {0, 2, 3, 2, 2};
        for (int cfg = 0; cfg < (int)(sizeof Rs / sizeof Rs[0]); cfg++) {
            g_skf_r = Rs[cfg];
            g_skf_nw = NWs[cfg];
            g_skf_d = Ds[cfg];
            char nm[80];
            snprintf(nm, sizeof nm, "skf lm R%d NW%d D%d nb16", Rs[cfg], NWs[cfg], Ds[cfg]);
            add(nm, timeit([&] { CK(launch_gemm_skf(xp, D, emb, nullptr, V, 16, Cs, V, st)); }, iters / 10 + 1, st), (double)V * D * 2);
        }
        g_skf_r = 0;
        g_skf_nw = 0;
        g_skf_d = 0;
        float* xr = (float*)dmalloc((size_t)16 * 9216 * 4, 1);
        add("rmsnorm fplanes 16x3072", timeit([&] { CK(launch_rmsnorm_fplanes(xr, 16, D, xr, xr, 1e-5f, xp, nullptr, 0, st)); }, iters, st), 16.0 * D * 10);
        add("resid(18)+rmsnorm fplanes 16x3072", timeit([&] { CK(launch_rmsnorm_fplanes(xr, 16, D, xr, xr, 1e-5f, xp, part, 18, st)); }, iters, st), 16.0 * D * (10 + 4 * 18));
        add("split fplanes 16x4096", timeit([&] { CK(launch_split_fplanes(xr, 16, DQ, xp, st)); }, iters, st), 16.0 * DQ * 10);
        add("swiglu(6) fplanes 16x9216", timeit([&] { CK(launch_swiglu_fplanes(part, 6, DH, 16, xp, st)); }, iters, st), 16.0 * DH * (6 * 8 + 6));
    }
    for (int L : {64, 187, 256, 1000, 2300, 4096, 8192}) {
        int st4[4] = {L - 1, 0, 0, 0};
        CK(hipMemcpy(state, st4, 16, hipMemcpyHostToDevice));
        char nm[64];
        snprintf(nm, sizeof nm, "attn decode L=%d", L);
        int splits = 1;
        while (splits * ATT_BLOCK_KEYS < L) splits *= 2;
        add(nm, timeit([&] { CK(launch_attn_decode(HD, x, Kc, Vc, cap, state, 0, 8192, 0.088f, H, KVH, part, y, splits, st)); }, iters, st),
            (double)L * DKV * 2 * 4);
        if (L <= 256) {
            g_attn_short = 0;
            snprintf(nm, sizeof nm, "attn decode L=%d k_attn_decode", L);
            add(nm, timeit([&] { CK(launch_attn_decode(HD, x, Kc, Vc, cap, state, 0, 8192, 0.088f, H, KVH, part, y, splits, st)); }, iters, st),
                (double)L * DKV * 2 * 4);
            g_attn_short = 1;
        }
        for (int lw : {2, 4}) {
            if (L <= 256) continue;
            g_attn_lw = lw;
            snprintf(nm, sizeof nm, "attn decode L=%d %d-key blocks", L, lw * 16);
            add(nm, timeit([&] { CK(launch_attn_decode(HD, x, Kc, Vc, cap, state, 0, 8192, 0.088f, H, KVH, part, y, splits, st)); }, iters, st),
                (double)L * DKV * 2 * 4);
            g_attn_lw = 0;
        }
    }
    {
        // streaming encoder chunk (-I 0.5): 25 query rows over the 750-row window, 32 heads x 64
        const int EHd = 64, EH = 32, M = 25, EQ = EH * EHd, ecap = 1024;
        float* eq = (float*)dmalloc((size_t)M * EQ * 4, 1);
        float* eo = (float*)dmalloc((size_t)M * EQ * 4, 0);
        const size_t wsn = (size_t)EH * M * 16 * (EHd + 2);
        float* ews = (float*)dmalloc(wsn * 4, 0);
        uint16_t* exs = (uint16_t*)dmalloc((size_t)2 * 3 * 16 * EQ * 2, 0);
        char nm0[64];
        for (int q0 : {750, 2000}) {
            snprintf(nm0, sizeof nm0, "attn mf enc M=25 q0=%d", q0);
            add(nm0, timeit([&] { CK(launch_attn_rows_mf(EHd, eq, EQ, Kc, Vc, ecap, eo, EQ, M, EH, EH, q0, 0, 750, 0.125f, st, ews, wsn)); }, iters, st),
                (double)std::min(q0 + M, 750 + M - 1) * EQ * 2 * 4);
        }
        for (int nbk : {128, 256, 1024}) {
            g_attn_blocks = nbk;
            snprintf(nm0, sizeof nm0, "attn mf enc M=25 -> planes, ~%d blocks", nbk);
            add(nm0, timeit([&] { CK(launch_attn_rows_mf(EHd, eq, EQ, Kc, Vc, ecap, eo, EQ, M, EH, EH, 2000, 0, 750, 0.125f, st, ews, wsn, exs)); }, iters, st),
                (double)(750 + M - 1) * EQ * 2 * 4);
        }
        g_attn_blocks = 0;
        // one-shot encoder pass (jfk: 677 rows, keys from 0)
        {
            const int M1 = 677;
            float* q1 = (float*)dmalloc((size_t)M1 * EQ * 4, 1);
            float* o1 = (float*)dmalloc((size_t)M1 * EQ * 4, 0);
            add("attn mf enc M=677", timeit([&] { CK(launch_attn_rows_mf(EHd, q1, EQ, Kc, Vc, ecap, o1, EQ, M1, EH, EH, 0, 0, 750, 0.125f, st, ews, wsn)); }, iters / 4 + 1, st),
                (double)M1 * EQ * 2 * 4);
        }
    }
    {
        int st4[4] = {63, 0, 0, 0};
        CK(hipMemcpy(state, st4, 16, hipMemcpyHostToDevice));
        add("attn L=64 dbg1 (no merge)", timeit([&] { CK(launch_attn_dbg(1, x, Kc, Vc, cap, state, part, y, st)); }, iters, st), 1.0);
        add("attn L=64 dbg3 (loads+q only)", timeit([&] { CK(launch_attn_dbg(3, x, Kc, Vc, cap, state, part, y, st)); }, iters, st), 1.0);
    }
    {
        int st4[4] = {186, 0, 0, 0};
        CK(hipMemcpy(state, st4, 16, hipMemcpyHostToDevice));
        double acc[8] = {0}, cyc = 0, rt = 0, spread = 0, gstart = 0;
        int nrun = 20;
        for (int r = 0; r < nrun; r++) {
            CK(launch_attn_dbg(4, x, Kc, Vc, cap, state, part, y, st));
            CK(hipStreamSynchronize(st));
            std::vector<unsigned long long> h(32 * 16 * 10);
            CK(hipMemcpy(h.data(), part, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long g0 = ~0ull, g1 = 0;
            for (int b = 0; b < 32; b++) {
                unsigned long long mn = ~0ull, mx = 0;
                for (int w = 0; w < 12; w++) {
                    const unsigned long long* t = &h[(b * 16 + w) * 10];
                    acc[0] += t[6] - t[0];  // issue K/V
                    acc[1] += t[7] - t[6];  // q load + all loads landed
                    acc[2] += t[1] - t[7];  // barrier wait
                    acc[3] += t[2] - t[1];
                    acc[4] += t[3] - t[2];
                    acc[5] += t[4] - t[3];
                    acc[6] += t[5] - t[4];
                    cyc += t[5] - t[0];
                    rt += t[9] - t[8];
                    mn = std::min(mn, t[0]);
                    mx = std::max(mx, t[0]);
                    g0 = std::min(g0, t[8]);
                    g1 = std::max(g1, t[8]);
                }
                spread += mx - mn;
            }
            gstart += g1 - g0;
        }
        const double n = nrun * 384.0;
        printf("attn L=187 per-wave cycles: issue %.0f | loads land %.0f | barrier %.0f | QK/sm/PV %.0f | sO+sync %.0f | factors %.0f | merge %.0f ; total %.0f cyc = %.2f us (clk %.2f GHz); wave-start spread in block %.0f cyc; block start spread %.2f us\n",
               acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n, acc[6] / n, cyc / n, rt / n / 100.0,
               cyc / (rt / 100.0) / 1000.0, spread / (nrun * 32.0), gstart / nrun / 100.0);
    }
#ifdef VOX_GEMV_STAMPS
    {
        // per-block timeline of one launch of each big GEMV (s_memrealtime, 10 ns ticks)
        const int maxb = 4096;
        unsigned long long* dst;
        CK(hipMalloc(&dst, (size_t)maxb * 4 * 8));
        CK(gemv_set_stamps(dst));
        struct T { const char* n; int pro, epi, K, rows; const float* q; };
        for (T t : {T{"w13 bf16", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, nullptr}, T{"w2 bf16", PRO_NONE, EPI_RESID, DH, D, nullptr},
                    T{"qkv bf16", PRO_NORM, EPI_QKV, D, DQ + 2 * DKV, nullptr}, T{"wo bf16", PRO_NONE, EPI_RESID, DQ, D, nullptr},
                    T{"w13 q8", PRO_NORM_ADA, EPI_SWIGLU, D, 2 * DH, wsc}}) {
            const uint16_t* W = t.epi == EPI_SWIGLU ? w13[5] : t.epi == EPI_QKV ? wqkv[5] : t.K == DH ? w2[5] : wo[5];
            qs = t.q;
            for (int r = 0; r < 3; r++) {  // last run is measured; earlier ones flush other layers' buffers
                gemv(PRO_NONE, EPI_RESID, w2[(r + 7) % NL], DH, D);
                CK(hipMemset(dst, 0, (size_t)maxb * 32));
                gemv(t.pro, t.epi, W, t.K, t.rows);
                CK(hipStreamSynchronize(st));
            }
            qs = nullptr;
            const int nb = gemv_grid(t.rows);
            std::vector<unsigned long long> h((size_t)nb * 4);
            CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (int b = 0; b < nb; b++) t0 = std::min(t0, h[b * 4]);
            std::vector<double> st_, fd, en;
            for (int b = 0; b < nb; b++) {
                st_.push_back((h[b * 4] - t0) * 0.01);
                fd.push_back((h[b * 4 + 1] - t0) * 0.01);
                en.push_back((h[b * 4 + 2] - t0) * 0.01);
            }
            auto pct = [](std::vector<double> v, double p) { std::sort(v.begin(), v.end()); return v[(size_t)(p * (v.size() - 1))]; };
            printf("stamps %-9s blocks %4d | start p50 %.2f max %.2f | first data p10 %.2f p50 %.2f p90 %.2f | end p10 %.2f p50 %.2f p90 %.2f max %.2f us\n",
                   t.n, nb, pct(st_, 0.5), pct(st_, 1.0), pct(fd, 0.1), pct(fd, 0.5), pct(fd, 0.9), pct(en, 0.1), pct(en, 0.5),
                   pct(en, 0.9), pct(en, 1.0));
            printf("   end by blockIdx%%8:");
            for (int x = 0; x < 8; x++) {
                std::vector<double> v;
                for (int b = x; b < nb; b += 8) v.push_back(en[b]);
                printf(" [%d] p10 %.1f p50 %.1f max %.1f", x, pct(v, 0.1), pct(v, 0.5), pct(v, 1.0));
            }
            printf("\n   end by blockIdx/256:");
            for (int x = 0; x * 256 < nb; x++) {
                std::vector<double> v;
                for (int b = x * 256; b < std::min(nb, x * 256 + 256); b++) v.push_back(en[b]);
                printf(" [%d] p10 %.1f p50 %.1f max %.1f", x, pct(v, 0.1), pct(v, 0.5), pct(v, 1.0));
            }
            printf("\n");
        }
        CK(gemv_set_stamps(nullptr));
    }
#endif
    add("argmax+embed", timeit([&] { CK(launch_argmax_final(pv, pi, 1024, state, nullptr, 0, (float*)emb, 1024, emb, nullptr, D, x, nullptr, nullptr, st)); }, iters, st), 1.0);
    add("empty-ish (embed step)", timeit([&] { CK(launch_embed_step((float*)emb, emb, nullptr, state, D, x, st)); }, iters, st), 1.0);
    // whole-layer sequence (no graph)
    int st4[4] = {186, 0, 0, 0};
    CK(hipMemcpy(state, st4, 16, hipMemcpyHostToDevice));
    double t = timeit([&] {
        int l = layer++ % NL;
        gemv(PRO_NORM, EPI_QKV, wqkv[l], D, DQ + 2 * DKV);
        CK(launch_attn_decode(HD, x, Kc, Vc, cap, state, 0, 8192, 0.088f, H, KVH, part, y, 1, st));
        gemv(PRO_NONE, EPI_RESID, wo[l], DQ, D);
        gemv(PRO_NORM_ADA, EPI_SWIGLU, w13[l], D, 2 * DH);
        gemv(PRO_NONE, EPI_RESID, w2[l], DH, D);
    }, iters, st);
    add("layer (5 launches, eager)", t, 232783872.0);
    return 0;
}
