// vox_hip_pstep.hip -- the single-stream decode step's decoder layers as ONE persistent
// launch (voxtral_decoder.c:707-760 for every layer; the LM head and argmax stay separate
// launches).
//
// Why: as one launch per operation, each of the 130 per-token kernels pays a first-byte ramp,
// a tail and a boundary (~3-4 us each) on top of its bytes.  Here the
// weight stream never stops at an operation boundary: every workgroup (one per CU) owns a
// fixed slice of rows of every matrix, so the order in which it reads weights is known in
// advance, and each streamer wave keeps PS_D 16-B loads per lane (PS_D KiB) in flight in a
// register ring that runs ahead across the hand-offs between operations.
//
// Roles (16 waves per workgroup): waves 0-7 stream weights and do nothing else (their only
// vector-memory instructions are the ring's loads, so no other wait drains the ring; at an
// operation boundary they only pass workgroup barriers); waves 8-15 ("aux") do the
// epilogues, the hand-offs and the attention while the streamers' loads stay in flight.
//
// Hand-offs (MI355X_MICROARCH.md "inter-workgroup visibility", granule form R2): every output
// element is published as an 8-byte granule {f32 value, tag} with a write-through (sc1)
// store; consumers sweep the whole vector with sc1 loads until every tag matches.  tag =
// (launch epoch << 8) | (edge id + 1), the epoch advancing once per launch (ctl[0]), so a
// granule of an earlier launch never matches.  No counters, no fences on the data path.
//
// Work split: matrix rows in slices of R (a multiple of 4) per workgroup; streamer w takes
// rows rw = w & 3, rw + 4, ... over the K half kw = w >> 2, 64 16-B chunks per load (lane =
// chunk); the two halves meet in LDS.  W1|W3 slices are whole hidden units (both interleaved
// rows), QKV slices whole RoPE pairs.
//
// Attention (contexts of <= 256 keys; longer contexts use the per-operation graph): the aux
// waves of the first H workgroups each take one query head, 32 keys per wave, merged in LDS
// (voxtral_kernels.c:541-611 semantics: online softmax over the last min(pos+1, W) logical
// positions).
//
// Status (opt-in, VOX_HIP_PSTEP=1): bit-compatible with the oracle
// bars, and the weight stream alone runs at 35.7 us per Voxtral-4B layer (6.5 TB/s, flags=1
// in tools/pstep_dbg), but each of the five hand-offs per layer costs ~5 us (attention ~10)
// and the ring does not hide them: a streamer that issues its refill as it consumes runs at
// the issue rate of a full memory queue after a boundary, so a landed prefetch is not drained
// faster than new loads go out.  59 us per layer against 53 for the per-operation graph.  An
// LDS-DMA loader / consumer split (loaders issue, consumers only read LDS) streamed at only
// 3.7-4.1 TB/s here.
#include "vox_hip_pstep.h"
#include "../../voxtral.c_amd/csrc/vox_hip_dev.h"

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace vox {

// PS_DIAG (tools/pstep_dbg builds only): 1 = no streamer timeline stamps, 2 = also no operand
// reads in the streamer's dot products, 3 = a one-add stand-in for the dot product
#ifndef PS_DIAG
#define PS_DIAG 0
#endif
#define PS_STREAMER_STAMPS (PS_DIAG == 0)

constexpr int PS_SW = 8;                 // streamer waves
constexpr int PS_AW = 8;                 // aux waves
constexpr int PS_NT = (PS_SW + PS_AW) * 64;
constexpr int PS_AT = PS_AW * 64;        // aux threads
constexpr int PS_XMAX = 20480;           // operand floats (80 KiB: also keeps one workgroup per CU)
constexpr int PS_RMAX = 128;             // rows per workgroup per matrix
constexpr int PS_HD = 128;               // head_dim (Voxtral decoder)
constexpr int PS_MAXKEYS = 256;          // context handled in-launch (8 aux waves x 32 keys)
constexpr int PS_MAXL = 64;              // decoder layers

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ps_rsrc(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
// granule stores: write-through (sc1)
__device__ __forceinline__ void ps_put1(__amdgpu_buffer_rsrc_t g, int i, float v, uint32_t tag) {
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(v), tag}, g, i * 8, 0, 16);
}
__device__ __forceinline__ void ps_put2(__amdgpu_buffer_rsrc_t g, int i, float v0, float v1, uint32_t tag) {
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v0), tag, __float_as_uint(v1), tag}, g, i * 8, 0, 16);
}

struct PsGeo {
    int rows, K, C, CH, L, R, nk, rowbytes;
};

// Spin bound for a hand-off (~0.3 s): past it the launch records ctl[2] = 1 and stops
// waiting (its results are garbage, but it ends: no hung GPU).
constexpr int PS_SPIN_LIMIT = 1 << 18;

__device__ __forceinline__ u32x4 ps_poll(__amdgpu_buffer_rsrc_t g, int pair, u32x4 v, uint32_t tag, int* s_err) {
    int spins = 0;
    while ((v.y != tag || v.w != tag) && !*(volatile int*)s_err) {
        if (++spins > PS_SPIN_LIMIT) {
            *(volatile int*)s_err = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
        v = __builtin_amdgcn_raw_buffer_load_b128(g, pair * 16, 0, 16);
    }
    return v;
}

// Aux threads sweep n granules (n even) of g until every tag matches; values to dst (LDS).
// Element rows [rb, rb + rn) are also copied to xr (residual rows).  Returns this thread's
// sum of squares of the values it stored.  Thread at owns pairs at + PS_AT * m, 8 loads in
// flight; the pairs not ready yet are re-read together (one round trip per retry).
__device__ float ps_gather(__amdgpu_buffer_rsrc_t g, int n, uint32_t tag, float* dst, int* s_err, int at,
                           float* xr = nullptr, int rb = 0, int rn = 0) {
    const int np = n >> 1;
    float ss = 0.f;
    for (int i0 = 0; i0 < np; i0 += 8 * PS_AT) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = min(i0 + u * PS_AT + at, np - 1);
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(g, i * 16, 0, 16);
        }
        for (int spins = 0;; spins++) {
            bool ready = true;
#pragma unroll
            for (int u = 0; u < 8; u++) ready &= (v[u].y == tag && v[u].w == tag) || i0 + u * PS_AT + at >= np;
            if (ready || *(volatile int*)s_err) break;
            if (spins > PS_SPIN_LIMIT) {
                *(volatile int*)s_err = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int i = min(i0 + u * PS_AT + at, np - 1);
                if (v[u].y != tag || v[u].w != tag) v[u] = __builtin_amdgcn_raw_buffer_load_b128(g, i * 16, 0, 16);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = i0 + u * PS_AT + at;
            if (i >= np) break;
            const float a = __uint_as_float(v[u].x), b = __uint_as_float(v[u].z);
            dst[2 * i] = a;
            dst[2 * i + 1] = b;
            ss = fmaf(a, a, fmaf(b, b, ss));
            if (xr) {
                const int r0 = 2 * i - rb;
                if (r0 >= 0 && r0 < rn) xr[r0] = a;
                if (r0 + 1 >= 0 && r0 + 1 < rn) xr[r0 + 1] = b;
            }
        }
    }
    return ss;
}

__device__ __forceinline__ void ps_barrier() {
    // LDS writes done, then the workgroup barrier -- without the vmcnt(0) drain that
    // __syncthreads() would add (the streamers' ring loads stay in flight across it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// diagnostic timeline (tools/pstep_dbg): a.stamps[(layer * G + block) * 16 + point]
#define PS_STAMP(l, k) \
    do { if (a.stamps && at == 0) a.stamps[((size_t)(l) * gridDim.x + blockIdx.x) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)

// PS_D: ring depth, 16-B loads per lane in flight per streamer wave
template <int PS_D>
__global__ __launch_bounds__(PS_NT, 1) void k_pstep(const PStepArgs a) {
    __shared__ __attribute__((aligned(16))) float s_xo[PS_XMAX];
    __shared__ float s_part[2 * PS_RMAX];
    __shared__ float s_xr[PS_RMAX];   // residual x of this workgroup's rows (next wo / W2)
    __shared__ __attribute__((aligned(16))) float s_att[3 * PS_HD + PS_AW * PS_HD + 2 * PS_AW];
    __shared__ float s_red[PS_AW];
    __shared__ PsGeo s_geo[4];
    __shared__ unsigned long long s_wp[PS_MAXL * 4];  // weight base of (layer, matrix)
    __shared__ int s_err;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.x, G = gridDim.x;
    const int D = a.D, H = a.H, KVH = a.KVH, DH = a.DH, hd = PS_HD;
    const int DQ = H * hd, DKV = KVH * hd, nl = a.nl;
    if (tid < 4) {
        const int p = tid;
        const int rows = p == 0 ? DQ + 2 * DKV : p == 2 ? 2 * DH : D;
        const int K = p == 1 ? DQ : p == 3 ? DH : D;
        PsGeo q;
        q.rows = rows;
        q.K = K;
        q.C = K >> 3;
        q.CH = (((q.C + 1) >> 1) + 63) & ~63;
        q.L = q.CH >> 6;
        const int R = p == 2 ? 2 * ((DH + G - 1) / G) : (rows + G - 1) / G;
        q.R = (R + 3) & ~3;
        q.nk = q.R >> 2;  // rows per streamer wave (4 row lanes x 2 K halves)
        q.rowbytes = K * 2;
        s_geo[p] = q;
    }
    if (tid == 0) s_err = 0;
    for (int i = tid; i < nl * 4; i += PS_NT) s_wp[i] = (unsigned long long)(uintptr_t)a.layers[i >> 2].w[i & 3];
    __syncthreads();
    auto geo = [&](int p) {
        PsGeo q;
        q.rows = __builtin_amdgcn_readfirstlane(s_geo[p].rows);
        q.K = __builtin_amdgcn_readfirstlane(s_geo[p].K);
        q.C = __builtin_amdgcn_readfirstlane(s_geo[p].C);
        q.CH = __builtin_amdgcn_readfirstlane(s_geo[p].CH);
        q.L = __builtin_amdgcn_readfirstlane(s_geo[p].L);
        q.R = __builtin_amdgcn_readfirstlane(s_geo[p].R);
        q.nk = __builtin_amdgcn_readfirstlane(s_geo[p].nk);
        q.rowbytes = __builtin_amdgcn_readfirstlane(s_geo[p].rowbytes);
        return q;
    };
    const int U = (DH + G - 1) / G;  // hidden units per workgroup (W1|W3)

    if (wave < PS_SW) {
        // ======================= streamer waves =======================
        const int rw = wave & 3, kw = wave >> 2;
        // issue cursor: layer il, matrix ip, local row ik of this wave, round ij
        int il = 0, ip = 0, ik = 0, ij = 0;
        PsGeo ig = geo(0);
        // descriptor of matrix (il, ip) from wave-uniform values (SGPRs: no waterfall loop);
        // past the last layer a zero-length range (loads return 0, no traffic)
        auto mk_rsrc = [&]() {
            const unsigned long long p = s_wp[il < nl ? il * 4 + ip : 0];
            const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
            const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
            const int nbytes = il < nl ? ig.rows * ig.rowbytes : 0;
            return ps_rsrc(reinterpret_cast<const void*>(((uint64_t)hi << 32) | lo), nbytes);
        };
        __amdgpu_buffer_rsrc_t irs = mk_rsrc();
        auto row_off = [&]() -> int {
            const int q = rw + 4 * ik;
            int row;
            if (ip == 2) {
                const int u = min(b * U + (q >> 1), DH - 1);
                row = ((u >> 4) << 5) + (u & 15) + ((q & 1) << 4);
            } else {
                row = min(b * ig.R + q, ig.rows - 1);
            }
            return row * ig.rowbytes;
        };
        int isoff = row_off();
        int icol = kw * ig.CH;
        auto issue = [&]() -> u32x4 {
            int c = icol + lane;
            c = c < ig.C ? c : 0;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(irs, c * 16, isoff, 2);
            icol += 64;
            if (++ij == ig.L) {
                ij = 0;
                if (++ik == ig.nk) {
                    ik = 0;
                    if (++ip == 4) {
                        ip = 0;
                        ++il;
                    }
                    ig = geo(ip);
                    irs = mk_rsrc();
                }
                icol = kw * ig.CH;
                isoff = row_off();
            }
            return v;
        };
        u32x4 r[PS_D];
#pragma unroll
        for (int i = 0; i < PS_D; i++) r[i] = issue();
        // layer 0's QKV operand (aux): two barriers
        ps_barrier();
        ps_barrier();
        // consume cursor: layer cl, matrix cp, local row ck, round cj
        int cl = 0, cp = 0, ck = 0, cj = 0;
        PsGeo cg = geo(0);
        const float4* xo4 = reinterpret_cast<const float4*>(s_xo);
        int xb = 2 * (kw * cg.CH + lane);
        float acc = 0.f;
        // the operand chunk of the next slot is read from LDS one slot ahead, so its latency
        // hides behind this slot's FMAs and refill
        float4 xa = xo4[xb], xc = xo4[xb + 1];
        for (;;) {
#pragma unroll
            for (int i = 0; i < PS_D; i++) {
#if PS_DIAG == 3
                acc += __uint_as_float(r[i].x);
#elif PS_DIAG == 2
                acc = dot8(make_uint4(r[i].x, r[i].y, r[i].z, r[i].w), make_float4(1.f, 2.f, 3.f, 4.f), make_float4(acc, 2.f, 3.f, 4.f), acc);
#else
                acc = dot8(make_uint4(r[i].x, r[i].y, r[i].z, r[i].w), xa, xc, acc);
#endif
                if (PS_STREAMER_STAMPS && a.stamps && wave == 0 && lane == 0 && cp == 2 && cj == 0 && (ck == 0 || ck == 3))
                    a.stamps[((size_t)cl * gridDim.x + blockIdx.x) * 16 + 10 + (ck ? 1 : 0)] = __builtin_amdgcn_s_memrealtime();
                if (!(a.flags & 2)) r[i] = issue();  // flags & 2 (diagnostics): consume only, no refills
                if (++cj == cg.L) {
                    cj = 0;
                    acc = wave_sum63(acc);
                    if (lane == 63) s_part[(rw + 4 * ck) * 2 + kw] = acc;
                    acc = 0.f;
                    if (++ck == cg.nk) {
                        ck = 0;
                        // the aux waves' barriers of this boundary (see their sequence below)
                        const int nb = cp == 0 ? 4 : cp == 1 ? 3 : cp == 2 ? 2 : (cl == nl - 1 ? 1 : 3);
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        if (PS_STREAMER_STAMPS && a.stamps && wave == 0 && lane == 0 && cp == 2)
                            a.stamps[((size_t)cl * gridDim.x + blockIdx.x) * 16 + 12] = __builtin_amdgcn_s_memrealtime();
                        for (int q = 0; q < nb; q++) __builtin_amdgcn_s_barrier();
                        if (PS_STREAMER_STAMPS && a.stamps && wave == 0 && lane == 0 && cp == 1)
                            a.stamps[((size_t)cl * gridDim.x + blockIdx.x) * 16 + 13] = __builtin_amdgcn_s_memrealtime();
                        if (++cp == 4) {
                            cp = 0;
                            if (++cl == nl) goto streamed;
                        }
                        cg = geo(cp);
                        xb = 2 * (kw * cg.CH + lane);
                    }
                }
                xa = xo4[xb + 128 * cj];
                xc = xo4[xb + 128 * cj + 1];
            }
        }
    streamed:
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }

    // ======================= aux waves =======================
    const int at = tid - PS_SW * 64, aw = wave - PS_SW;
    const uint32_t epoch = (uint32_t)a.ctl[0];
    const int lp = a.state[0];
    const int L = min(lp + 1, a.window);
    const int first = lp - L + 1;
    const __amdgpu_buffer_rsrc_t Gq = ps_rsrc(a.gq, (DQ + 2 * DKV) * 8);
    const __amdgpu_buffer_rsrc_t Ga = ps_rsrc(a.ga, DQ * 8);
    const __amdgpu_buffer_rsrc_t Gx = ps_rsrc(a.gx, D * 8);
    const __amdgpu_buffer_rsrc_t Gg = ps_rsrc(a.gg, DH * 8);
    auto tagof = [&](int l, int e) -> uint32_t { return (epoch << 8) | (uint32_t)(l * 5 + e + 1); };
    auto zero_pad = [&](int p) {
        for (int i = s_geo[p].K + at; i < 2 * s_geo[p].CH * 8; i += PS_AT) s_xo[i] = 0.f;
    };
    auto block_ss = [&](float ss) {  // aux-wave partial sums of squares -> s_red (before a barrier)
        ss = wave_sum(ss);
        if (lane == 0) s_red[aw] = ss;
    };
    auto total_ss = [&]() {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < PS_AW; i++) t += s_red[i];
        return t;
    };
    // normalize the elements this thread gathered: x * inv * w (* (1 + ada))
    auto normalize = [&](const float* nw, const float* ada) {
        const float inv = 1.0f / sqrtf(total_ss() / (float)D + a.eps);
        for (int i = 2 * at; i < D; i += 2 * PS_AT) {
            float v0 = s_xo[i] * inv * nw[i], v1 = s_xo[i + 1] * inv * nw[i + 1];
            if (ada) {
                v0 *= (1.0f + ada[i]);
                v1 *= (1.0f + ada[i + 1]);
            }
            s_xo[i] = v0;
            s_xo[i + 1] = v1;
        }
    };
    const int Rq = s_geo[0].R, Ro = s_geo[1].R, R2 = s_geo[3].R;
    const bool skip = (a.flags & 7) != 0;  // diagnostics: barriers only (timing of the weight stream alone)

    // layer 0's QKV operand: the step input x (plain: written by the previous launch)
    {
        float ss = 0.f;
        for (int i = 2 * at; i < D; i += 2 * PS_AT) {
            const float2 v = *reinterpret_cast<const float2*>(a.x + i);
            s_xo[i] = v.x;
            s_xo[i + 1] = v.y;
            ss = fmaf(v.x, v.x, fmaf(v.y, v.y, ss));
            const int r0 = i - b * Ro;
            if (r0 >= 0 && r0 < Ro) s_xr[r0] = v.x;
            if (r0 + 1 >= 0 && r0 + 1 < Ro) s_xr[r0 + 1] = v.y;
        }
        block_ss(ss);
        ps_barrier();
        normalize(a.layers[0].attn_norm, nullptr);
        zero_pad(0);
        ps_barrier();
    }
    for (int l = 0; l < nl; l++) {
        const PLayer& Ly = a.layers[l];
        const int lcap = a.cap;
        PS_STAMP(l, 0);
        if (skip) {
            // flags & 4 (diagnostics): every hand-off replaced by a wait of flags >> 8 ticks (10 ns)
            const uint64_t T = (uint64_t)(a.flags >> 8);
            auto edge = [&](int nb) {
                ps_barrier();
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (__builtin_amdgcn_s_memrealtime() - t0 < T) __builtin_amdgcn_s_sleep(1);
                for (int q = 1; q < nb; q++) ps_barrier();
            };
            edge(4);
            edge(3);
            edge(2);
            edge(l != nl - 1 ? 3 : 1);
            continue;
        }
        // attention: wave aw takes keys [first + 32 aw, +32) in 4 blocks of 8; lane = (key kk,
        // 16-dim chunk c); the new key (position lp) comes from its granules
        const int kk = lane >> 3, c = lane & 7;
        const int k0 = first + 32 * aw;
        const int kn = min(32, lp + 1 - k0);  // keys of this wave (<= 0: none)
        const int kvh = b < H ? b / (H / KVH) : 0;
        auto cache_row = [&](int sb) -> size_t {
            const int key = k0 + 8 * sb + kk;
            return (8 * sb + kk < kn && key != lp) ? (size_t)(key % lcap) * DKV + kvh * hd + 16 * c : 0;
        };
        // ---- after QKV: RoPE + KV append epilogue, attention, wo operand (4 barriers) ----
        ps_barrier();
        PS_STAMP(l, 1);
        {
            const float* rp = a.rope + (size_t)lp * hd;
            const size_t slot = (size_t)(lp % lcap) * DKV;
            for (int m = at; m < Rq / 2; m += PS_AT) {
                const int r = b * Rq + 2 * m;
                if (r >= DQ + 2 * DKV) break;
                const float v0 = s_part[4 * m] + s_part[4 * m + 1];
                const float v1 = s_part[4 * m + 2] + s_part[4 * m + 3];
                if (r < DQ + DKV) {
                    const int col = r < DQ ? r : r - DQ;
                    const int d = (col % hd) & ~1;
                    const float cs = rp[d], sn = rp[d + 1];
                    const float o0 = v0 * cs - v1 * sn, o1 = v0 * sn + v1 * cs;
                    ps_put2(Gq, r, o0, o1, tagof(l, 0));
                    if (r >= DQ) {
                        Ly.Kc[slot + col] = o0;
                        Ly.Kc[slot + col + 1] = o1;
                    }
                } else {
                    ps_put2(Gq, r, v0, v1, tagof(l, 0));
                    Ly.Vc[slot + r - DQ - DKV] = v0;
                    Ly.Vc[slot + r - DQ - DKV + 1] = v1;
                }
            }
        }
        float* sq = s_att;
        float* skn = s_att + PS_HD;
        float* svn = s_att + 2 * PS_HD;
        float* sO = s_att + 3 * PS_HD;
        float* sM = sO + PS_AW * PS_HD;
        float* sL = sM + PS_AW;
        const int h = b;
        if (b < H && at < 3 * PS_HD / 2) {
            const int part = at / (PS_HD / 2), e = (at % (PS_HD / 2)) * 2;
            const int src = part == 0 ? h * hd + e : part == 1 ? DQ + kvh * hd + e : DQ + DKV + kvh * hd + e;
            u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(Gq, src * 8, 0, 16);
            v = ps_poll(Gq, src / 2, v, tagof(l, 0), &s_err);
            float* dst = part == 0 ? sq : part == 1 ? skn : svn;
            dst[e] = __uint_as_float(v.x);
            dst[e + 1] = __uint_as_float(v.z);
        }
        ps_barrier();
        PS_STAMP(l, 2);
        if (b < H) {
            const float* Vc = Ly.Vc;
            const float4* qr = reinterpret_cast<const float4*>(sq + 16 * c);
            // K rows of the 4 blocks in flight together (the new key's from LDS: its cache row
            // was written in this launch), then the V rows into the same registers
            float4 kv[4][4];
#pragma unroll
            for (int sb = 0; sb < 4; sb++) {
                const bool isnew = 8 * sb + kk < kn && k0 + 8 * sb + kk == lp;
                const float4* kr = isnew ? reinterpret_cast<const float4*>(skn + 16 * c)
                                         : reinterpret_cast<const float4*>(Ly.Kc + cache_row(sb));
#pragma unroll
                for (int i = 0; i < 4; i++) kv[sb][i] = kr[i];
            }
            float sc[4];
#pragma unroll
            for (int sb = 0; sb < 4; sb++) {
                float dot = 0.f;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float4 qv = qr[i];
                    dot = fmaf(qv.x, kv[sb][i].x, fmaf(qv.y, kv[sb][i].y, fmaf(qv.z, kv[sb][i].z, fmaf(qv.w, kv[sb][i].w, dot))));
                }
                dot += __shfl_xor(dot, 1, 64);
                dot += __shfl_xor(dot, 2, 64);
                dot += __shfl_xor(dot, 4, 64);
                sc[sb] = (8 * sb + kk < kn) ? dot * a.scale : -INFINITY;
            }
#pragma unroll
            for (int sb = 0; sb < 4; sb++) {
                const bool isnew = 8 * sb + kk < kn && k0 + 8 * sb + kk == lp;
                const float4* vr = isnew ? reinterpret_cast<const float4*>(svn + 16 * c)
                                         : reinterpret_cast<const float4*>(Ly.Vc + cache_row(sb));
#pragma unroll
                for (int i = 0; i < 4; i++) kv[sb][i] = vr[i];
            }
            float mx = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
            mx = wave_max(mx);
            float ls = 0.f;
#pragma unroll
            for (int sb = 0; sb < 4; sb++) {
                sc[sb] = (8 * sb + kk < kn) ? expf(sc[sb] - mx) : 0.f;
                ls += sc[sb];
            }
            ls += __shfl_xor(ls, 8, 64);
            ls += __shfl_xor(ls, 16, 64);
            ls += __shfl_xor(ls, 32, 64);
            float o[16];
#pragma unroll
            for (int e = 0; e < 16; e++) o[e] = 0.f;
#pragma unroll
            for (int sb = 0; sb < 4; sb++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    o[4 * i] = fmaf(sc[sb], kv[sb][i].x, o[4 * i]);
                    o[4 * i + 1] = fmaf(sc[sb], kv[sb][i].y, o[4 * i + 1]);
                    o[4 * i + 2] = fmaf(sc[sb], kv[sb][i].z, o[4 * i + 2]);
                    o[4 * i + 3] = fmaf(sc[sb], kv[sb][i].w, o[4 * i + 3]);
                }
#pragma unroll
            for (int e = 0; e < 16; e++) {
                o[e] += __shfl_xor(o[e], 8, 64);
                o[e] += __shfl_xor(o[e], 16, 64);
                o[e] += __shfl_xor(o[e], 32, 64);
            }
            if (kk == 0) {
#pragma unroll
                for (int e = 0; e < 16; e++) sO[aw * PS_HD + 16 * c + e] = o[e];
            }
            if (lane == 0) {
                sM[aw] = kn > 0 ? mx : -1e30f;
                sL[aw] = ls;
            }
        }
        ps_barrier();
        PS_STAMP(l, 3);
        if (b < H && at < PS_HD / 2) {
            float M = -1e30f;
#pragma unroll
            for (int w = 0; w < PS_AW; w++) M = fmaxf(M, sM[w]);
            float den = 0.f, n0 = 0.f, n1 = 0.f;
#pragma unroll
            for (int w = 0; w < PS_AW; w++) {
                const float f = expf(sM[w] - M);
                den = fmaf(f, sL[w], den);
                n0 = fmaf(f, sO[w * PS_HD + 2 * at], n0);
                n1 = fmaf(f, sO[w * PS_HD + 2 * at + 1], n1);
            }
            const float inv = den > 0.f ? 1.0f / den : 0.f;
            ps_put2(Ga, h * hd + 2 * at, n0 * inv, n1 * inv, tagof(l, 1));
        }
        ps_gather(Ga, DQ, tagof(l, 1), s_xo, &s_err, at);
        zero_pad(1);
        ps_barrier();
        PS_STAMP(l, 4);
        // ---- after wo: residual epilogue, W1|W3 operand = norm(x') * (1 + ada) (3 barriers) ----
        ps_barrier();
        PS_STAMP(l, 5);
        for (int i = at; i < Ro; i += PS_AT) {
            const int r = b * Ro + i;
            if (r >= D) break;
            ps_put1(Gx, r, s_xr[i] + (s_part[2 * i] + s_part[2 * i + 1]), tagof(l, 2));
        }
        block_ss(ps_gather(Gx, D, tagof(l, 2), s_xo, &s_err, at, s_xr, b * R2, R2));
        ps_barrier();
        normalize(Ly.ffn_norm, Ly.ada);
        zero_pad(2);
        ps_barrier();
        PS_STAMP(l, 6);
        // ---- after W1|W3: silu * up epilogue, W2 operand (2 barriers) ----
        ps_barrier();
        PS_STAMP(l, 7);
        for (int m = at; m < U; m += PS_AT) {
            const int u = b * U + m;
            if (u >= DH) break;
            const float gv = s_part[4 * m] + s_part[4 * m + 1], uv = s_part[4 * m + 2] + s_part[4 * m + 3];
            ps_put1(Gg, u, silu(gv) * uv, tagof(l, 3));
        }
        ps_gather(Gg, DH, tagof(l, 3), s_xo, &s_err, at);
        zero_pad(3);
        ps_barrier();
        PS_STAMP(l, 8);
        // ---- after W2: residual epilogue, next layer's QKV operand (3 barriers; last: 1) ----
        ps_barrier();
        PS_STAMP(l, 9);
        const bool last = l == nl - 1;
        for (int i = at; i < R2; i += PS_AT) {
            const int r = b * R2 + i;
            if (r >= D) break;
            const float v = s_xr[i] + (s_part[2 * i] + s_part[2 * i + 1]);
            if (last) a.x[r] = v;
            else ps_put1(Gx, r, v, tagof(l, 4));
        }
        if (!last) {
            block_ss(ps_gather(Gx, D, tagof(l, 4), s_xo, &s_err, at, s_xr, b * Ro, Ro));
            ps_barrier();
            normalize(a.layers[l + 1].attn_norm, nullptr);
            zero_pad(0);
            ps_barrier();
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (at == 0) {
        if (s_err) atomicOr(&a.ctl[2], 1);
        const int old = atomicAdd(&a.ctl[1], 1);
        if (old == G - 1) {
            // the last workgroup: every other one has passed its last wait
            a.ctl[1] = 0;
            a.ctl[0] = (int)(epoch + 1);
        }
    }
}

bool pstep_ok(int D, int H, int KVH, int hd, int DH, int G) {
    if (hd != PS_HD || H % KVH || G < H || D % 8 || DH % 2 || D % 2) return false;
    const int DQ = H * hd, DKV = KVH * hd;
    const int rows[4] = {DQ + 2 * DKV, D, 2 * DH, D};
    const int Ks[4] = {D, DQ, D, DH};
    for (int p = 0; p < 4; p++) {
        const int C = Ks[p] / 8, CH = ((C + 1) / 2 + 63) / 64 * 64;
        if (Ks[p] % 8 || 2 * CH * 8 > PS_XMAX) return false;
        int R = p == 2 ? 2 * ((DH + G - 1) / G) : (rows[p] + G - 1) / G;
        R = (R + 3) / 4 * 4;
        if (R > PS_RMAX) return false;
        if ((long long)rows[p] * Ks[p] * 2 >= (1ll << 31)) return false;  // buffer descriptor range
    }
    return true;
}

int pstep_max_keys() { return PS_MAXKEYS; }

int g_pstep_d = 0;  // tools/pstep_dbg knob: ring depth (0 = default)

static const void* pstep_fn() {
    switch (g_pstep_d) {
        case 8: return reinterpret_cast<const void*>(&k_pstep<8>);
        default: return reinterpret_cast<const void*>(&k_pstep<16>);
    }
}

hipError_t launch_pstep(const PStepArgs& a, int G, hipStream_t st) {
    PStepArgs args = a;
    void* kargs[] = {&args};
    return hipLaunchKernel(pstep_fn(), dim3(G), dim3(PS_NT), kargs, 0, st);
}

// the same launch with HIP events recorded by its own dispatch packet (eager steps only)
hipError_t launch_pstep_timed(const PStepArgs& a, int G, hipEvent_t start, hipEvent_t stop, hipStream_t st) {
    PStepArgs args = a;
    void* kargs[] = {&args};
    return hipExtLaunchKernel(pstep_fn(), dim3(G), dim3(PS_NT), kargs, 0, st, start, stop, 0);
}

}  // namespace vox
