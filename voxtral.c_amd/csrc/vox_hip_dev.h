// vox_hip_dev.h -- device helpers shared by the kernel files (bf16 conversion, DPP
// reductions, activations, the f32 -> 3 x bf16 split, 8/16-weight dot products).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vox_hip_internal.h"

namespace vox {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

// streamed-once weights: non-temporal 16-B load (MI355X_MICROARCH.md row nt-weights)
__device__ __forceinline__ uint4 ldnt(const uint4* p) {
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ float bf2f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }
__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// round-to-nearest-even f32 -> bf16 bits: the native conversion (hipcc emits
// v_cvt_pk_bf16_f32 on gfx950, two values per instruction)
__device__ __forceinline__ uint32_t f2bf(float f) {
    const __bf16 b = (__bf16)f;
    return __builtin_bit_cast(unsigned short, b);
}

// Cross-lane reductions: DPP inside each 16-lane row (quad_perm xor1 / xor2, row half
// mirror, row mirror -- VALU ops with no LDS round trip), then two ds_bpermute steps
// across rows.  The pairing pattern is fixed, so results are deterministic.
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// v uniform within each row of 16 lanes: the 4 rows combined through scalar reads of lanes
// 0 / 16 / 32 / 48 (no ds_bpermute round trip); (r0 + r1) + (r2 + r3), the order of the
// xor-16-then-32 shuffle reduction, so the sums are the same bits
__device__ __forceinline__ float rows4_sum(float v) {
    const int iv = __float_as_int(v);
    const float a = __int_as_float(__builtin_amdgcn_readlane(iv, 0)), b = __int_as_float(__builtin_amdgcn_readlane(iv, 16));
    const float c = __int_as_float(__builtin_amdgcn_readlane(iv, 32)), d = __int_as_float(__builtin_amdgcn_readlane(iv, 48));
    return (a + b) + (c + d);
}
__device__ __forceinline__ float rows4_max(float v) {
    const int iv = __float_as_int(v);
    const float a = __int_as_float(__builtin_amdgcn_readlane(iv, 0)), b = __int_as_float(__builtin_amdgcn_readlane(iv, 16));
    const float c = __int_as_float(__builtin_amdgcn_readlane(iv, 32)), d = __int_as_float(__builtin_amdgcn_readlane(iv, 48));
    return fmaxf(fmaxf(a, b), fmaxf(c, d));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);  // row_half_mirror
    v += dpp<0x140>(v);  // row_mirror
    return v;
}
__device__ __forceinline__ float row_max16(float v) {
    v = fmaxf(v, dpp<0xB1>(v));
    v = fmaxf(v, dpp<0x4E>(v));
    v = fmaxf(v, dpp<0x141>(v));
    v = fmaxf(v, dpp<0x140>(v));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
    v = row_sum16(v);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
}
// All-DPP wave64 sum (no LDS round trip): the total lands in lane 63 only.
// row_bcast:15 adds row r-1's lane 15 into rows 1 and 3, row_bcast:31 adds lane 31 into rows 2 and 3.
__device__ __forceinline__ float wave_sum63(float v) {
    v = row_sum16(v);
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    v = row_max16(v);
    v = fmaxf(v, __shfl_xor(v, 16, 64));
    v = fmaxf(v, __shfl_xor(v, 32, 64));
    return v;
}

__device__ __forceinline__ float gelu_tanh(float v) {  // voxtral_kernels.c:505-513
    float x3 = v * v * v;
    float inner = 0.7978845608028654f * (v + 0.044715f * x3);
    return 0.5f * v * (1.0f + tanhf(inner));
}
__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }
__device__ __forceinline__ float silu(float v) { return v / (1.0f + expf(-v)); }  // :498-503

// f32 -> three bf16 terms hi + mid + lo (= the exact f32 value; see k_gemm)
__device__ __forceinline__ void split3(float v, uint16_t& h, uint16_t& m, uint16_t& l) {
    const uint32_t b0 = f2bf(v);
    const float r1 = v - __uint_as_float(b0 << 16);
    const uint32_t b1 = f2bf(r1);
    const float r2 = r1 - __uint_as_float(b1 << 16);
    h = (uint16_t)b0;
    m = (uint16_t)b1;
    l = (uint16_t)f2bf(r2);
}

// element (row j, col k) of a fragment-major plane [16][K] (k_skl / k_skf B operand)
__device__ __forceinline__ size_t frag_off(int j, int k) {  // element (row j, col k) in a plane
    const int b = k >> 6, r = k & 63;
    return ((size_t)(b * 2 + ((r >> 3) & 1)) * 64 + (r >> 4) * 16 + j) * 8 + (r & 7);
}

// element (row j, column n) of a split-K result: the S partial slabs summed in order.  Rows
// come in blocks of 16 (k_skl's B operand): row j's slabs are those of row block j / 16,
// laid out [row block][S][16][N].
__device__ __forceinline__ float psum(const float* __restrict__ part, int S, int N, int j, int n) {
    part += (size_t)(j >> 4) * S * SK_ROWS * N;
    j &= 15;
    float v = part[(size_t)j * N + n];
    // unrolled: four slab loads in flight before their (in-order) adds
#pragma unroll 4
    for (int s = 1; s < S; s++) v += part[((size_t)s * SK_ROWS + j) * N + n];
    return v;
}
// the pair (n, n + 1) of psum (n even), every slab load of a chunk of 8 in flight before
// its adds (same order of additions: slab 0, 1, 2, ...)
__device__ __forceinline__ float2 psum2(const float* __restrict__ part, int S, int N, int j, int n) {
    part += (size_t)(j >> 4) * S * SK_ROWS * N + (size_t)(j & 15) * N + n;
    const size_t stride = (size_t)SK_ROWS * N;
    float2 v = *reinterpret_cast<const float2*>(part);
    for (int s0 = 1; s0 < S; s0 += 8) {
        float2 t[8];
#pragma unroll
        for (int c = 0; c < 8; c++)
            t[c] = s0 + c < S ? *reinterpret_cast<const float2*>(part + (s0 + c) * stride) : make_float2(0.f, 0.f);
#pragma unroll
        for (int c = 0; c < 8; c++)
            if (s0 + c < S) {
                v.x += t[c].x;
                v.y += t[c].y;
            }
    }
    return v;
}
// element (row j, col k) of the fragment-major planes of a row set: plane p of row block j / 16
__device__ __forceinline__ size_t frag_at(int j, int K, int p, int k) {
    return ((size_t)(j >> 4) * 3 + p) * SK_ROWS * K + frag_off(j & 15, k);
}

// dot of 8 bf16 weights (one uint4) with 8 f32 activations
__device__ __forceinline__ float dot8(uint4 w, float4 a, float4 b, float acc) {
    acc = fmaf(bflo(w.x), a.x, acc);
    acc = fmaf(bfhi(w.x), a.y, acc);
    acc = fmaf(bflo(w.y), a.z, acc);
    acc = fmaf(bfhi(w.y), a.w, acc);
    acc = fmaf(bflo(w.z), b.x, acc);
    acc = fmaf(bfhi(w.z), b.y, acc);
    acc = fmaf(bflo(w.w), b.z, acc);
    acc = fmaf(bfhi(w.w), b.w, acc);
    return acc;
}

// dot of 16 int8 weights (one uint4, Q8 rows) with 16 f32 activations: each byte is
// sign-extended and converted exactly (q8_matvec_fused, voxtral_kernels.c:277-318)
__device__ __forceinline__ float i8f(uint32_t w, int b) { return (float)((int32_t)(w << (24 - 8 * b)) >> 24); }
__device__ __forceinline__ float dot16q(uint4 w, const float4 (&x)[4], float acc) {
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        acc = fmaf(i8f(d[k], 0), x[k].x, acc);
        acc = fmaf(i8f(d[k], 1), x[k].y, acc);
        acc = fmaf(i8f(d[k], 2), x[k].z, acc);
        acc = fmaf(i8f(d[k], 3), x[k].w, acc);
    }
    return acc;
}

}  // namespace vox
