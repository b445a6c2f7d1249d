/*
 * vox_synth.c -- deterministic synthetic weights and inputs.
 *
 * The real Voxtral-Mini-4B-Realtime checkpoint is not available offline, so tests and
 * the benchmark use seeded random weights of the exact architecture (same tensor names,
 * shapes and dtype => same bytes and FLOPs).  Values are a counter-based hash
 * (splitmix64) of (seed, element index), so any slice can be generated independently
 * and in parallel; they are uniform with the requested standard deviation.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static inline float unif(uint64_t seed, uint64_t i) {
    uint64_t h = splitmix64(seed ^ splitmix64(i));
    return (float)((h >> 40) * (1.0 / 16777216.0)) * 2.0f - 1.0f; /* [-1, 1) */
}

/* bf16 bits of offset + std * sqrt(3) * U[-1,1), round-to-nearest-even */
void vox_synth_bf16(uint16_t *out, size_t n, uint64_t seed, float std, float offset) {
    const float a = std * 1.7320508075688772f;
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < (long long)n; i++) {
        float v = offset + a * unif(seed, (uint64_t)i);
        uint32_t u;
        memcpy(&u, &v, 4);
        u += 0x7fffu + ((u >> 16) & 1u);
        out[i] = (uint16_t)(u >> 16);
    }
}

void vox_synth_f32(float *out, size_t n, uint64_t seed, float lo, float hi) {
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < (long long)n; i++) {
        float u = 0.5f * (unif(seed, (uint64_t)i) + 1.0f);
        out[i] = lo + (hi - lo) * u;
    }
}

/* bf16 -> f32 (exact) */
void vox_bf16_to_f32(float *out, const uint16_t *in, size_t n) {
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < (long long)n; i++) {
        uint32_t u = ((uint32_t)in[i]) << 16;
        memcpy(&out[i], &u, 4);
    }
}

/* Per-row symmetric int8 quantisation of a bf16 [rows, cols] matrix, restating the
 * reference's quantize.py:35-46 (quantize_q8_row) and :96-125: amax = max|row| in f32;
 * scale = f32(amax / 127.0 in double); q = round-half-even(row / scale) in f32, clipped to
 * [-128, 127]; an all-zero row gets scale 0 and zeros.  Output layout as quantize.py
 * writes it (safetensors.c:393-408): scales [rows] f32, then q [rows, cols] int8. */
void vox_quantize_q8_bf16(const uint16_t *in, long long rows, long long cols, float *scales,
                          int8_t *q) {
#pragma omp parallel for schedule(dynamic, 16)
    for (long long r = 0; r < rows; r++) {
        const uint16_t *src = in + r * cols;
        int8_t *dst = q + r * cols;
        float amax = 0.0f;
        for (long long c = 0; c < cols; c++) {
            uint32_t u = ((uint32_t)src[c]) << 16;
            float v;
            memcpy(&v, &u, 4);
            v = fabsf(v);
            if (v > amax) amax = v;
        }
        if (amax == 0.0f) {
            scales[r] = 0.0f;
            memset(dst, 0, (size_t)cols);
            continue;
        }
        const float s = (float)((double)amax / 127.0);
        scales[r] = s;
        for (long long c = 0; c < cols; c++) {
            uint32_t u = ((uint32_t)src[c]) << 16;
            float v;
            memcpy(&v, &u, 4);
            float t = rintf(v / s);
            t = t < -128.0f ? -128.0f : (t > 127.0f ? 127.0f : t);
            dst[c] = (int8_t)t;
        }
    }
}

/* (float)q * scale per row: safetensors_get_f32 of a Q8 tensor (safetensors.c:393-408) */
void vox_dequant_q8(float *out, const int8_t *q, const float *scales, long long rows, long long cols) {
#pragma omp parallel for schedule(static)
    for (long long r = 0; r < rows; r++)
        for (long long c = 0; c < cols; c++) out[r * cols + c] = (float)q[r * cols + c] * scales[r];
}
