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
