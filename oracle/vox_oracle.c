/*
 * vox_oracle.c -- TEST INFRASTRUCTURE ONLY (see vox_oracle.h).
 *
 * CPU restatement of the reference CPU/BLAS path.  M>1 linears go through the same
 * cblas sgemm call the reference makes (voxtral_kernels.c:90-101), bound here to the
 * OpenBLAS that ships inside scipy (the image has no cblas.h; the prototype below is
 * this file's own declaration of that library's exported symbol).  M=1 linears are the
 * scalar fused bf16 matvec of voxtral_kernels.c:154-195.
 */
#include "vox_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* scipy's bundled OpenBLAS (libscipy_openblas-*.so) exports prefixed cblas symbols. */
extern void scipy_cblas_sgemm(int order, int transa, int transb, int M, int N, int K,
                              float alpha, const float *A, int lda, const float *B, int ldb,
                              float beta, float *C, int ldc);
extern void scipy_openblas_set_num_threads(int n);
enum { RowMajor = 101, NoTrans = 111, Trans = 112 };

#define TOKEN_BOS 1
#define TOKEN_EOS 2
#define TOKEN_STREAMING_PAD 32

static int g_threads = 1;
/* test-only invariance knob (tests/test_oracle_cpu.py): 1 = never compact the KV caches
 * (grow instead), so a run with physical compaction can be compared with one without */
static int g_no_compact = 0;
void vo_set_no_compaction(int on) { g_no_compact = on; }

/* The fp16 decoder KV cache (VOX_DECODER_KV_FP16, voxtral.c:189-190): the Metal path stores
 * K (after RoPE) and V as IEEE half and attention reads them back widened to f32
 * (voxtral_decoder.c:151-178 f16_to_f32; the store is the shader's half(x), round to nearest
 * even).  Restated as a rounding of every value appended to the decoder cache. */
static int g_kv_fp16 = 0;
void vo_set_kv_fp16(int on) { g_kv_fp16 = on; }

/* f32 -> IEEE half (round to nearest even, subnormals kept, overflow to inf) -> f32 */
static float f16_round(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = x & 0x80000000u, ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return f;                 /* inf / nan */
    if (ax >= 0x477ff000u) {                         /* >= 65520: rounds past 65504 */
        uint32_t r = sign | 0x7f800000u;
        float o;
        memcpy(&o, &r, 4);
        return o;
    }
    if (ax < 0x38800000u) {                          /* below 2^-14: multiples of 2^-24 */
        float a = fabsf(f) * 16777216.0f;            /* exact (power of two), < 1024 */
        float q = rintf(a) / 16777216.0f;            /* rintf: nearest even (default mode) */
        return sign ? -q : q;
    }
    uint32_t r = ax + 0xfffu + ((ax >> 13) & 1u);    /* 13 dropped mantissa bits, ties to even */
    r = (r & ~0x1fffu) | sign;
    float o;
    memcpy(&o, &r, 4);
    return o;
}
void vo_f16_round(const float *x, int n, float *out) { for (int i = 0; i < n; i++) out[i] = f16_round(x[i]); }

void vo_set_threads(int n) {
    g_threads = n < 1 ? 1 : n;
    scipy_openblas_set_num_threads(g_threads);
}

static inline float bf16f(uint16_t v) {
    uint32_t u = ((uint32_t)v) << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* ------------------------------------------------------------------------
 * Linear layers (voxtral_kernels.c:154-240)
 * ------------------------------------------------------------------------ */

/* bf16_matvec_fused, voxtral_kernels.c:154-195 (scalar path: sum starts at bias,
 * accumulates w*x in k order). Rows are independent, so threading over rows keeps the
 * per-row arithmetic identical. */
static void matvec_bf16(float *y, const float *x, const uint16_t *W, const float *bias,
                        int in_dim, int out_dim) {
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int o = 0; o < out_dim; o++) {
        const uint16_t *w = W + (size_t)o * in_dim;
        /* The reference is built with -ffast-math (Makefile:13), which lets gcc vectorise
         * this reduction; a SIMD reduction reproduces that (same math, reassociated). */
        float sum = 0.0f;
#pragma omp simd reduction(+ : sum)
        for (int k = 0; k < in_dim; k++) sum += bf16f(w[k]) * x[k];
        y[o] = (bias ? bias[o] : 0.0f) + sum;
    }
}

static float *g_scratch = NULL;
static size_t g_scratch_cap = 0;

/* vox_linear_bf16 / vox_linear_nobias_bf16 (voxtral_kernels.c:197-240): M==1 fused
 * matvec; M>1 converts the whole matrix to f32 scratch (bf16_to_f32_buf, :124-128) and
 * calls sgemm(NoTrans, Trans), then adds the bias row-wise (:90-101). */
void vo_linear_bf16(float *y, const float *x, const uint16_t *W, const float *b,
                    int M, int in_dim, int out_dim) {
    if (M <= 0) return;
    if (M == 1) { matvec_bf16(y, x, W, b, in_dim, out_dim); return; }
    size_t n = (size_t)out_dim * in_dim;
    if (n > g_scratch_cap) {
        free(g_scratch);
        g_scratch = (float *)malloc(n * sizeof(float));
        g_scratch_cap = g_scratch ? n : 0;
    }
    uint32_t *d = (uint32_t *)(void *)g_scratch;
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (size_t i = 0; i < n; i++) d[i] = ((uint32_t)W[i]) << 16;
    scipy_cblas_sgemm(RowMajor, NoTrans, Trans, M, out_dim, in_dim, 1.0f, x, in_dim,
                      g_scratch, in_dim, 0.0f, y, out_dim);
    if (b) {
        for (int s = 0; s < M; s++)
            for (int o = 0; o < out_dim; o++) y[(size_t)s * out_dim + o] += b[o];
    }
}

/* q8_matvec_fused, voxtral_kernels.c:277-318 (non-NEON path): sum of int8->f32 weight
 * times x in k order from 0, then y = sum * scale + bias. */
static void matvec_q8(float *y, const float *x, const int8_t *W, const float *scales,
                      const float *bias, int in_dim, int out_dim) {
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int o = 0; o < out_dim; o++) {
        const int8_t *w = W + (size_t)o * in_dim;
        float sum = 0.0f;
#pragma omp simd reduction(+ : sum)
        for (int k = 0; k < in_dim; k++) sum += (float)w[k] * x[k];
        y[o] = sum * scales[o] + (bias ? bias[o] : 0.0f);
    }
}

/* vox_linear_q8 / vox_linear_nobias_q8 / vox_matmul_t_q8 (voxtral_kernels.c:320-393):
 * M==1 fused matvec; M>1 dequantises W[r][c] = (float)q * scale[r] into f32 scratch and
 * takes the f32 sgemm path (vox_linear / vox_linear_nobias / vox_matmul_t). */
void vo_linear_q8(float *y, const float *x, const int8_t *W, const float *scales, const float *b,
                  int M, int in_dim, int out_dim) {
    if (M <= 0) return;
    if (M == 1) { matvec_q8(y, x, W, scales, b, in_dim, out_dim); return; }
    size_t n = (size_t)out_dim * in_dim;
    if (n > g_scratch_cap) {
        free(g_scratch);
        g_scratch = (float *)malloc(n * sizeof(float));
        g_scratch_cap = g_scratch ? n : 0;
    }
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int r = 0; r < out_dim; r++) {
        const float sc = scales[r];
        for (int c = 0; c < in_dim; c++) g_scratch[(size_t)r * in_dim + c] = (float)W[(size_t)r * in_dim + c] * sc;
    }
    scipy_cblas_sgemm(RowMajor, NoTrans, Trans, M, out_dim, in_dim, 1.0f, x, in_dim,
                      g_scratch, in_dim, 0.0f, y, out_dim);
    if (b) {
        for (int s = 0; s < M; s++)
            for (int o = 0; o < out_dim; o++) y[(size_t)s * out_dim + o] += b[o];
    }
}

/* bf16 or q8 by the presence of a scale array (the reference branches on *_weight_q8) */
static void lin(float *y, const float *x, const uint16_t *W, const float *scales, const float *b,
                int M, int in_dim, int out_dim) {
    if (scales) vo_linear_q8(y, x, (const int8_t *)(const void *)W, scales, b, M, in_dim, out_dim);
    else vo_linear_bf16(y, x, W, b, M, in_dim, out_dim);
}
#define SC(field, l) (w->field ? w->field[l] : NULL)

/* ------------------------------------------------------------------------
 * Element-wise / normalisation (voxtral_kernels.c:475-513)
 * ------------------------------------------------------------------------ */

void vo_rms_norm(float *out, const float *x, const float *w, int M, int hidden, float eps) {
    for (int s = 0; s < M; s++) {
        const float *xr = x + (size_t)s * hidden;
        float *orow = out + (size_t)s * hidden;
        float sum_sq = 0.0f;
        for (int i = 0; i < hidden; i++) sum_sq += xr[i] * xr[i];
        float rms = sqrtf(sum_sq / hidden + eps);
        float inv = 1.0f / rms;
        for (int i = 0; i < hidden; i++) orow[i] = xr[i] * inv * w[i];
    }
}

void vo_silu(float *x, int n) {
    for (int i = 0; i < n; i++) {
        float v = x[i];
        x[i] = v / (1.0f + expf(-v));
    }
}

void vo_gelu(float *x, int n, int erf_mode) {
    if (erf_mode) { /* python_simple_implementation.py F.gelu (exact) */
        for (int i = 0; i < n; i++) {
            float v = x[i];
            x[i] = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
        }
        return;
    }
    for (int i = 0; i < n; i++) { /* voxtral_kernels.c:505-513 */
        float v = x[i];
        float x3 = v * v * v;
        float inner = 0.7978845608028654f * (v + 0.044715f * x3);
        x[i] = 0.5f * v * (1.0f + tanhf(inner));
    }
}

/* ------------------------------------------------------------------------
 * Causal conv1d, im2col + sgemm (voxtral_kernels.c:422-469)
 * ------------------------------------------------------------------------ */
void vo_causal_conv1d(float *out, const float *in, const float *w, const float *b,
                      int cin, int cout, int length, int ks, int stride) {
    int padding_total = ks - stride;
    float n_frames = ((float)length - ks + padding_total) / (float)stride + 1.0f;
    int out_len = (int)ceilf(n_frames);
    if (out_len <= 0) return;
    int left_pad = padding_total;
    int K = cin * ks;
    float *im2col = (float *)calloc((size_t)K * out_len, sizeof(float));
    for (int ol = 0; ol < out_len; ol++)
        for (int ic = 0; ic < cin; ic++)
            for (int k = 0; k < ks; k++) {
                int il = ol * stride - left_pad + k;
                if (il >= 0 && il < length)
                    im2col[(size_t)(ic * ks + k) * out_len + ol] = in[(size_t)ic * length + il];
            }
    scipy_cblas_sgemm(RowMajor, NoTrans, NoTrans, cout, out_len, K, 1.0f, w, K, im2col,
                      out_len, 0.0f, out, out_len);
    free(im2col);
    if (b) {
        for (int oc = 0; oc < cout; oc++) {
            float *row = out + (size_t)oc * out_len;
            for (int ol = 0; ol < out_len; ol++) row[ol] += b[oc];
        }
    }
}

/* ------------------------------------------------------------------------
 * Attention with online softmax (voxtral_kernels.c:541-611)
 * ------------------------------------------------------------------------ */
void vo_causal_attention(float *out, const float *Q, const float *K, const float *V,
                         int seq_q, int seq_k, int n_heads, int n_kv_heads, int head_dim,
                         float scale, int window, int q_offset) {
    int hpk = n_heads / n_kv_heads;
    int qh = n_heads * head_dim, kvh = n_kv_heads * head_dim;
#pragma omp parallel for collapse(2) schedule(static) num_threads(g_threads) if (g_threads > 1)
    for (int h = 0; h < n_heads; h++) {
        for (int i = 0; i < seq_q; i++) {
            int kv_h = h / hpk;
            const float *q = Q + (size_t)i * qh + (size_t)h * head_dim;
            float *o = out + (size_t)i * qh + (size_t)h * head_dim;
            int gp = q_offset + i;
            int k_start = 0;
            if (window > 0 && gp - window + 1 > 0) k_start = gp - window + 1;
            int k_end = gp + 1;
            if (k_end > seq_k) k_end = seq_k;
            float max_score = -1e30f, sum_exp = 0.0f;
            for (int d = 0; d < head_dim; d++) o[d] = 0.0f;
            for (int j = k_start; j < k_end; j++) {
                const float *kr = K + (size_t)j * kvh + (size_t)kv_h * head_dim;
                const float *vr = V + (size_t)j * kvh + (size_t)kv_h * head_dim;
                float score = 0.0f;
                for (int d = 0; d < head_dim; d++) score += q[d] * kr[d];
                score *= scale;
                if (score > max_score) {
                    float corr = expf(max_score - score);
                    sum_exp = sum_exp * corr + 1.0f;
                    for (int d = 0; d < head_dim; d++) o[d] = o[d] * corr + vr[d];
                    max_score = score;
                } else {
                    float wgt = expf(score - max_score);
                    sum_exp += wgt;
                    for (int d = 0; d < head_dim; d++) o[d] += wgt * vr[d];
                }
            }
            if (sum_exp > 0.0f) {
                float inv = 1.0f / sum_exp;
                for (int d = 0; d < head_dim; d++) o[d] *= inv;
            }
        }
    }
}

/* RoPE (voxtral_kernels.c:617-655): interleaved pairs, freqs from float powf. */
void vo_rope_freqs(float *freqs, const int *pos, int seq, int dim, float theta) {
    int half = dim / 2;
    for (int s = 0; s < seq; s++) {
        float p = (float)pos[s];
        for (int d = 0; d < half; d++) {
            float freq = 1.0f / powf(theta, (float)(2 * d) / (float)dim);
            float angle = p * freq;
            freqs[(size_t)s * half * 2 + d * 2] = cosf(angle);
            freqs[(size_t)s * half * 2 + d * 2 + 1] = sinf(angle);
        }
    }
}

void vo_apply_rope(float *x, const float *freqs, int seq, int heads, int head_dim) {
    int half = head_dim / 2, hidden = heads * head_dim;
    for (int s = 0; s < seq; s++)
        for (int h = 0; h < heads; h++) {
            float *v = x + (size_t)s * hidden + (size_t)h * head_dim;
            for (int d = 0; d < half; d++) {
                float c = freqs[(size_t)s * half * 2 + d * 2];
                float sn = freqs[(size_t)s * half * 2 + d * 2 + 1];
                float x0 = v[d * 2], x1 = v[d * 2 + 1];
                v[d * 2] = x0 * c - x1 * sn;
                v[d * 2 + 1] = x0 * sn + x1 * c;
            }
        }
}

/* TimeEmbedding (voxtral.c:31-45). */
void vo_time_embedding(float *out, int dim, float t) {
    int half = dim / 2;
    float log_theta = logf(10000.0f);
    for (int i = 0; i < half; i++) {
        float inv_freq = expf(-log_theta * (float)i / (float)half);
        float emb = t * inv_freq;
        out[i] = cosf(emb);
        out[i + half] = sinf(emb);
    }
}

/* ------------------------------------------------------------------------
 * Model
 * ------------------------------------------------------------------------ */
struct vo_model {
    vo_config_t c;
    vo_weights_t w;
    int delay_tokens;
    float *ada_scale; /* [dec_layers * dec_dim] */
};

/* vox_update_time_conditioning (voxtral.c:47-80) */
static void update_time_conditioning(vo_model_t *m) {
    const vo_config_t *c = &m->c;
    int D = c->dec_dim, A = c->ada_dim;
    float *t_cond = (float *)malloc(sizeof(float) * D);
    float *hidden = (float *)malloc(sizeof(float) * A);
    vo_time_embedding(t_cond, D, (float)m->delay_tokens);
    for (int l = 0; l < c->dec_layers; l++) {
        const float *down = m->w.dec_ada_down[l], *up = m->w.dec_ada_up[l];
        for (int i = 0; i < A; i++) {
            float sum = 0.0f;
            for (int j = 0; j < D; j++) sum += down[(size_t)i * D + j] * t_cond[j];
            hidden[i] = sum;
        }
        vo_gelu(hidden, A, c->gelu_erf);
        float *sc = m->ada_scale + (size_t)l * D;
        for (int i = 0; i < D; i++) {
            float sum = 0.0f;
            for (int j = 0; j < A; j++) sum += up[(size_t)i * A + j] * hidden[j];
            sc[i] = sum;
        }
    }
    free(t_cond);
    free(hidden);
}

vo_model_t *vo_model_create(const vo_config_t *cfg, const vo_weights_t *w, int delay_tokens) {
    vo_model_t *m = (vo_model_t *)calloc(1, sizeof(*m));
    m->c = *cfg;
    m->w = *w;
    m->delay_tokens = delay_tokens;
    m->ada_scale = (float *)malloc(sizeof(float) * (size_t)cfg->dec_layers * cfg->dec_dim);
    update_time_conditioning(m);
    return m;
}

void vo_model_set_delay(vo_model_t *m, int delay_tokens) {
    m->delay_tokens = delay_tokens;
    update_time_conditioning(m);
}

const float *vo_model_ada_scale(const vo_model_t *m) { return m->ada_scale; }

void vo_model_free(vo_model_t *m) {
    if (!m) return;
    free(m->ada_scale);
    free(m);
}

/* ------------------------------------------------------------------------
 * Stream state (voxtral.c:457-522 + the KV fields of vox_ctx_t, voxtral.h:197-238)
 * ------------------------------------------------------------------------ */
struct vo_stream {
    vo_model_t *m;
    /* encoder KV cache: [L][max][kv_dim], physical rows + logical offset */
    float *ek, *ev;
    int e_len, e_max, e_off;
    /* decoder KV cache */
    float *dk, *dv;
    int d_len, d_max, d_off;
    /* conv stem state */
    float *mel_tail, *conv0_tail, *conv0_res;
    int conv0_res_count, conv_init;
    /* downsample residual */
    float *enc_res;
    int enc_res_count;
    /* adapter buffer */
    float *adapter;
    int total_adapter, adapter_cap;
    /* decoder */
    int started, gen_pos, prev_token, eos_seen, n_generated;
};

vo_stream_t *vo_stream_create(vo_model_t *m) {
    vo_stream_t *s = (vo_stream_t *)calloc(1, sizeof(*s));
    const vo_config_t *c = &m->c;
    s->m = m;
    s->mel_tail = (float *)calloc((size_t)c->mel_bins * 2, sizeof(float));
    s->conv0_tail = (float *)calloc((size_t)c->enc_dim * 2, sizeof(float));
    s->conv0_res = (float *)calloc((size_t)c->enc_dim, sizeof(float));
    s->enc_res = (float *)calloc((size_t)c->enc_dim * (c->downsample - 1), sizeof(float));
    s->prev_token = TOKEN_BOS;
    return s;
}

void vo_stream_free(vo_stream_t *s) {
    if (!s) return;
    free(s->ek); free(s->ev); free(s->dk); free(s->dv);
    free(s->mel_tail); free(s->conv0_tail); free(s->conv0_res); free(s->enc_res);
    free(s->adapter);
    free(s);
}

/* stream_reset_decoder_state (voxtral.c:766-783): KV length 0, adapter backlog dropped */
void vo_stream_reset_decoder(vo_stream_t *s) {
    s->d_len = 0;
    s->d_off = 0;
    s->total_adapter = 0;
    s->gen_pos = 0;
    s->started = 0;
    s->prev_token = TOKEN_BOS;
    s->eos_seen = 0;
    s->n_generated = 0;
}

/* stream_reset_full_state (voxtral.c:786-814) minus the mel context (the caller's) */
void vo_stream_reset_full(vo_stream_t *s) {
    const vo_config_t *c = &s->m->c;
    s->conv_init = 0;
    s->conv0_res_count = 0;
    s->enc_res_count = 0;
    memset(s->mel_tail, 0, sizeof(float) * (size_t)c->mel_bins * 2);
    memset(s->conv0_tail, 0, sizeof(float) * (size_t)c->enc_dim * 2);
    memset(s->conv0_res, 0, sizeof(float) * (size_t)c->enc_dim);
    memset(s->enc_res, 0, sizeof(float) * (size_t)c->enc_dim * (c->downsample - 1));
    s->e_len = 0;
    s->e_off = 0;
    vo_stream_reset_decoder(s);
}

void vo_stream_state(const vo_stream_t *s, int *o) {
    o[0] = s->e_len; o[1] = s->e_off; o[2] = s->d_len; o[3] = s->d_off;
    o[4] = s->total_adapter; o[5] = s->gen_pos; o[6] = s->enc_res_count; o[7] = s->conv0_res_count;
}

/* ------------------------------------------------------------------------
 * Conv stem, incremental (voxtral.c:581-759)
 * ------------------------------------------------------------------------ */
static void gelu_m(vo_model_t *m, float *x, int n) { vo_gelu(x, n, m->c.gelu_erf); }

int vo_conv_stem(vo_stream_t *s, const float *mel_new, int n_new, float *out, int out_cap) {
    vo_model_t *m = s->m;
    const vo_config_t *c = &m->c;
    int dim = c->enc_dim, MB = c->mel_bins;
    if (n_new <= 0) return 0;
    int is_first = 0;
    int c0_len = n_new;
    float *c0_new = (float *)malloc(sizeof(float) * (size_t)dim * c0_len);

    if (!s->conv_init) {
        is_first = 1;
        float *cin = (float *)malloc(sizeof(float) * (size_t)MB * n_new);
        for (int f = 0; f < n_new; f++)
            for (int b = 0; b < MB; b++) cin[(size_t)b * n_new + f] = mel_new[(size_t)f * MB + b];
        vo_causal_conv1d(c0_new, cin, m->w.conv0_w, m->w.conv0_b, MB, dim, n_new, 3, 1);
        gelu_m(m, c0_new, dim * c0_len);
        free(cin);
        s->conv_init = 1;
    } else {
        int plen = 2 + n_new;
        float *cin = (float *)malloc(sizeof(float) * (size_t)MB * plen);
        for (int b = 0; b < MB; b++) {
            cin[(size_t)b * plen + 0] = s->mel_tail[b * 2 + 0];
            cin[(size_t)b * plen + 1] = s->mel_tail[b * 2 + 1];
            for (int f = 0; f < n_new; f++)
                cin[(size_t)b * plen + 2 + f] = mel_new[(size_t)f * MB + b];
        }
        float *full = (float *)malloc(sizeof(float) * (size_t)dim * plen);
        vo_causal_conv1d(full, cin, m->w.conv0_w, m->w.conv0_b, MB, dim, plen, 3, 1);
        gelu_m(m, full, dim * plen);
        free(cin);
        for (int d = 0; d < dim; d++)
            memcpy(c0_new + (size_t)d * c0_len, full + (size_t)d * plen + 2, sizeof(float) * c0_len);
        free(full);
    }
    /* mel tail (last 2 frames, column-major [MB,2]) */
    {
        int ts = n_new >= 2 ? n_new - 2 : 0, tc = n_new >= 2 ? 2 : n_new;
        memset(s->mel_tail, 0, sizeof(float) * MB * 2);
        for (int f = 0; f < tc; f++)
            for (int b = 0; b < MB; b++) s->mel_tail[b * 2 + (2 - tc + f)] = mel_new[(size_t)(ts + f) * MB + b];
    }

    /* stride alignment */
    int prev_res = s->conv0_res_count;
    int total = prev_res + c0_len;
    int new_res = total & 1;
    int feed_new = c0_len - new_res;
    int feed_total = prev_res + feed_new;
    if (feed_total <= 0) {
        if (new_res && c0_len > 0)
            for (int d = 0; d < dim; d++) s->conv0_res[d] = c0_new[(size_t)d * c0_len + c0_len - 1];
        s->conv0_res_count = new_res;
        free(c0_new);
        return 0;
    }
    float *feed = (float *)malloc(sizeof(float) * (size_t)dim * feed_total);
    int fpos = 0;
    if (prev_res == 1) {
        for (int d = 0; d < dim; d++) feed[(size_t)d * feed_total] = s->conv0_res[d];
        fpos = 1;
    }
    for (int d = 0; d < dim; d++)
        memcpy(feed + (size_t)d * feed_total + fpos, c0_new + (size_t)d * c0_len, sizeof(float) * feed_new);
    if (new_res)
        for (int d = 0; d < dim; d++) s->conv0_res[d] = c0_new[(size_t)d * c0_len + c0_len - 1];
    s->conv0_res_count = new_res;
    free(c0_new);

    float *c1_in;
    int c1_len, discard;
    if (is_first) {
        c1_in = feed;
        c1_len = feed_total;
        discard = 0;
    } else {
        c1_len = 2 + feed_total;
        c1_in = (float *)malloc(sizeof(float) * (size_t)dim * c1_len);
        for (int d = 0; d < dim; d++) {
            c1_in[(size_t)d * c1_len + 0] = s->conv0_tail[d * 2 + 0];
            c1_in[(size_t)d * c1_len + 1] = s->conv0_tail[d * 2 + 1];
            memcpy(c1_in + (size_t)d * c1_len + 2, feed + (size_t)d * feed_total, sizeof(float) * feed_total);
        }
        discard = 1;
    }
    for (int d = 0; d < dim; d++) {
        s->conv0_tail[d * 2 + 0] = feed[(size_t)d * feed_total + feed_total - 2];
        s->conv0_tail[d * 2 + 1] = feed[(size_t)d * feed_total + feed_total - 1];
    }
    if (!is_first) free(feed);

    int c1_out_len = c1_len / 2;
    float *c1_out = (float *)malloc(sizeof(float) * (size_t)dim * c1_out_len);
    vo_causal_conv1d(c1_out, c1_in, m->w.conv1_w, m->w.conv1_b, dim, dim, c1_len, 3, 2);
    gelu_m(m, c1_out, dim * c1_out_len);
    free(c1_in);
    int res_len = c1_out_len - discard;
    if (res_len <= 0) { free(c1_out); return 0; }
    if (res_len > out_cap) res_len = out_cap;
    for (int i = 0; i < res_len; i++)
        for (int d = 0; d < dim; d++)
            out[(size_t)i * dim + d] = c1_out[(size_t)d * c1_out_len + discard + i];
    free(c1_out);
    return res_len;
}

/* ------------------------------------------------------------------------
 * Encoder, incremental (voxtral_encoder.c:371-693)
 * ------------------------------------------------------------------------ */
static void enc_kv_grow(vo_stream_t *s, int required) {
    const vo_config_t *c = &s->m->c;
    if (s->e_max >= required) return;
    int kvd = c->enc_kv_heads * c->enc_head_dim;
    int nm = s->e_max ? s->e_max : 256;
    while (nm < required) nm *= 2;
    size_t ns = (size_t)nm * kvd;
    float *nk = (float *)calloc((size_t)c->enc_layers * ns, sizeof(float));
    float *nv = (float *)calloc((size_t)c->enc_layers * ns, sizeof(float));
    if (s->e_len > 0 && s->ek) {
        size_t os = (size_t)s->e_max * kvd;
        for (int l = 0; l < c->enc_layers; l++) {
            memcpy(nk + l * ns, s->ek + l * os, sizeof(float) * (size_t)s->e_len * kvd);
            memcpy(nv + l * ns, s->ev + l * os, sizeof(float) * (size_t)s->e_len * kvd);
        }
    }
    free(s->ek); free(s->ev);
    s->ek = nk; s->ev = nv; s->e_max = nm;
}

static void enc_kv_compact(vo_stream_t *s) {
    const vo_config_t *c = &s->m->c;
    int keep = c->enc_window;
    if (s->e_len <= keep) return;
    int discard = s->e_len - keep;
    int kvd = c->enc_kv_heads * c->enc_head_dim;
    size_t stride = (size_t)s->e_max * kvd;
    for (int l = 0; l < c->enc_layers; l++) {
        memmove(s->ek + l * stride, s->ek + l * stride + (size_t)discard * kvd, sizeof(float) * (size_t)keep * kvd);
        memmove(s->ev + l * stride, s->ev + l * stride + (size_t)discard * kvd, sizeof(float) * (size_t)keep * kvd);
    }
    s->e_off += discard;
    s->e_len = keep;
}

int vo_encoder_incremental(vo_stream_t *s, float *x, int new_len) {
    vo_model_t *m = s->m;
    const vo_config_t *c = &m->c;
    const vo_weights_t *w = &m->w;
    int dim = c->enc_dim, H = c->enc_heads, KVH = c->enc_kv_heads, hd = c->enc_head_dim;
    int hidden = c->enc_hidden, qd = H * hd, kvd = KVH * hd;
    if (new_len <= 0) return 0;
    if (s->e_len + new_len > c->enc_window && !g_no_compact) enc_kv_compact(s);
    enc_kv_grow(s, s->e_len + new_len);
    int cache_len = s->e_len;

    float *xn = (float *)malloc(sizeof(float) * (size_t)new_len * dim);
    float *q = (float *)malloc(sizeof(float) * (size_t)new_len * qd);
    float *k = (float *)malloc(sizeof(float) * (size_t)new_len * kvd);
    float *v = (float *)malloc(sizeof(float) * (size_t)new_len * kvd);
    float *att = (float *)malloc(sizeof(float) * (size_t)new_len * qd);
    float *proj = (float *)malloc(sizeof(float) * (size_t)new_len * dim);
    float *gate = (float *)malloc(sizeof(float) * (size_t)new_len * hidden);
    float *up = (float *)malloc(sizeof(float) * (size_t)new_len * hidden);
    int *pos = (int *)malloc(sizeof(int) * new_len);
    float *rope = (float *)malloc(sizeof(float) * (size_t)new_len * hd);
    int logical_start = s->e_off + cache_len;
    for (int i = 0; i < new_len; i++) pos[i] = logical_start + i;
    vo_rope_freqs(rope, pos, new_len, hd, c->rope_theta);
    float scale = 1.0f / sqrtf((float)hd);
    size_t lstride = (size_t)s->e_max * kvd;

    for (int l = 0; l < c->enc_layers; l++) {
        vo_rms_norm(xn, x, w->enc_attn_norm[l], new_len, dim, c->enc_eps);
        lin(q, xn, w->enc_wq[l], SC(enc_wq_s, l), w->enc_wq_b[l], new_len, dim, qd);
        lin(k, xn, w->enc_wk[l], SC(enc_wk_s, l), NULL, new_len, dim, kvd);
        lin(v, xn, w->enc_wv[l], SC(enc_wv_s, l), w->enc_wv_b[l], new_len, dim, kvd);
        vo_apply_rope(q, rope, new_len, H, hd);
        vo_apply_rope(k, rope, new_len, KVH, hd);
        float *kc = s->ek + l * lstride, *vc = s->ev + l * lstride;
        memcpy(kc + (size_t)cache_len * kvd, k, sizeof(float) * (size_t)new_len * kvd);
        memcpy(vc + (size_t)cache_len * kvd, v, sizeof(float) * (size_t)new_len * kvd);
        vo_causal_attention(att, q, kc, vc, new_len, cache_len + new_len, H, KVH, hd, scale,
                            c->enc_window, cache_len);
        lin(proj, att, w->enc_wo[l], SC(enc_wo_s, l), w->enc_wo_b[l], new_len, qd, dim);
        for (size_t i = 0; i < (size_t)new_len * dim; i++) x[i] += proj[i];
        vo_rms_norm(xn, x, w->enc_ffn_norm[l], new_len, dim, c->enc_eps);
        lin(gate, xn, w->enc_w1[l], SC(enc_w1_s, l), NULL, new_len, dim, hidden);
        vo_silu(gate, new_len * hidden);
        lin(up, xn, w->enc_w3[l], SC(enc_w3_s, l), NULL, new_len, dim, hidden);
        for (size_t i = 0; i < (size_t)new_len * hidden; i++) gate[i] *= up[i];
        lin(proj, gate, w->enc_w2[l], SC(enc_w2_s, l), w->enc_w2_b[l], new_len, hidden, dim);
        for (size_t i = 0; i < (size_t)new_len * dim; i++) x[i] += proj[i];
    }
    vo_rms_norm(x, x, w->enc_norm, new_len, dim, c->enc_eps);
    s->e_len = cache_len + new_len;
    free(xn); free(q); free(k); free(v); free(att); free(proj); free(gate); free(up);
    free(pos); free(rope);
    return new_len;
}

/* vox_adapter_forward (voxtral_encoder.c:699-737): 4 consecutive rows are already a
 * contiguous [4*enc_dim] row in [rows, enc_dim] layout. */
int vo_adapter(vo_model_t *m, const float *enc, int enc_rows, float *out) {
    const vo_config_t *c = &m->c;
    int ds = enc_rows / c->downsample, dsd = c->enc_dim * c->downsample, D = c->dec_dim;
    if (ds <= 0) return 0;
    float *mid = (float *)malloc(sizeof(float) * (size_t)ds * D);
    lin(mid, enc, m->w.ad0, m->w.ad0_s, NULL, ds, dsd, D);
    gelu_m(m, mid, ds * D);
    lin(out, mid, m->w.ad1, m->w.ad1_s, NULL, ds, D, D);
    free(mid);
    return ds;
}

static void adapter_append(vo_stream_t *s, const float *rows, int n) {
    int D = s->m->c.dec_dim;
    if (s->total_adapter + n > s->adapter_cap) {
        int nc = s->adapter_cap ? s->adapter_cap * 2 : 256;
        while (nc < s->total_adapter + n) nc *= 2;
        s->adapter = (float *)realloc(s->adapter, sizeof(float) * (size_t)nc * D);
        s->adapter_cap = nc;
    }
    memcpy(s->adapter + (size_t)s->total_adapter * D, rows, sizeof(float) * (size_t)n * D);
    s->total_adapter += n;
}

/* stream_run_encoder (voxtral.c:827-951), from the conv stem on. */
int vo_stream_encode_mel(vo_stream_t *s, const float *mel, int n_frames) {
    vo_model_t *m = s->m;
    const vo_config_t *c = &m->c;
    int ed = c->enc_dim, DS = c->downsample;
    if (n_frames <= 0) return 0;
    int cap = n_frames / 2 + 4;
    float *conv = (float *)malloc(sizeof(float) * (size_t)cap * ed);
    int conv_len = vo_conv_stem(s, mel, n_frames, conv, cap);
    if (conv_len <= 0) { free(conv); return 0; }
    vo_encoder_incremental(s, conv, conv_len);
    int total = s->enc_res_count + conv_len;
    int usable = (total / DS) * DS;
    int leftover = total - usable;
    int added = 0;
    if (usable > 0) {
        float *comb = (float *)malloc(sizeof(float) * (size_t)usable * ed);
        int p = 0;
        if (s->enc_res_count > 0) {
            int fr = s->enc_res_count < usable ? s->enc_res_count : usable;
            memcpy(comb, s->enc_res, sizeof(float) * (size_t)fr * ed);
            p = fr;
        }
        int from_enc = usable - p;
        if (from_enc > 0) memcpy(comb + (size_t)p * ed, conv, sizeof(float) * (size_t)from_enc * ed);
        float *ad = (float *)malloc(sizeof(float) * (size_t)(usable / DS) * c->dec_dim);
        added = vo_adapter(m, comb, usable, ad);
        adapter_append(s, ad, added);
        free(ad);
        free(comb);
    }
    if (leftover > 0 && usable > 0) {
        int enc_used = usable - s->enc_res_count;
        memcpy(s->enc_res, conv + (size_t)enc_used * ed, sizeof(float) * (size_t)leftover * ed);
    } else if (leftover > 0) {
        /* Deviation (DESIGN.md "Known reference defects"): with usable == 0 the reference
         * copies `leftover` rows from enc_out although enc_out holds only conv_len of them
         * (voxtral.c:923-930, a heap over-read); the intended result -- old residual rows
         * followed by the new rows -- is kept instead. */
        memcpy(s->enc_res + (size_t)s->enc_res_count * ed, conv, sizeof(float) * (size_t)conv_len * ed);
    }
    s->enc_res_count = leftover;
    free(conv);
    return added;
}

int vo_stream_adapter_tokens(const vo_stream_t *s) { return s->total_adapter; }
const float *vo_stream_adapter(const vo_stream_t *s) { return s->adapter; }

/* ------------------------------------------------------------------------
 * Decoder (voxtral_decoder.c:208-780)
 * ------------------------------------------------------------------------ */
static int dec_kv_dim(const vo_config_t *c) { return c->dec_kv_heads * c->dec_head_dim; }

static void dec_kv_init(vo_stream_t *s, int max_seq) { /* kv_cache_init, decoder.c:208-249 */
    const vo_config_t *c = &s->m->c;
    size_t n = (size_t)c->dec_layers * max_seq * dec_kv_dim(c);
    free(s->dk); free(s->dv);
    s->dk = (float *)calloc(n, sizeof(float));
    s->dv = (float *)calloc(n, sizeof(float));
    s->d_len = 0;
    s->d_max = max_seq;
}

static void dec_kv_grow(vo_stream_t *s, int required) { /* kv_cache_grow, decoder.c:257-348 */
    const vo_config_t *c = &s->m->c;
    if (required <= s->d_max) return;
    int kvd = dec_kv_dim(c);
    int nm = s->d_max;
    while (nm < required) nm *= 2;
    size_t ns = (size_t)nm * kvd, os = (size_t)s->d_max * kvd;
    float *nk = (float *)calloc((size_t)c->dec_layers * ns, sizeof(float));
    float *nv = (float *)calloc((size_t)c->dec_layers * ns, sizeof(float));
    for (int l = 0; l < c->dec_layers; l++) {
        memcpy(nk + l * ns, s->dk + l * os, sizeof(float) * (size_t)s->d_len * kvd);
        memcpy(nv + l * ns, s->dv + l * os, sizeof(float) * (size_t)s->d_len * kvd);
    }
    free(s->dk); free(s->dv);
    s->dk = nk; s->dv = nv; s->d_max = nm;
}

static void dec_kv_compact(vo_stream_t *s) { /* kv_cache_compact, decoder.c:354-384 */
    const vo_config_t *c = &s->m->c;
    int keep = c->dec_window;
    if (s->d_len <= keep) return;
    int discard = s->d_len - keep, kvd = dec_kv_dim(c);
    size_t stride = (size_t)s->d_max * kvd;
    for (int l = 0; l < c->dec_layers; l++) {
        memmove(s->dk + l * stride, s->dk + l * stride + (size_t)discard * kvd, sizeof(float) * (size_t)keep * kvd);
        memmove(s->dv + l * stride, s->dv + l * stride + (size_t)discard * kvd, sizeof(float) * (size_t)keep * kvd);
    }
    s->d_off += discard;
    s->d_len = keep;
}

/* One decoder layer stack over seq rows starting at physical start_pos (shared by
 * prefill, decoder.c:496-606, and forward, decoder.c:707-746). */
static void dec_layers(vo_stream_t *s, float *x, int seq, int start_pos, const float *rope) {
    vo_model_t *m = s->m;
    const vo_config_t *c = &m->c;
    const vo_weights_t *w = &m->w;
    int D = c->dec_dim, H = c->dec_heads, KVH = c->dec_kv_heads, hd = c->dec_head_dim;
    int hidden = c->dec_hidden, qd = H * hd, kvd = KVH * hd;
    float *xn = (float *)malloc(sizeof(float) * (size_t)seq * D);
    float *q = (float *)malloc(sizeof(float) * (size_t)seq * qd);
    float *k = (float *)malloc(sizeof(float) * (size_t)seq * kvd);
    float *v = (float *)malloc(sizeof(float) * (size_t)seq * kvd);
    float *att = (float *)malloc(sizeof(float) * (size_t)seq * qd);
    float *proj = (float *)malloc(sizeof(float) * (size_t)seq * D);
    float *gate = (float *)malloc(sizeof(float) * (size_t)seq * hidden);
    float *up = (float *)malloc(sizeof(float) * (size_t)seq * hidden);
    float scale = 1.0f / sqrtf((float)hd);
    size_t lstride = (size_t)s->d_max * kvd;
    for (int l = 0; l < c->dec_layers; l++) {
        vo_rms_norm(xn, x, w->dec_attn_norm[l], seq, D, c->dec_eps);
        lin(q, xn, w->dec_wq[l], SC(dec_wq_s, l), NULL, seq, D, qd);
        lin(k, xn, w->dec_wk[l], SC(dec_wk_s, l), NULL, seq, D, kvd);
        lin(v, xn, w->dec_wv[l], SC(dec_wv_s, l), NULL, seq, D, kvd);
        vo_apply_rope(q, rope, seq, H, hd);
        vo_apply_rope(k, rope, seq, KVH, hd);
        float *kc = s->dk + l * lstride, *vc = s->dv + l * lstride;
        if (g_kv_fp16)
            for (size_t i = 0; i < (size_t)seq * kvd; i++) { k[i] = f16_round(k[i]); v[i] = f16_round(v[i]); }
        memcpy(kc + (size_t)start_pos * kvd, k, sizeof(float) * (size_t)seq * kvd);
        memcpy(vc + (size_t)start_pos * kvd, v, sizeof(float) * (size_t)seq * kvd);
        vo_causal_attention(att, q, kc, vc, seq, start_pos + seq, H, KVH, hd, scale,
                            c->dec_window, start_pos);
        lin(proj, att, w->dec_wo[l], SC(dec_wo_s, l), NULL, seq, qd, D);
        for (size_t i = 0; i < (size_t)seq * D; i++) x[i] += proj[i];
        vo_rms_norm(xn, x, w->dec_ffn_norm[l], seq, D, c->dec_eps);
        const float *ada = m->ada_scale + (size_t)l * D;
        for (int r = 0; r < seq; r++)
            for (int i = 0; i < D; i++) xn[(size_t)r * D + i] *= (1.0f + ada[i]);
        lin(gate, xn, w->dec_w1[l], SC(dec_w1_s, l), NULL, seq, D, hidden);
        vo_silu(gate, seq * hidden);
        lin(up, xn, w->dec_w3[l], SC(dec_w3_s, l), NULL, seq, D, hidden);
        for (size_t i = 0; i < (size_t)seq * hidden; i++) gate[i] *= up[i];
        lin(proj, gate, w->dec_w2[l], SC(dec_w2_s, l), NULL, seq, hidden, D);
        for (size_t i = 0; i < (size_t)seq * D; i++) x[i] += proj[i];
    }
    free(xn); free(q); free(k); free(v); free(att); free(proj); free(gate); free(up);
}

void vo_decoder_prefill(vo_stream_t *s, const float *embeds, int seq_len) {
    const vo_config_t *c = &s->m->c;
    int D = c->dec_dim, hd = c->dec_head_dim;
    if (!s->dk) dec_kv_init(s, c->dec_window + seq_len + 1024);
    else if (s->d_len + seq_len > s->d_max) dec_kv_grow(s, s->d_len + seq_len + 1024);
    float *x = (float *)malloc(sizeof(float) * (size_t)seq_len * D);
    memcpy(x, embeds, sizeof(float) * (size_t)seq_len * D);
    int start = s->d_len;
    int *pos = (int *)malloc(sizeof(int) * seq_len);
    for (int i = 0; i < seq_len; i++) pos[i] = s->d_off + start + i;
    float *rope = (float *)malloc(sizeof(float) * (size_t)seq_len * hd);
    vo_rope_freqs(rope, pos, seq_len, hd, c->rope_theta);
    dec_layers(s, x, seq_len, start, rope);
    s->d_len = start + seq_len;
    free(x); free(pos); free(rope);
}

int vo_decoder_forward(vo_stream_t *s, const float *embed, float *logits) {
    vo_model_t *m = s->m;
    const vo_config_t *c = &m->c;
    int D = c->dec_dim, hd = c->dec_head_dim;
    float *x = (float *)malloc(sizeof(float) * D);
    memcpy(x, embed, sizeof(float) * D);
    if (!s->dk) dec_kv_init(s, c->dec_window + 1 + 1024);
    int pos = s->d_len;
    if (pos >= s->d_max) {
        if (s->d_len > c->dec_window && !g_no_compact) { dec_kv_compact(s); pos = s->d_len; }
        if (pos >= s->d_max) dec_kv_grow(s, pos + 1024);
    }
    int lp = s->d_off + pos;
    float rope[512];
    vo_rope_freqs(rope, &lp, 1, hd, c->rope_theta);
    dec_layers(s, x, 1, pos, rope);
    s->d_len = pos + 1;
    vo_rms_norm(x, x, m->w.dec_norm, 1, D, c->dec_eps);
    lin(logits, x, m->w.tok_emb, m->w.tok_emb_s, NULL, 1, D, c->vocab);
    int best = 0;
    float bv = logits[0];
    for (int i = 1; i < c->vocab; i++)
        if (logits[i] > bv) { bv = logits[i]; best = i; }
    free(x);
    return best;
}

/* tok_embed_bf16_to_f32 / tok_embed_q8_to_f32 (voxtral.c:434-451) + adapter add
 * (voxtral.c:1106-1113) */
static void step_embed(vo_stream_t *s, float *dst, int adapter_row, int token) {
    const vo_config_t *c = &s->m->c;
    int D = c->dec_dim;
    const float *a = s->adapter + (size_t)adapter_row * D;
    if (s->m->w.tok_emb_s) {
        const int8_t *e = (const int8_t *)(const void *)s->m->w.tok_emb + (size_t)token * D;
        const float sc = s->m->w.tok_emb_s[token];
        for (int j = 0; j < D; j++) dst[j] = a[j] + (float)e[j] * sc;
        return;
    }
    const uint16_t *e = s->m->w.tok_emb + (size_t)token * D;
    for (int j = 0; j < D; j++) dst[j] = a[j] + bf16f(e[j]);
}

int vo_stream_decode(vo_stream_t *s, int max_steps, int stop_at_eos, int *tokens_out,
                     float *logits_out) {
    vo_model_t *m = s->m;
    const vo_config_t *c = &m->c;
    int D = c->dec_dim, V = c->vocab;
    int prompt_len = 1 + 32 + m->delay_tokens;
    int n = 0;
    float *emb = (float *)malloc(sizeof(float) * D);
    float *lg = (float *)malloc(sizeof(float) * V);
    if (!s->started) {
        if (s->total_adapter < prompt_len || max_steps <= 0) { free(emb); free(lg); return 0; }
        float *pe = (float *)malloc(sizeof(float) * (size_t)prompt_len * D);
        for (int i = 0; i < prompt_len; i++)
            step_embed(s, pe + (size_t)i * D, i, i == 0 ? TOKEN_BOS : TOKEN_STREAMING_PAD);
        s->d_len = 0;
        s->d_off = 0;
        vo_decoder_prefill(s, pe, prompt_len - 1);
        s->prev_token = vo_decoder_forward(s, pe + (size_t)(prompt_len - 1) * D, lg);
        free(pe);
        if (tokens_out) tokens_out[n] = s->prev_token;
        if (logits_out) memcpy(logits_out + (size_t)n * V, lg, sizeof(float) * V);
        n++;
        s->n_generated++;
        if (s->prev_token == TOKEN_EOS && stop_at_eos) s->eos_seen = 1;
        s->gen_pos = prompt_len;
        s->started = 1;
    }
    while (n < max_steps && !s->eos_seen && s->gen_pos < s->total_adapter) {
        step_embed(s, emb, s->gen_pos, s->prev_token);
        s->prev_token = vo_decoder_forward(s, emb, lg);
        if (tokens_out) tokens_out[n] = s->prev_token;
        if (logits_out) memcpy(logits_out + (size_t)n * V, lg, sizeof(float) * V);
        n++;
        s->n_generated++;
        s->gen_pos++;
        if (s->prev_token == TOKEN_EOS && stop_at_eos) { s->eos_seen = 1; break; }
    }
    free(emb);
    free(lg);
    return n;
}

/* ------------------------------------------------------------------------
 * Incremental mel (voxtral_audio.c:223-285 filters, 405-633 incremental driver).
 * Sample compaction (audio.c:432-450) and frame discard are memory housekeeping
 * only and are omitted.
 * ------------------------------------------------------------------------ */
#define MEL_SR 16000
#define MEL_N 128
#define MEL_HOP 160
#define MEL_WIN 400
#define MEL_NFFT 400
#define MEL_NFREQ 201
#define MEL_LOGMAX 1.5f
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

struct vo_mel {
    float *filters, *dcos, *dsin;
    float window[MEL_WIN];
    float *samples;
    int n_samples, cap;
    float *mel;
    int n_frames, mel_cap;
    int finished;
};

static float hz_to_mel(float f) {
    const float min_log_hz = 1000.0f, min_log_mel = 15.0f;
    const float logstep = 27.0f / logf(6.4f);
    float mels = 3.0f * f / 200.0f;
    if (f >= min_log_hz) mels = min_log_mel + logf(f / min_log_hz) * logstep;
    return mels;
}

static float mel_to_hz(float mels) {
    const float min_log_hz = 1000.0f, min_log_mel = 15.0f;
    const float logstep = logf(6.4f) / 27.0f;
    float f = 200.0f * mels / 3.0f;
    if (mels >= min_log_mel) f = min_log_hz * expf(logstep * (mels - min_log_mel));
    return f;
}

vo_mel_t *vo_mel_create(int left_pad_samples) {
    vo_mel_t *m = (vo_mel_t *)calloc(1, sizeof(*m));
    m->filters = (float *)calloc((size_t)MEL_N * MEL_NFREQ, sizeof(float));
    float fft_freqs[MEL_NFREQ], ff[MEL_N + 2], fd[MEL_N + 1];
    for (int i = 0; i < MEL_NFREQ; i++)
        fft_freqs[i] = (float)i * ((float)MEL_SR / 2.0f) / (float)(MEL_NFREQ - 1);
    float mmin = hz_to_mel(0.0f), mmax = hz_to_mel((float)MEL_SR / 2.0f);
    for (int i = 0; i < MEL_N + 2; i++)
        ff[i] = mel_to_hz(mmin + (mmax - mmin) * (float)i / (float)(MEL_N + 1));
    for (int i = 0; i < MEL_N + 1; i++) {
        fd[i] = ff[i + 1] - ff[i];
        if (fd[i] == 0.0f) fd[i] = 1e-6f;
    }
    for (int b = 0; b < MEL_N; b++) {
        float enorm = 2.0f / (ff[b + 2] - ff[b]);
        for (int f = 0; f < MEL_NFREQ; f++) {
            float down = (fft_freqs[f] - ff[b]) / fd[b];
            float up = (ff[b + 2] - fft_freqs[f]) / fd[b + 1];
            float val = fminf(down, up);
            if (val < 0.0f) val = 0.0f;
            m->filters[(size_t)b * MEL_NFREQ + f] = val * enorm;
        }
    }
    m->dcos = (float *)malloc(sizeof(float) * MEL_NFREQ * MEL_NFFT);
    m->dsin = (float *)malloc(sizeof(float) * MEL_NFREQ * MEL_NFFT);
    for (int k = 0; k < MEL_NFREQ; k++)
        for (int n = 0; n < MEL_NFFT; n++) {
            float ang = 2.0f * (float)M_PI * (float)k * (float)n / (float)MEL_NFFT;
            m->dcos[k * MEL_NFFT + n] = cosf(ang);
            m->dsin[k * MEL_NFFT + n] = sinf(ang);
        }
    for (int i = 0; i < MEL_WIN; i++)
        m->window[i] = 0.5f * (1.0f - cosf(2.0f * (float)M_PI * (float)i / (float)MEL_WIN));
    int lp = 200 + left_pad_samples;
    m->cap = lp + 16000;
    m->samples = (float *)calloc((size_t)m->cap, sizeof(float));
    m->n_samples = lp;
    return m;
}

static void mel_reserve(vo_mel_t *m, int need) {
    if (need <= m->cap) return;
    int nc = m->cap;
    while (nc < need) nc *= 2;
    m->samples = (float *)realloc(m->samples, sizeof(float) * (size_t)nc);
    m->cap = nc;
}

static int mel_compute(vo_mel_t *m) {
    int nf = 0;
    float win[MEL_NFFT], pw[MEL_NFREQ];
    for (;;) {
        int t = m->n_frames;
        long start = (long)t * MEL_HOP;
        if (start + MEL_WIN > m->n_samples) break;
        if (t >= m->mel_cap) {
            int nc = m->mel_cap ? m->mel_cap * 2 : 1024;
            m->mel = (float *)realloc(m->mel, sizeof(float) * (size_t)nc * MEL_N);
            m->mel_cap = nc;
        }
        for (int i = 0; i < MEL_NFFT; i++) win[i] = m->samples[start + i] * m->window[i];
        for (int k = 0; k < MEL_NFREQ; k++) {
            float re = 0, im = 0;
            const float *cr = m->dcos + k * MEL_NFFT, *sr = m->dsin + k * MEL_NFFT;
            for (int n = 0; n < MEL_NFFT; n++) {
                re += win[n] * cr[n];
                im += win[n] * sr[n];
            }
            pw[k] = re * re + im * im;
        }
        float *row = m->mel + (size_t)t * MEL_N;
        for (int b = 0; b < MEL_N; b++) {
            float sum = 0.0f;
            const float *fl = m->filters + (size_t)b * MEL_NFREQ;
            for (int k = 0; k < MEL_NFREQ; k++) sum += fl[k] * pw[k];
            if (sum < 1e-10f) sum = 1e-10f;
            float val = log10f(sum);
            float mn = MEL_LOGMAX - 8.0f;
            if (val < mn) val = mn;
            row[b] = (val + 4.0f) / 4.0f;
        }
        m->n_frames++;
        nf++;
    }
    return nf;
}

int vo_mel_feed(vo_mel_t *m, const float *samples, int n) {
    if (n <= 0) return 0;
    mel_reserve(m, m->n_samples + n);
    memcpy(m->samples + m->n_samples, samples, sizeof(float) * (size_t)n);
    m->n_samples += n;
    return mel_compute(m);
}

int vo_mel_finish(vo_mel_t *m, int right_pad) {
    if (m->finished) return m->n_frames;
    if (right_pad > 0) {
        mel_reserve(m, m->n_samples + right_pad);
        memset(m->samples + m->n_samples, 0, sizeof(float) * (size_t)right_pad);
        m->n_samples += right_pad;
    }
    mel_reserve(m, m->n_samples + 200);
    int real_end = m->n_samples - right_pad;
    for (int i = 0; i < 200; i++) {
        int src = real_end - 2 - i;
        m->samples[m->n_samples + i] = src >= 0 ? m->samples[src] : 0.0f;
    }
    m->n_samples += 200;
    mel_compute(m);
    if (m->n_frames > 0) m->n_frames--;
    m->finished = 1;
    return m->n_frames;
}

const float *vo_mel_data(vo_mel_t *m, int *n_frames) {
    if (n_frames) *n_frames = m->n_frames;
    return m->mel;
}

void vo_mel_free(vo_mel_t *m) {
    if (!m) return;
    free(m->filters); free(m->dcos); free(m->dsin); free(m->samples); free(m->mel);
    free(m);
}
