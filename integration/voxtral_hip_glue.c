/*
 * voxtral_hip_glue.c -- see voxtral_hip_glue.h.  Built into the reference's `hip` target
 *  next to voxtral.c / voxtral_encoder.c / voxtral_decoder.c.
 */
#include "voxtral_hip_glue.h"
#include "voxtral_kernels.h"  /* reference: vox_compute_rope_freqs (voxtral_kernels.c:617-629) */

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* bf16 view, or the int8 view (cast) when the checkpoint is Q8 (voxtral_encoder.c /
 * voxtral_decoder.c load one of the two per matrix, quantize.py layout) */
#define MAT(L, name) ((L)->name##_weight_bf16 ? (const uint16_t *)(L)->name##_weight_bf16 \
                                               : (const uint16_t *)(L)->name##_weight_q8)
#define SCL(L, name) ((L)->name##_weight_bf16 ? (const float *)0 : (const float *)(L)->name##_scale_q8)

/* the per-layer pointer arrays of vox_hip_weights_t, for one vox_hip_bind_load: heap-owned
 * and freed once vox_hip_model_create has uploaded (and packed) everything, so two contexts
 * loaded in one process never share them */
typedef struct {
    const uint16_t *ewq[VOX_ENC_LAYERS], *ewk[VOX_ENC_LAYERS], *ewv[VOX_ENC_LAYERS], *ewo[VOX_ENC_LAYERS];
    const uint16_t *ew1[VOX_ENC_LAYERS], *ew2[VOX_ENC_LAYERS], *ew3[VOX_ENC_LAYERS];
    const float *ewqb[VOX_ENC_LAYERS], *ewvb[VOX_ENC_LAYERS], *ewob[VOX_ENC_LAYERS], *ew2b[VOX_ENC_LAYERS];
    const float *ean[VOX_ENC_LAYERS], *efn[VOX_ENC_LAYERS];
    const float *ewqs[VOX_ENC_LAYERS], *ewks[VOX_ENC_LAYERS], *ewvs[VOX_ENC_LAYERS], *ewos[VOX_ENC_LAYERS];
    const float *ew1s[VOX_ENC_LAYERS], *ew2s[VOX_ENC_LAYERS], *ew3s[VOX_ENC_LAYERS];
    const uint16_t *dwq[VOX_DEC_LAYERS], *dwk[VOX_DEC_LAYERS], *dwv[VOX_DEC_LAYERS], *dwo[VOX_DEC_LAYERS];
    const uint16_t *dw1[VOX_DEC_LAYERS], *dw2[VOX_DEC_LAYERS], *dw3[VOX_DEC_LAYERS];
    const float *dan[VOX_DEC_LAYERS], *dfn[VOX_DEC_LAYERS], *dad[VOX_DEC_LAYERS], *dau[VOX_DEC_LAYERS];
    const float *dwqs[VOX_DEC_LAYERS], *dwks[VOX_DEC_LAYERS], *dwvs[VOX_DEC_LAYERS], *dwos[VOX_DEC_LAYERS];
    const float *dw1s[VOX_DEC_LAYERS], *dw2s[VOX_DEC_LAYERS], *dw3s[VOX_DEC_LAYERS];
} vox_hip_tables_t;

static int bind_model(const vox_ctx_t *ctx, vox_hip_binding_t *b, vox_hip_tables_t *t);

int vox_hip_bind_load(const vox_ctx_t *ctx, vox_hip_binding_t *b) {
    b->model = NULL;
    b->stream = NULL;
    vox_hip_tables_t *t = (vox_hip_tables_t *)calloc(1, sizeof *t);
    if (!t) return -1;
    const int rc = bind_model(ctx, b, t);
    free(t);
    return rc;
}

static int bind_model(const vox_ctx_t *ctx, vox_hip_binding_t *b, vox_hip_tables_t *t) {
    const uint16_t **ewq = t->ewq, **ewk = t->ewk, **ewv = t->ewv, **ewo = t->ewo;
    const uint16_t **ew1 = t->ew1, **ew2 = t->ew2, **ew3 = t->ew3;
    const float **ewqb = t->ewqb, **ewvb = t->ewvb, **ewob = t->ewob, **ew2b = t->ew2b;
    const float **ean = t->ean, **efn = t->efn;
    const float **ewqs = t->ewqs, **ewks = t->ewks, **ewvs = t->ewvs, **ewos = t->ewos;
    const float **ew1s = t->ew1s, **ew2s = t->ew2s, **ew3s = t->ew3s;
    const uint16_t **dwq = t->dwq, **dwk = t->dwk, **dwv = t->dwv, **dwo = t->dwo;
    const uint16_t **dw1 = t->dw1, **dw2 = t->dw2, **dw3 = t->dw3;
    const float **dan = t->dan, **dfn = t->dfn, **dad = t->dad, **dau = t->dau;
    const float **dwqs = t->dwqs, **dwks = t->dwks, **dwvs = t->dwvs, **dwos = t->dwos;
    const float **dw1s = t->dw1s, **dw2s = t->dw2s, **dw3s = t->dw3s;
    const int q8 = ctx->use_q8;

    if (!vox_hip_available() && !vox_hip_init()) return -1;
    for (int l = 0; l < VOX_ENC_LAYERS; l++) {
        const vox_enc_layer_t *L = &ctx->encoder.layers[l];
        ewq[l] = MAT(L, wq); ewk[l] = MAT(L, wk); ewv[l] = MAT(L, wv); ewo[l] = MAT(L, wo);
        ew1[l] = MAT(L, w1); ew2[l] = MAT(L, w2); ew3[l] = MAT(L, w3);
        ewqs[l] = SCL(L, wq); ewks[l] = SCL(L, wk); ewvs[l] = SCL(L, wv); ewos[l] = SCL(L, wo);
        ew1s[l] = SCL(L, w1); ew2s[l] = SCL(L, w2); ew3s[l] = SCL(L, w3);
        ewqb[l] = L->wq_bias; ewvb[l] = L->wv_bias; ewob[l] = L->wo_bias; ew2b[l] = L->w2_bias;
        ean[l] = L->attention_norm; efn[l] = L->ffn_norm;
    }
    for (int l = 0; l < VOX_DEC_LAYERS; l++) {
        const vox_dec_layer_t *L = &ctx->decoder.layers[l];
        dwq[l] = MAT(L, wq); dwk[l] = MAT(L, wk); dwv[l] = MAT(L, wv); dwo[l] = MAT(L, wo);
        dw1[l] = MAT(L, w1); dw2[l] = MAT(L, w2); dw3[l] = MAT(L, w3);
        dwqs[l] = SCL(L, wq); dwks[l] = SCL(L, wk); dwvs[l] = SCL(L, wv); dwos[l] = SCL(L, wo);
        dw1s[l] = SCL(L, w1); dw2s[l] = SCL(L, w2); dw3s[l] = SCL(L, w3);
        dan[l] = L->attention_norm; dfn[l] = L->ffn_norm;
        dad[l] = L->ada_norm_down; dau[l] = L->ada_norm_up;
    }
    vox_hip_weights_t w;
    memset(&w, 0, sizeof w);
    w.conv0_w = ctx->encoder.conv0_weight; w.conv0_b = ctx->encoder.conv0_bias;
    w.conv1_w = ctx->encoder.conv1_weight; w.conv1_b = ctx->encoder.conv1_bias;
    w.enc_wq = ewq; w.enc_wk = ewk; w.enc_wv = ewv; w.enc_wo = ewo;
    w.enc_w1 = ew1; w.enc_w2 = ew2; w.enc_w3 = ew3;
    w.enc_wq_b = ewqb; w.enc_wv_b = ewvb; w.enc_wo_b = ewob; w.enc_w2_b = ew2b;
    w.enc_attn_norm = ean; w.enc_ffn_norm = efn;
    w.enc_norm = ctx->encoder.norm;
    w.ad0 = ctx->adapter.linear0_weight_bf16 ? ctx->adapter.linear0_weight_bf16
                                             : (const uint16_t *)ctx->adapter.linear0_weight_q8;
    w.ad1 = ctx->adapter.linear1_weight_bf16 ? ctx->adapter.linear1_weight_bf16
                                             : (const uint16_t *)ctx->adapter.linear1_weight_q8;
    w.tok_emb = ctx->decoder.tok_embeddings_bf16 ? ctx->decoder.tok_embeddings_bf16
                                                 : (const uint16_t *)ctx->decoder.tok_embeddings_q8;
    w.dec_wq = dwq; w.dec_wk = dwk; w.dec_wv = dwv; w.dec_wo = dwo;
    w.dec_w1 = dw1; w.dec_w2 = dw2; w.dec_w3 = dw3;
    w.dec_attn_norm = dan; w.dec_ffn_norm = dfn; w.dec_ada_down = dad; w.dec_ada_up = dau;
    w.dec_norm = ctx->decoder.norm;
    if (q8) {
        w.enc_wq_s = ewqs; w.enc_wk_s = ewks; w.enc_wv_s = ewvs; w.enc_wo_s = ewos;
        w.enc_w1_s = ew1s; w.enc_w2_s = ew2s; w.enc_w3_s = ew3s;
        w.ad0_s = ctx->adapter.linear0_weight_bf16 ? NULL : ctx->adapter.linear0_scale_q8;
        w.ad1_s = ctx->adapter.linear1_weight_bf16 ? NULL : ctx->adapter.linear1_scale_q8;
        w.tok_emb_s = ctx->decoder.tok_embeddings_bf16 ? NULL : ctx->decoder.tok_embeddings_scale_q8;
        w.dec_wq_s = dwqs; w.dec_wk_s = dwks; w.dec_wv_s = dwvs; w.dec_wo_s = dwos;
        w.dec_w1_s = dw1s; w.dec_w2_s = dw2s; w.dec_w3_s = dw3s;
    }
    vox_hip_config_t cfg;
    vox_hip_config_voxtral_4b(&cfg);
    b->model = vox_hip_model_create(&cfg, &w, ctx->delay_tokens);
    if (!b->model) return -1;
    /* the reference's KV precision switch (voxtral.c:189-190) */
    if (ctx->kv_cache_fp16) vox_hip_model_set_kv_fp16(b->model, 1);
    b->stream = vox_hip_stream_create(b->model);
    if (!b->stream) {
        vox_hip_model_free(b->model);
        b->model = NULL;
        return -1;
    }
    return 0;
}

void vox_hip_bind_free(vox_hip_binding_t *b) {
    if (b->stream) vox_hip_stream_free(b->stream);
    if (b->model) vox_hip_model_free(b->model);
    b->stream = NULL;
    b->model = NULL;
}

int vox_hip_bind_set_delay(const vox_ctx_t *ctx, vox_hip_binding_t *b) {
    return b->model ? vox_hip_model_set_delay(b->model, ctx->delay_tokens) : -1;
}

float *vox_hip_bind_encoder_incremental(vox_ctx_t *ctx, vox_hip_binding_t *b, const float *x_new,
                                        int new_len, int *out_len) {
    *out_len = 0;
    if (new_len <= 0) return NULL;
    /* the HBM cache is a ring indexed by logical position: no host compaction / growth, the
     * host keeps only the logical count (enc_kv_pos_offset; enc_kv_cache_len stays 0) */
    const int logical = ctx->enc_kv_pos_offset + ctx->enc_kv_cache_len;
    float *x = (float *)malloc((size_t)new_len * VOX_ENC_DIM * sizeof(float));
    int *pos = (int *)malloc((size_t)new_len * sizeof(int));
    float *rope = (float *)malloc((size_t)new_len * VOX_ENC_HEAD_DIM * sizeof(float));
    if (!x || !pos || !rope) {
        free(x); free(pos); free(rope);
        return NULL;
    }
    memcpy(x, x_new, (size_t)new_len * VOX_ENC_DIM * sizeof(float));
    for (int i = 0; i < new_len; i++) pos[i] = logical + i;
    vox_compute_rope_freqs(rope, pos, new_len, VOX_ENC_HEAD_DIM, VOX_ROPE_THETA);
    const int rc = vox_hip_encoder_full_step(b->stream, x, new_len, rope, logical);
    free(pos);
    free(rope);
    if (rc != 0) {  /* no silent CPU fallback: the caller sees NULL, the reason in last_error */
        free(x);
        return NULL;
    }
    ctx->enc_kv_pos_offset = logical + new_len;
    ctx->enc_kv_cache_len = 0;
    *out_len = new_len;
    return x;
}

int vox_hip_bind_decoder_prefill(vox_ctx_t *ctx, vox_hip_binding_t *b, const float *input_embeds, int seq_len) {
    const int start = ctx->kv_cache_len, logical = ctx->kv_pos_offset + start;
    float *x = (float *)malloc((size_t)seq_len * VOX_DEC_DIM * sizeof(float));
    int *pos = (int *)malloc((size_t)seq_len * sizeof(int));
    float *rope = (float *)malloc((size_t)seq_len * VOX_DEC_HEAD_DIM * sizeof(float));
    int rc = -1;
    if (x && pos && rope) {
        memcpy(x, input_embeds, (size_t)seq_len * VOX_DEC_DIM * sizeof(float));
        for (int i = 0; i < seq_len; i++) pos[i] = logical + i;
        vox_compute_rope_freqs(rope, pos, seq_len, VOX_DEC_HEAD_DIM, VOX_ROPE_THETA);
        rc = vox_hip_decoder_prefill_step(b->stream, x, seq_len, rope, logical);
        if (rc == 0) ctx->kv_cache_len = start + seq_len;
    }
    free(x); free(pos); free(rope);
    return rc;
}

int vox_hip_bind_decoder_forward(vox_ctx_t *ctx, vox_hip_binding_t *b, const float *input_embeds, float *logits) {
    /* the device ring holds window + 64 logical positions: the host never compacts or grows
     * a cache (voxtral_decoder.c:667-677 is skipped), kv_cache_len counts logical steps */
    const int pos = ctx->kv_cache_len, logical = ctx->kv_pos_offset + pos;
    float rope[VOX_DEC_HEAD_DIM];
    vox_compute_rope_freqs(rope, &logical, 1, VOX_DEC_HEAD_DIM, VOX_ROPE_THETA);
    vox_hip_decoder_start(b->stream, input_embeds, VOX_DEC_DIM);
    const int token = vox_hip_decoder_full_step(b->stream, rope, logical, logits);
    vox_hip_decoder_end(b->stream);
    if (token < 0) return -1;
    ctx->kv_cache_len = pos + 1;
    return token;
}

int vox_hip_bind_reset_decoder(vox_ctx_t *ctx, vox_hip_binding_t *b) {
    (void)ctx;
    return vox_hip_stream_reset_decoder(b->stream);
}

int vox_hip_bind_reset_full(vox_ctx_t *ctx, vox_hip_binding_t *b) {
    (void)ctx;
    return vox_hip_stream_reset(b->stream);
}

/* ---- the single-op linears of voxtral_kernels.c (M > 1 callers: the adapter's two
 * projections, voxtral.c:895, and the non-incremental encoder) ----
 * The reference's USE_METAL branches call vox_metal_sgemm_bf16 / _q8 and return
 * (voxtral_kernels.c:197-264, 316-377); these do the same on the device (weights cached in
 * HBM by host pointer on first use).  A device error is not hidden behind the CPU path: it
 * is reported and the process stops, as a wrong result would otherwise go unnoticed. */
static void linear_done(const char *what) {
    const char *e = vox_hip_last_error();
    if (e && e[0]) {
        fprintf(stderr, "HIP backend: %s: %s\n", what, e);
        abort();
    }
}

static void add_bias(float *y, const float *bias, int rows, int cols) {
    if (!bias) return;
    for (int s = 0; s < rows; s++)
        for (int o = 0; o < cols; o++) y[(size_t)s * cols + o] += bias[o];
}

void vox_hip_bind_linear_bf16(float *y, const float *x, const uint16_t *W_bf16, const float *bias,
                              int seq_len, int in_dim, int out_dim) {
    vox_hip_clear_error();
    vox_hip_sgemm_bf16(seq_len, out_dim, in_dim, x, W_bf16, y);
    linear_done("vox_linear_bf16");
    add_bias(y, bias, seq_len, out_dim);
}

void vox_hip_bind_matmul_t_bf16(float *C, const float *A, const uint16_t *B_bf16, int M, int K, int N) {
    vox_hip_clear_error();
    vox_hip_sgemm_bf16(M, N, K, A, B_bf16, C);
    linear_done("vox_matmul_t_bf16");
}

void vox_hip_bind_linear_q8(float *y, const float *x, const int8_t *W_q8, const float *scales, const float *bias,
                            int seq_len, int in_dim, int out_dim) {
    vox_hip_clear_error();
    vox_hip_sgemm_q8(seq_len, out_dim, in_dim, x, W_q8, scales, y);
    linear_done("vox_linear_q8");
    add_bias(y, bias, seq_len, out_dim);
}

void vox_hip_bind_matmul_t_q8(float *C, const float *A, const int8_t *B_q8, const float *scales, int M, int K, int N) {
    vox_hip_clear_error();
    vox_hip_sgemm_q8(M, N, K, A, B_q8, scales, C);
    linear_done("vox_matmul_t_q8");
}
