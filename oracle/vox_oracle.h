/*
 * vox_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference voxtral.c CPU/BLAS path (SeungheonOh/voxtral.c,
 * snapshot 2026-02-20).  It is the checker the HIP path is compared against: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is
 * never linked into, or called by, the product library (libvoxtral_hip.so).
 *
 * Each function cites the reference file:line it restates.  Differences from the
 * reference that are deliberate:
 *   - model dimensions are a runtime config (vo_config_t) instead of #defines
 *     (voxtral.h:26-50), so the same code runs the real Voxtral-4B shapes and the tiny
 *     configurations the tests use;
 *   - gelu_erf selects the erf GELU of python_simple_implementation.py (used only to pin
 *     this oracle against the Python reference); 0 = tanh GELU of voxtral_kernels.c:505-513.
 *
 * Pinning: the mel front-end is checked bit-for-bit (within 1e-6) against the
 * reference's own voxtral_audio.c compiled in place (oracle/_ref); the model math is
 * checked against fixtures produced by the Python reference (tests/golden/).  See
 * DESIGN.md "Oracle".
 */
#ifndef VOX_ORACLE_H
#define VOX_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int enc_dim, enc_layers, enc_heads, enc_kv_heads, enc_head_dim, enc_hidden, enc_window;
    int dec_dim, dec_layers, dec_heads, dec_kv_heads, dec_head_dim, dec_hidden, dec_window;
    int vocab, mel_bins, downsample, ada_dim;
    float rope_theta, enc_eps, dec_eps;
    int gelu_erf;
} vo_config_t;

/* Weight views.  Matrices are bf16 [out, in] row-major (safetensors.c:446-451);
 * small tensors are f32 (the reference converts them at load: encoder.c:31-38). */
typedef struct {
    const float *conv0_w, *conv0_b, *conv1_w, *conv1_b;          /* [D,mel*3] [D] [D,D*3] [D] */
    const uint16_t **enc_wq, **enc_wk, **enc_wv, **enc_wo, **enc_w1, **enc_w2, **enc_w3;
    const float **enc_wq_b, **enc_wv_b, **enc_wo_b, **enc_w2_b, **enc_attn_norm, **enc_ffn_norm;
    const float *enc_norm;
    const uint16_t *ad0, *ad1;                                   /* [dec, enc*4], [dec, dec] */
    const uint16_t *tok_emb;                                     /* [vocab, dec] (tied LM head) */
    const uint16_t **dec_wq, **dec_wk, **dec_wv, **dec_wo, **dec_w1, **dec_w2, **dec_w3;
    const float **dec_attn_norm, **dec_ffn_norm, **dec_ada_down, **dec_ada_up;
    const float *dec_norm;
    /* Q8 checkpoints (quantize.py; voxtral_safetensors.c:393-408, 457-468): a non-NULL
     * per-row scale array selects the q8 path for that matrix, whose pointer above then
     * addresses its int8 [out, in] data.  ada_down/up arrive dequantized (load_f32). */
    const float **enc_wq_s, **enc_wk_s, **enc_wv_s, **enc_wo_s, **enc_w1_s, **enc_w2_s, **enc_w3_s;
    const float *ad0_s, *ad1_s, *tok_emb_s;
    const float **dec_wq_s, **dec_wk_s, **dec_wv_s, **dec_wo_s, **dec_w1_s, **dec_w2_s, **dec_w3_s;
} vo_weights_t;

typedef struct vo_model vo_model_t;
typedef struct vo_stream vo_stream_t;

/* ---- per-op restatements (voxtral_kernels.c) ---- */
void vo_set_threads(int n);
/* test-only: 1 = grow the KV caches instead of compacting them (invariance tests) */
void vo_set_no_compaction(int on);
/* decoder KV appends rounded to IEEE half (the reference's VOX_DECODER_KV_FP16 cache) */
void vo_set_kv_fp16(int on);
/* f32 -> half -> f32 of n values (for tests of the rounding) */
void vo_f16_round(const float *x, int n, float *out);
void vo_linear_bf16(float *y, const float *x, const uint16_t *W, const float *b,
                    int M, int in_dim, int out_dim);
/* vox_linear_q8 / vox_linear_nobias_q8 / vox_matmul_t_q8 (voxtral_kernels.c:277-393) */
void vo_linear_q8(float *y, const float *x, const int8_t *W, const float *scales, const float *b,
                  int M, int in_dim, int out_dim);
void vo_rms_norm(float *out, const float *x, const float *w, int M, int hidden, float eps);
void vo_gelu(float *x, int n, int erf_mode);
void vo_silu(float *x, int n);
void vo_causal_conv1d(float *out, const float *in, const float *w, const float *b,
                      int cin, int cout, int length, int ks, int stride);
void vo_causal_attention(float *out, const float *Q, const float *K, const float *V,
                         int seq_q, int seq_k, int n_heads, int n_kv_heads, int head_dim,
                         float scale, int window, int q_offset);
void vo_rope_freqs(float *freqs, const int *pos, int seq, int dim, float theta);
void vo_apply_rope(float *x, const float *freqs, int seq, int heads, int head_dim);
void vo_time_embedding(float *out, int dim, float t);

/* ---- model / stream ---- */
vo_model_t *vo_model_create(const vo_config_t *cfg, const vo_weights_t *w, int delay_tokens);
void vo_model_free(vo_model_t *m);
const float *vo_model_ada_scale(const vo_model_t *m);
void vo_model_set_delay(vo_model_t *m, int delay_tokens);

vo_stream_t *vo_stream_create(vo_model_t *m);
void vo_stream_free(vo_stream_t *s);
/* stream_conv_stem (voxtral.c:581-759): returns rows written to out ([rows, enc_dim]) */
int vo_conv_stem(vo_stream_t *s, const float *mel_new, int n_new, float *out, int out_cap);
/* vox_encoder_forward_incremental (encoder.c:495-693), in place on x [new_len, enc_dim] */
int vo_encoder_incremental(vo_stream_t *s, float *x, int new_len);
/* vox_adapter_forward (encoder.c:699-737) */
int vo_adapter(vo_model_t *m, const float *enc, int enc_rows, float *out);
/* stream_run_encoder body (voxtral.c:827-951) on n mel frames; returns adapter tokens added */
int vo_stream_encode_mel(vo_stream_t *s, const float *mel, int n_frames);
int vo_stream_adapter_tokens(const vo_stream_t *s);
const float *vo_stream_adapter(const vo_stream_t *s);
/* vox_decoder_prefill (decoder.c:447-612) / vox_decoder_forward (decoder.c:640-780) */
void vo_decoder_prefill(vo_stream_t *s, const float *embeds, int seq_len);
int vo_decoder_forward(vo_stream_t *s, const float *embed, float *logits);
/* stream_run_decoder (voxtral.c:1013-1240), non-continuous mode, no alternatives.
 * Runs prefill when possible, then up to max_steps steps.  tokens_out[i] and, if
 * logits_out != NULL, logits_out[i*vocab..] for every generated token. */
int vo_stream_decode(vo_stream_t *s, int max_steps, int stop_at_eos, int *tokens_out,
                     float *logits_out);
void vo_stream_state(const vo_stream_t *s, int *out8);
/* stream_reset_decoder_state (voxtral.c:766-783) / stream_reset_full_state (:786-814, the
 * mel context excluded: it belongs to the caller) */
void vo_stream_reset_decoder(vo_stream_t *s);
void vo_stream_reset_full(vo_stream_t *s);

/* ---- incremental mel (voxtral_audio.c:405-662) ---- */
typedef struct vo_mel vo_mel_t;
vo_mel_t *vo_mel_create(int left_pad_samples);
int vo_mel_feed(vo_mel_t *m, const float *samples, int n);
int vo_mel_finish(vo_mel_t *m, int right_pad_samples);
const float *vo_mel_data(vo_mel_t *m, int *n_frames);
void vo_mel_free(vo_mel_t *m);

#ifdef __cplusplus
}
#endif
#endif
