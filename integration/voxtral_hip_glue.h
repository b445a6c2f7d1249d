/*
 * voxtral_hip_glue.h -- the USE_HIP binding of libvoxtral_hip.so into the reference's C host
 * (SeungheonOh/voxtral.c @ 2026-02-20).  These functions are what the reference's call sites
 * call under `#ifdef USE_HIP` (INTEGRATION.md sections 3-6 show each call site); they compile
 * against the reference's own voxtral.h / voxtral_kernels.h (tests/test_integration.py
 * type-checks them there).  Owned by a maintainer patch, not part of the reference.
 */
#ifndef VOXTRAL_HIP_GLUE_H
#define VOXTRAL_HIP_GLUE_H

#include "voxtral.h"      /* reference: vox_ctx_t and the VOX_* dimensions */
#include "voxtral_hip.h"  /* this repository's C ABI */

/* The HIP state a vox_ctx_t carries (the patch adds `vox_hip_binding_t hip;` to vox_ctx_t,
 * voxtral.h:188-239).  One model and one device stream per context; nothing is shared between
 * contexts (a process may load several). */
typedef struct {
    vox_hip_model_t *model;
    vox_hip_stream_t *stream;
} vox_hip_binding_t;

/* vox_load (voxtral.c:186-284, the Metal warm-up block): upload every weight vox_load holds
 * (bf16 or Q8 views off the safetensors mmap, small tensors already f32) into HBM and open the
 * context's stream.  0, or -1 with vox_hip_last_error(). */
int vox_hip_bind_load(const vox_ctx_t *ctx, vox_hip_binding_t *b);
/* vox_free */
void vox_hip_bind_free(vox_hip_binding_t *b);
/* vox_set_delay (voxtral.c:1681-1687), after vox_update_time_conditioning */
int vox_hip_bind_set_delay(const vox_ctx_t *ctx, vox_hip_binding_t *b);

/* vox_encoder_forward_incremental (voxtral_encoder.c:495-693) in full: the 32 layers + final
 * norm on the device, K/V appended to the stream's rolling HBM cache at the logical positions
 * that follow the ones already seen.  Returns a malloc'd [new_len, VOX_ENC_DIM] buffer the
 * caller frees (as the reference's), NULL on error. */
float *vox_hip_bind_encoder_incremental(vox_ctx_t *ctx, vox_hip_binding_t *b, const float *x_new,
                                        int new_len, int *out_len);
/* vox_decoder_prefill (voxtral_decoder.c:447-612): seq_len rows through the 26 layers, K/V
 * written at logical positions kv_pos_offset + kv_cache_len ..  0 / -1. */
int vox_hip_bind_decoder_prefill(vox_ctx_t *ctx, vox_hip_binding_t *b, const float *input_embeds, int seq_len);
/* vox_decoder_forward (voxtral_decoder.c:640-780): one token, final norm, LM head, argmax
 * (first max wins); logits [VOX_VOCAB_SIZE] filled if non-NULL.  The token id, or -1. */
int vox_hip_bind_decoder_forward(vox_ctx_t *ctx, vox_hip_binding_t *b, const float *input_embeds, float *logits);
/* stream_reset_decoder_state (voxtral.c:766-783) / stream_reset_full_state (:786-814) */
int vox_hip_bind_reset_decoder(vox_ctx_t *ctx, vox_hip_binding_t *b);
int vox_hip_bind_reset_full(vox_ctx_t *ctx, vox_hip_binding_t *b);

/* The USE_HIP branches of voxtral_kernels.c's linears (vox_linear_bf16 / vox_linear_nobias_bf16
 * / vox_matmul_t_bf16, :197-264, and the Q8 trio, :316-377), taken when vox_hip_available():
 * y[seq_len, out_dim] = x W^T (+ bias) on the device, the bf16 / int8 weights cached in HBM by
 * host pointer.  The adapter's M > 1 projections (voxtral.c:895) reach the device this way.
 * A device error prints vox_hip_last_error() and aborts (no silent CPU fallback). */
void vox_hip_bind_linear_bf16(float *y, const float *x, const uint16_t *W_bf16, const float *bias,
                              int seq_len, int in_dim, int out_dim);
void vox_hip_bind_matmul_t_bf16(float *C, const float *A, const uint16_t *B_bf16, int M, int K, int N);
void vox_hip_bind_linear_q8(float *y, const float *x, const int8_t *W_q8, const float *scales, const float *bias,
                            int seq_len, int in_dim, int out_dim);
void vox_hip_bind_matmul_t_q8(float *C, const float *A, const int8_t *B_q8, const float *scales, int M, int K, int N);

#endif
