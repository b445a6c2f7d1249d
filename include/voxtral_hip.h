/*
 * voxtral_hip.h -- C ABI of the MI355X (gfx950 / CDNA4) backend for voxtral.c.
 *
 * This header is the drop-in boundary.  It replaces the reference's Metal backend
 * interface (voxtral_metal.h, SeungheonOh/voxtral.c @ 2026-02-20); every entry point
 * below cites the reference declaration it replaces.  Signatures use plain pointers and
 * sizes only.  All functions are synchronous with respect to host pointers they are
 * given, like the Metal backend (voxtral_metal.m waits on every command buffer).
 *
 * Differences from voxtral_metal.h that the discrete-GPU design forces (see
 * INTEGRATION.md for the call-site patch):
 *   - the Metal backend read weights and KV state out of the reference's vox_ctx_t via
 *     `void *ctx` (voxtral_metal.m:2888-3174).  Here weights are handed over once as a
 *     table of host pointers (vox_hip_weights_t, filled from vox_ctx_t at vox_load) and
 *     per-stream device state lives in an opaque vox_hip_stream_t;
 *   - the decoder/encoder KV caches live in HBM as rolling buffers indexed by LOGICAL
 *     position (slot = pos mod capacity), so the host-side memmove compaction of
 *     voxtral_decoder.c:354-384 / voxtral_encoder.c:431-449 becomes unnecessary.  The
 *     step functions therefore take the logical start position instead of the physical
 *     cache length.  Attention semantics are unchanged: the last `window` logical
 *     positions are visible (identical to the CPU path after compaction).
 *
 * Errors: functions returning int return a negative value on failure (the reference's
 * step functions return -1 to request the CPU fallback; this backend never falls back
 * silently -- a failure is reported and the caller decides).
 */
#ifndef VOXTRAL_HIP_H
#define VOXTRAL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------
 * Runtime (voxtral_metal.h:20-26)
 * ------------------------------------------------------------------------ */
int vox_hip_init(void);          /* voxtral_metal.h:20  vox_metal_init: 1 on success */
int vox_hip_available(void);     /* voxtral_metal.h:23  vox_metal_available */
void vox_hip_shutdown(void);     /* voxtral_metal.h:26  vox_metal_shutdown */
size_t vox_hip_memory_used(void);/* voxtral_metal.h:282 vox_metal_memory_used */
const char *vox_hip_last_error(void);  /* "" when no error since the last clear */
void vox_hip_clear_error(void);          /* the void twins below report only through last_error */
int vox_hip_set_device(int device);

/* ------------------------------------------------------------------------
 * Model dimensions (voxtral.h:18-50 are compile-time #defines in the reference;
 * here they are a runtime record so test configurations can shrink the model).
 * ------------------------------------------------------------------------ */
typedef struct {
    int enc_dim, enc_layers, enc_heads, enc_kv_heads, enc_head_dim, enc_hidden, enc_window;
    int dec_dim, dec_layers, dec_heads, dec_kv_heads, dec_head_dim, dec_hidden, dec_window;
    int vocab, mel_bins, downsample, ada_dim;
    float rope_theta, enc_eps, dec_eps;
    int gelu_erf; /* 0: tanh GELU (voxtral_kernels.c:505-513), the default */
} vox_hip_config_t;

void vox_hip_config_voxtral_4b(vox_hip_config_t *cfg); /* voxtral.h:26-50 values */

/* Weight table: host pointers, exactly the views vox_ctx_t holds after vox_load
 * (voxtral.h:56-239): bf16 matrices straight off the safetensors mmap, small tensors
 * already converted to f32.  Per-layer tensors are arrays of `layers` pointers. */
typedef struct {
    const float *conv0_w, *conv0_b, *conv1_w, *conv1_b;
    const uint16_t **enc_wq, **enc_wk, **enc_wv, **enc_wo, **enc_w1, **enc_w2, **enc_w3;
    const float **enc_wq_b, **enc_wv_b, **enc_wo_b, **enc_w2_b, **enc_attn_norm, **enc_ffn_norm;
    const float *enc_norm;
    const uint16_t *ad0, *ad1;
    const uint16_t *tok_emb;
    const uint16_t **dec_wq, **dec_wk, **dec_wv, **dec_wo, **dec_w1, **dec_w2, **dec_w3;
    const float **dec_attn_norm, **dec_ffn_norm, **dec_ada_down, **dec_ada_up;
    const float *dec_norm;
    /* Q8 checkpoints (quantize.py output; voxtral_safetensors.c:393-408, 457-468).  A
     * non-NULL per-row scale array (safetensors_get_q8_scales_direct) selects int8 for that
     * matrix, whose pointer above then carries safetensors_get_q8_data_direct, cast
     * (int8 [out, in]).  Q/K/V of a layer and its w1/w3 must agree.  ada_down/up and the
     * conv weights stay f32 (load_f32 dequantises / quantize.py keeps 3-D tensors f32).
     * Leave all NULL (zero-initialise the struct) for a bf16 checkpoint. */
    const float **enc_wq_s, **enc_wk_s, **enc_wv_s, **enc_wo_s, **enc_w1_s, **enc_w2_s, **enc_w3_s;
    const float *ad0_s, *ad1_s, *tok_emb_s;
    const float **dec_wq_s, **dec_wk_s, **dec_wv_s, **dec_wo_s, **dec_w1_s, **dec_w2_s, **dec_w3_s;
} vox_hip_weights_t;

typedef struct vox_hip_model vox_hip_model_t;
typedef struct vox_hip_stream vox_hip_stream_t;

/* Upload + pack all weights into HBM once (replaces the Metal warm-up and weight
 * caches, voxtral.c:186-284 / voxtral_metal.m:133-501: QKV and W1|W3 are merged here).
 * delay_tokens sets the time conditioning (voxtral.c:47-80). */
vox_hip_model_t *vox_hip_model_create(const vox_hip_config_t *cfg, const vox_hip_weights_t *w,
                                      int delay_tokens);
void vox_hip_model_free(vox_hip_model_t *m);
/* vox_set_delay (voxtral.c:1681-1687): recompute ada_scale and re-upload it (the Metal
 * backend's pointer-keyed f32 cache went stale here, voxtral_metal.m:471-501). */
int vox_hip_model_set_delay(vox_hip_model_t *m, int delay_tokens);
/* ada_scale [dec_layers*dec_dim] as computed on the host (for tests). */
int vox_hip_model_ada_scale(vox_hip_model_t *m, float *out);
/* The reference's fp16 decoder KV cache (VOX_DECODER_KV_FP16, voxtral.c:189-190, the Metal
 * default; voxtral_decoder.c:180-243 allocates the dual-format cache): streams created after
 * this call keep their decoder K/V rings in IEEE half (stores round to nearest even, all
 * attention arithmetic f32), halving the ring's HBM bytes per decode step.  Opt-in here: off
 * unless VOX_DECODER_KV_FP16 is set nonzero at model creation or on = 1 is passed; the
 * default f32 ring is the CPU reference's (voxtral_decoder.c:232-234).  head_dim 128 only
 * (Voxtral's); returns 0, or -1 (vox_hip_last_error) for another head_dim. */
int vox_hip_model_set_kv_fp16(vox_hip_model_t *m, int on);
/* Arithmetic of the M > 1 GEMMs (encoder, adapter, prefill; no reference counterpart: the
 * CPU path's cblas_sgemm, voxtral_kernels.c:197-240, is f32): every f32 activation is split
 * into bf16 planes that multiply the exact bf16 weights on MFMA.  planes = 3 (hi + mid + lo,
 * the default) reproduces the f32 activation exactly (only the summation order differs from
 * sgemm); planes = 2 (or VOX_HIP_GEMM_PLANES=2) keeps ~2^-18 of it and issues 2/3 of the
 * MFMAs (measured against the 5e-5 parity bar in tests/test_gpu_gemm_planes.py).
 * Process-wide; returns 0, or -1 for another value. */
int vox_hip_set_gemm_planes(int planes);
int vox_hip_gemm_planes(void);
/* Diagnostic (no reference counterpart): the encoder GEMM's stream-K owner waits up to
 * `ticks` (100 MHz) for each later part of a tile before computing that stage range itself
 * (same code and order: same bits); ticks < 0 never waits, so the tests can force that
 * backstop.  Default 5000 (50 us).  Process-wide; returns the previous value. */
int vox_hip_set_gemmf_wait(int ticks);

/* Per-stream device state: encoder/decoder rolling KV, conv-stem tails, adapter buffer,
 * scratch and a HIP stream.  One model serves many streams. */
vox_hip_stream_t *vox_hip_stream_create(vox_hip_model_t *m);
void vox_hip_stream_free(vox_hip_stream_t *s);
/* 1 if the stream's decoder KV rings hold IEEE half (vox_hip_model_set_kv_fp16), else 0 */
int vox_hip_stream_kv_fp16(const vox_hip_stream_t *s);
/* stream_reset_full_state (voxtral.c:786-814) / stream_reset_decoder_state (:766-783) */
int vox_hip_stream_reset(vox_hip_stream_t *s);
int vox_hip_stream_reset_decoder(vox_hip_stream_t *s);

/* ------------------------------------------------------------------------
 * Device-resident streaming pipeline (the fast path).  Inputs are log-mel frames
 * [n, mel_bins] as produced by vox_mel_feed/vox_mel_finish (voxtral_audio.c:560-633).
 * ------------------------------------------------------------------------ */
/* stream_run_encoder body (voxtral.c:845-951): incremental conv stem (voxtral.c:581-759),
 * 32-layer encoder with rolling KV (voxtral_encoder.c:495-693), 4x downsample with the
 * leftover-row residual, adapter (voxtral_encoder.c:699-737); adapter rows stay in HBM.
 * mel is a host pointer (mel_on_device=0) or a device pointer (1).
 * Returns the number of adapter tokens appended, <0 on error. */
int vox_hip_stream_encode_mel(vox_hip_stream_t *s, const float *mel, int n_frames,
                              int mel_on_device);
int vox_hip_stream_adapter_tokens(vox_hip_stream_t *s);
/* on != 0: vox_hip_stream_encode_mel returns once the pass is enqueued on the stream's HIP
 * queue (its adapter-row count is known on the host); everything later on the same stream
 * (decode, read_adapter, reset) is ordered behind it and the batched step waits for every
 * member stream, so a scheduler can have several streams' encoder chunks in flight at once.
 * Host mel pointers must stay valid until vox_hip_stream_sync.  Default 0 (synchronous). */
int vox_hip_stream_set_async_encode(vox_hip_stream_t *s, int on);
/* stream_run_encoder for B streams at once: each stream's conv stem on its own queue, the
 * stacked new rows of all of them through the 32 encoder layers in one pass (projections
 * over all rows: every weight byte read once for the batch; RoPE, K/V append and attention
 * per stream against its own ring), then each stream's downsample + adapter.  The same
 * results as B vox_hip_stream_encode_mel calls up to summation order.  added[b] = adapter
 * rows appended to stream b.  Synchronous unless every stream is in async-encode mode.
 * Returns 0, <0 on error. */
int vox_hip_stream_encode_mel_batch(vox_hip_stream_t *const *streams, const float *const *mels,
                                    const int *n_frames, int B, int mel_on_device, int *added);

/* Incremental log-mel on the device: a vox_mel_ctx_t
 * (voxtral_audio.c:405-671) whose padded sample buffer and frames live in HBM, computed on
 * the stream's HIP queue ahead of the encoder (one block per frame: Hann window, direct
 * 201 x 400 DFT, Slaney filters, log10 clamp).  Frame indices are global, as in the
 * reference (vox_mel_frame_offset + position); a frame's device pointer feeds
 * vox_hip_stream_encode_mel(..., mel_on_device = 1) directly. */
typedef struct vox_hip_mel vox_hip_mel_t;
/* vox_mel_ctx_init (voxtral_audio.c:515-558): 200 + left_pad_samples zeros of padding */
vox_hip_mel_t *vox_hip_mel_create(vox_hip_stream_t *s, int left_pad_samples);
/* vox_mel_feed (voxtral_audio.c:560-582): returns the frames added, <0 on error */
int vox_hip_mel_feed(vox_hip_mel_t *m, const float *samples, int n_samples);
/* vox_mel_finish (voxtral_audio.c:584-633): right_pad zeros, 200-sample reflect, last frame
 * dropped; returns the live frame count */
int vox_hip_mel_finish(vox_hip_mel_t *m, int right_pad_samples);
/* vox_mel_data's count and vox_mel_frame_offset (voxtral_audio.c:635-643) */
int vox_hip_mel_frames(const vox_hip_mel_t *m, int *frame_offset);
/* device pointer of global frame f (frame_offset <= f <= frame_offset + frames) */
const float *vox_hip_mel_frame_ptr(const vox_hip_mel_t *m, int global_frame);
/* vox_mel_discard_before (voxtral_audio.c:645-662) */
int vox_hip_mel_discard_before(vox_hip_mel_t *m, int keep_from_frame);
/* copy live frames [first, first + n) to the host (tests) */
int vox_hip_mel_read(vox_hip_mel_t *m, int global_first, int n, float *out);
/* vox_mel_free (voxtral_audio.c:664-671) */
void vox_hip_mel_free(vox_hip_mel_t *m);
/* The state vox_hip_mel_create leaves (200 + left_pad_samples zeros, no frames), keeping the
 * context's device tables and buffers: a reused stream's new audio (vh_stream_reset). */
int vox_hip_mel_reset(vox_hip_mel_t *m, int left_pad_samples);
/* Copy adapter rows [first, first+n) to host (tests). */
int vox_hip_stream_read_adapter(vox_hip_stream_t *s, int first, int n, float *out);

/* stream_run_decoder (voxtral.c:1013-1145), non-continuous part: prefill when enough
 * adapter tokens exist (prompt BOS + STREAMING_PAD x (32+delay)), then greedy steps
 * while adapter tokens remain.  Generates at most max_steps tokens; stop_at_eos stops
 * after token 2 (EOS).  tokens_out receives the ids; logits_out (may be NULL) receives
 * [n, vocab] logits.  Returns the number of tokens generated (<0 on error). */
int vox_hip_stream_decode(vox_hip_stream_t *s, int max_steps, int stop_at_eos,
                          int *tokens_out, float *logits_out);
/* Alternative tokens (--alt, voxtral.h:294-304).  vox_stream_set_alt (voxtral.c:1329-1337):
 * n_alt clamped to 1..VOX_HIP_MAX_ALT, cutoff to [0,1]; n_alt > 1 makes every later step
 * also keep the softmax candidates of stream_fill_alts (voxtral.c:955-1010) on the device
 * (no logits download).  read_alts returns, for generated steps [first, first+n), the
 * chosen id and the accepted alternatives ([n][VOX_HIP_MAX_ALT], -1 = none) and optionally
 * their probabilities.  Callers apply it to text tokens only, as the reference does. */
#define VOX_HIP_MAX_ALT 4
int vox_hip_stream_set_alt(vox_hip_stream_t *s, int n_alt, float cutoff);
int vox_hip_stream_read_alts(vox_hip_stream_t *s, int first, int n, int *ids_out, float *probs_out);
/* Cross-stream batched greedy decoding (C4; the reference decodes each
 * vox_stream_t separately, voxtral.c:1105-1145).  A batch object holds scratch for up to
 * max_streams (<= 32: two 16-row blocks) streams of one model.  vox_hip_batch_decode advances every listed
 * stream that has adapter rows left by one greedy token per step; the weights are streamed
 * once per step for all of them, attention / KV / argmax use each stream's own state.
 * Streams not started yet whose prompt is complete are prefilled first (several of them in
 * one stacked pass) and take their first token in the batched steps.  Every stream stops on
 * the device when it has used its adapter rows, after max_steps tokens or (stop_at_eos) after
 * EOS, while the others go on; streams join and leave a batch without a graph capture (the
 * step graphs read a device slot table).  Streams with alternatives on
 * (vox_hip_stream_set_alt) stay in the batch and get their stream_fill_alts records.
 * Results and device state are those of vox_hip_stream_decode on each stream (up to f32
 * summation order of the shared GEMMs).  tokens_out: [n][max_steps]; counts_out[n].
 * Returns the total number of tokens, < 0 on error. */
typedef struct vox_hip_batch vox_hip_batch_t;
vox_hip_batch_t *vox_hip_batch_create(vox_hip_model_t *m, int max_streams);
void vox_hip_batch_free(vox_hip_batch_t *b);
int vox_hip_batch_decode(vox_hip_batch_t *b, vox_hip_stream_t **streams, int n, int max_steps,
                         int stop_at_eos, int *tokens_out, int *counts_out);
/* The same with stream i reading only its first rows[i] adapter rows (<= its count), which the
 * caller guarantees are complete; the streams' own queues are not waited for, so an encoder
 * pass enqueued on them after those rows (async encode, vox_hip_stream_encode_mel_batch) runs
 * beside the batched steps (the per-GPU scheduler's overlap, vh_sched_run). */
int vox_hip_batch_decode_rows(vox_hip_batch_t *b, vox_hip_stream_t **streams, int n, const int *rows,
                              int max_steps, int stop_at_eos, int *tokens_out, int *counts_out);
/* vox_hip_batch_decode_rows in two halves: begin enqueues the call's prefills and its first
 * 16 steps on the batch queue and returns without waiting (0, or <0 on error); finish waits,
 * runs any further steps and fills tokens_out / counts_out (which must stay valid in between),
 * returning the total as decode_rows does.  In between the caller may enqueue work on other
 * queues -- the per-GPU scheduler enqueues the cross-stream encoder pass there, after the
 * steps, so the steps are on the device first -- but must not touch the listed streams'
 * decoder state or call another batch function on b. */
int vox_hip_batch_begin_rows(vox_hip_batch_t *b, vox_hip_stream_t **streams, int n, const int *rows,
                             int max_steps, int stop_at_eos, int *tokens_out, int *counts_out);
int vox_hip_batch_finish(vox_hip_batch_t *b);
/* Logits [vocab] of the last batched step, for a stream that step advanced (the logits the
 * reference's vox_decoder_forward returns, voxtral_decoder.c:762-779; for tests and --alt
 * style callers).  Returns 0, or <0 if s was not in that step. */
int vox_hip_batch_read_logits(vox_hip_batch_t *b, vox_hip_stream_t *s, float *out);
/* Counters since creation: [0] calls, [1] step replays, [2] live rows over those steps,
 * [3] step-graph captures, [4] batched prefill passes, [5] prefilled streams. */
int vox_hip_batch_stats(const vox_hip_batch_t *b, long long *out6);
/* Decoder state snapshot: [0]=kv logical length, [1]=next adapter row, [2]=prev token,
 * [3]=started, [4]=eos_seen, [5]=tokens generated. */
int vox_hip_stream_state(vox_hip_stream_t *s, int *out6);

/* ------------------------------------------------------------------------
 * Reference-boundary twins (host pointers in and out, synchronous).  These are what
 * voxtral_encoder.c / voxtral_decoder.c / voxtral_kernels.c call under USE_HIP in
 * place of the vox_metal_* functions.
 * ------------------------------------------------------------------------ */
/* voxtral_metal.h:38  C[M,N] = A[M,K] @ B[N,K]^T (B is a host bf16 weight pointer,
 * uploaded once and cached by pointer like voxtral_metal.m:165-201) */
void vox_hip_sgemm_bf16(int M, int N, int K, const float *A, const uint16_t *B_bf16, float *C);
/* voxtral_metal.h:262-265  C[M,N] = A[M,K] @ (scales[n] * B_q8[N,K])^T (vox_linear_q8 /
 * vox_matmul_t_q8 under USE_HIP, voxtral_kernels.c:316-377); B and scales are host
 * pointers, uploaded once and cached by pointer; bias is added by the caller. */
void vox_hip_sgemm_q8(int M, int N, int K, const float *A, const int8_t *B_q8, const float *scales,
                      float *C);
/* voxtral_metal.h:59 */
void vox_hip_fused_qkv_bf16(int M, int K, const float *input,
                            const uint16_t *wq_bf16, int Nq, const uint16_t *wk_bf16, int Nk,
                            const uint16_t *wv_bf16, int Nv, float *q, float *k, float *v);
/* voxtral_metal.h:86 */
void vox_hip_fused_ffn_bf16(int M, int dim, int hidden, const float *input,
                            const uint16_t *w1_bf16, const uint16_t *w3_bf16,
                            const uint16_t *w2_bf16, float *output);
/* voxtral_metal.h:136  (same semantics as vox_causal_attention, voxtral_kernels.c:541-611) */
void vox_hip_encoder_attention(float *out, const float *Q, const float *K, const float *V,
                               int seq_q, int seq_k, int n_heads, int n_kv_heads,
                               int head_dim, float scale, int window_size, int q_offset);
/* voxtral_metal.h:245  32 encoder layers + final norm in place on host x [new_len, enc_dim];
 * K/V appended to the stream's rolling cache at logical positions
 * logical_start..logical_start+new_len-1.  rope_freqs [new_len, head_dim/2, 2] from the
 * caller (vox_compute_rope_freqs).  Returns 0 / <0. */
int vox_hip_encoder_full_step(vox_hip_stream_t *s, float *x, int new_len,
                              const float *rope_freqs, int logical_start);
/* voxtral_metal.h:254  26 decoder layers on seq_len rows, KV written at logical
 * positions logical_start.. ; x [seq_len, dec_dim] updated in place. */
int vox_hip_decoder_prefill_step(vox_hip_stream_t *s, float *x, int seq_len,
                                 const float *rope_freqs, int logical_start);
/* voxtral_metal.h:161/164  upload the step input / release it */
void vox_hip_decoder_start(vox_hip_stream_t *s, const float *x, int dim);
void vox_hip_decoder_end(vox_hip_stream_t *s);
/* voxtral_metal.h:219  one token through all layers + final norm + LM head + argmax.
 * KV written at logical position logical_pos; returns the argmax id (first max wins,
 * voxtral_decoder.c:771-779) and fills logits [vocab] if non-NULL. */
int vox_hip_decoder_full_step(vox_hip_stream_t *s, const float *rope_freqs, int logical_pos,
                              float *logits);

/* ------------------------------------------------------------------------
 * Timing hooks for the benchmark (HIP events on the stream's own queue).
 * ------------------------------------------------------------------------ */
/* Average device time (ms) of the last decode call's dominant per-layer GEMV launches and
 * the bytes they streamed; filled only when profiling was enabled.  out8: [0] ms, [1] bytes,
 * [2] launches, [3] ms per launch, [5] bytes per launch, [6] encoder-GEMM stage ranges an
 * owner recomputed because a partial tile did not arrive in time (since creation). */
int vox_hip_stream_set_profiling(vox_hip_stream_t *s, int enable);
int vox_hip_stream_profile(vox_hip_stream_t *s, double *out8);
/* Synchronise the stream's HIP queue. */
int vox_hip_stream_sync(vox_hip_stream_t *s);

/* Device buffers for callers that keep their inputs resident in HBM (benchmark, tests). */
void *vox_hip_device_upload(const void *host, size_t bytes);
int vox_hip_device_free(void *dev);

#ifdef __cplusplus
}
#endif
#endif /* VOXTRAL_HIP_H */
