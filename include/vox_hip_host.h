/*
 * vox_hip_host.h -- C host side of the MI355X backend: the reference's model loading and
 * streaming API (voxtral.h:251-337, voxtral.c) rewritten over the C ABI of
 * voxtral_hip.h, in the reference's own language (C99).  A C program that used
 * vox_load / vox_stream_init / vox_stream_feed / vox_stream_finish / vox_stream_get can
 * switch to the vh_* calls one for one; everything between the samples and the token ids
 * (log-mel, conv stem, encoder, adapter, decoder, argmax) runs on the GPU.
 *
 * Differences from the reference API:
 *   - vh_stream_get returns token ids (every generated id, control ids included); the
 *     tokenizer (voxtral_tokenizer.c) stays out of scope;
 *   - WAV input must be 16 kHz mono 16-bit PCM (the reference's loader also converts
 *     other formats, voxtral_audio.c:49-165);
 *   - the text / control / invalid classification the live-mode restarts use
 *     (stream_classify_token, voxtral.c:532-539) works on ids (vh_token_class): the
 *     reference asks its tokenizer whether a text id decodes to an empty string, which for
 *     the Tekken vocabulary is id 1000 (raw byte 0x00).
 */
#ifndef VOX_HIP_HOST_H
#define VOX_HIP_HOST_H

#include "voxtral_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vh_ctx vh_ctx_t;       /* vox_ctx_t twin: one model on one GPU */
typedef struct vh_stream vh_stream_t; /* vox_stream_t twin */

/* Read a consolidated.safetensors header (BF16, or the Q8/F32 layout quantize.py writes)
 * and derive the model dimensions from the tensor shapes, with the reference's fixed
 * constants for what the file does not hold (head dims 64 / 128, windows 750 / 8192,
 * theta 1e6, eps 1e-5; voxtral.h:26-50).  No GPU work.  0 on success. */
int vh_inspect(const char *path, vox_hip_config_t *cfg);

/* vox_load (voxtral.c:131-284): mmap the checkpoint, convert the small tensors to f32 as
 * the reference does, hand the weight table to vox_hip_model_create (which uploads and
 * packs everything into HBM), unmap.  NULL on failure (vh_last_error). */
vh_ctx_t *vh_load(const char *path);
void vh_free(vh_ctx_t *ctx);
const vox_hip_config_t *vh_config(const vh_ctx_t *ctx);
/* vox_set_delay (voxtral.c:1681-1687): clamp to 80..2400 ms, 80 ms per token */
int vh_set_delay(vh_ctx_t *ctx, int delay_ms);
const char *vh_last_error(void);

/* vox_stream_init (voxtral.c:1242-1286) */
vh_stream_t *vh_stream_init(vh_ctx_t *ctx);
void vh_stream_free(vh_stream_t *s);
/* A detached stream back to the state vh_stream_init leaves, keeping its device buffers and its
 * settings (processing interval, live mode, alternatives): new audio on a reused stream, as a
 * server keeps a pool of them, without vh_stream_init's allocations (no reference counterpart;
 * the state reset is stream_reset_full_state's, voxtral.c:786-814).  0, or -1. */
int vh_stream_reset(vh_stream_t *s);
/* vox_set_processing_interval (voxtral.c:1669-1675) */
void vh_set_processing_interval(vh_stream_t *s, float seconds);
/* vox_stream_feed / vox_stream_flush / vox_stream_finish (voxtral.c:1288-1316,
 * 1640-1667): 0 on success, -1 on error or after finish */
int vh_stream_feed(vh_stream_t *s, const float *samples, int n_samples);
int vh_stream_flush(vh_stream_t *s);
int vh_stream_finish(vh_stream_t *s);
/* vox_stream_get (voxtral.c:1319-1327), ids instead of strings: up to max queued ids */
int vh_stream_get(vh_stream_t *s, int *ids, int max);

/* vox_stream_set_continuous (voxtral.c:1677-1679): live mode (main.c enables it for --stdin
 * and the microphone).  After each decoder drain the decoder restarts on EOS, on more than
 * 2000 KV positions, on 64 non-text tokens in a row, or after 20 s of fed audio without a
 * decoded token; restarts other than EOS, and two EOS restarts in a row without text,
 * reset the whole stream (mel, conv stem, encoder, decoder; voxtral.c:410-420, 1189-1239). */
void vh_stream_set_continuous(vh_stream_t *s, int on);

/* vox_stream_set_alt (voxtral.c:1329-1337): n_alt clamped to 1..VH_MAX_ALT, cutoff to
 * [0, 1]; candidates are kept on the device per step (stream_fill_alts, voxtral.c:955-1010) */
#define VH_MAX_ALT 4
int vh_stream_set_alt(vh_stream_t *s, int n_alt, float cutoff);
/* vox_stream_get_alt (voxtral.c:1339-1353), ids: up to max records of VH_MAX_ALT ints --
 * the chosen id, then its accepted alternatives (text tokens only), -1 for none */
int vh_stream_get_alt(vh_stream_t *s, int *records, int max);

/* stream_classify_token (voxtral.c:532-539) on ids */
enum { VH_TOK_TEXT = 0, VH_TOK_CONTROL = 1, VH_TOK_INVALID = 2, VH_TOK_EOS = 3 };
int vh_token_class(int id);
/* the stats vox_stream_free prints (voxtral.c:1358-1370) */
typedef struct {
    int mel_frames, adapter_tokens, generated, chunks;
    double encoder_ms, decoder_ms, prefill_ms;
    int restarts, full_resets;   /* continuous mode */
} vh_stats_t;
void vh_stream_stats(const vh_stream_t *s, vh_stats_t *out);
/* adapter rows the stream's decoder has not consumed yet (0 once it has drained them or met
 * EOS); a scheduled stream with a step cap (vh_sched_set_step_cap) may finish its feeds with
 * rows still pending */
int vh_stream_pending(vh_stream_t *s);

/* Wrap a model the caller created with vox_hip_model_create (Python mirror, servers that
 * load once and share): vh_free on the result leaves the model alone. */
vh_ctx_t *vh_ctx_wrap(vox_hip_model_t *model, const vox_hip_config_t *cfg, int delay_tokens);

/* Per-GPU stream scheduler.  The reference decodes each vox_stream_t on its
 * own: stream_run_decoder's token loop (voxtral.c:1105-1145) streams every decoder weight
 * once per token per stream.  A scheduler owns up to VH_SCHED_MAX streams of one model on
 * one GPU; attached streams run their mel front-end and encoder in vh_stream_feed / flush /
 * finish as audio arrives, and leave the decoder to vh_sched_run, which
 *   0. encodes the chunk every attached stream deferred since the last run (its feeds leave
 *      the chunk's frames in place) in one vox_hip_stream_encode_mel_batch pass: the encoder
 *      weights are read once for all streams (VOX_HIP_SCHED_BATCH_ENC=0: each chunk alone),
 *   1-2. advances every stream whose decoder can run by batched greedy steps
 *      (vox_hip_batch_decode: one weight read per step for all of them, attention / KV /
 *      argmax per stream): streams whose prompt rows just completed are prefilled together
 *      in one stacked pass and take their first token in the batched steps, and every stream
 *      stops on the device when it has used its adapter rows or produced EOS,
 *   3. waits for step 0's pass when it ran beside the steps (below),
 *   4. applies each stream's live-mode restarts (vh_stream_set_continuous) as run after its
 *      own drain.
 * By default (VOX_HIP_SCHED_OVERLAP=0: off; off too while a live-mode stream is attached) step
 * 0's pass is only enqueued and steps 1-2 decode the rows that were complete when the run
 * started (vox_hip_batch_decode_rows), so the pass runs beside the batched steps; it completes
 * before the run returns and its rows are decoded by the next run.  Greedy ids do not depend
 * on when a row is decoded.  vh_stream_pending counts those rows.
 * Called after every round of feeds, it yields per stream the ids vh_stream_feed would have
 * queued (vh_stream_get / get_alt read them as before).  Streams with --alt (n_alt > 1) stay
 * in the batch (the batched argmax keeps their candidates); a live-mode stream drains on its
 * own path inside vh_stream_flush (and so inside vh_stream_finish), where the reference's
 * restart checks run between the flush and the final chunk. */
#define VH_SCHED_MAX 32
typedef struct vh_sched vh_sched_t;
typedef struct {
    int runs, prefills, batch_calls;
    long long tokens;        /* ids from batched steps */
    double run_ms, batch_ms; /* wall time in vh_sched_run / in vox_hip_batch_decode */
    int enc_batches;         /* batched encoder passes (step 0) */
    long long steps;         /* batched step replays (tokens / steps = rows per step) */
    long long captures;      /* step-graph captures (vox_hip_batch_stats) */
    long long prefill_passes;/* prefill passes (several new streams share one) */
    double enc_ms;           /* wall time of the batched encoder passes (step 0: to completion;
                              * with the overlap, the enqueue only) */
} vh_sched_stats_t;
vh_sched_t *vh_sched_create(vh_ctx_t *ctx, int max_streams);
void vh_sched_free(vh_sched_t *q);          /* detaches its streams */
int vh_sched_attach(vh_sched_t *q, vh_stream_t *s);
int vh_sched_detach(vh_sched_t *q, vh_stream_t *s);
int vh_sched_run(vh_sched_t *q);            /* ids generated, < 0 on error */
void vh_sched_stats(const vh_sched_t *q, vh_sched_stats_t *out);
/* Serving policy (no reference counterpart): cap > 0 advances each stream by at most `cap`
 * greedy steps per vh_sched_run, so a stream with a burst of rows (its prompt, the flush
 * padding of vox_stream_flush) spreads them over the next runs inside full batched steps
 * instead of stepping alone; ids are unchanged, only their timing.  Run until every
 * stream's vh_stream_pending is 0 to drain.  cap <= 0 (the default): every run drains every
 * stream, as vox_stream_feed does. */
void vh_sched_set_step_cap(vh_sched_t *q, int cap);

/* vox_load_wav (voxtral_audio.c:49-166): 16-bit PCM WAV of any channel count and rate, mixed
 * to mono and linearly resampled to 16 kHz as the reference does: malloc'd samples */
float *vh_load_wav(const char *path, int *n_samples);

#ifdef __cplusplus
}
#endif
#endif
