/*
 * vox_hip_transcribe -- main.c's file mode (main.c:107-118, 126-210, 383-410) on the
 * MI355X backend through the C host API (include/vox_hip_host.h):
 *
 *   vox_hip_transcribe -d consolidated.safetensors -i audio.wav [-I secs] [--delay ms]
 *
 * The audio is fed in pieces of min(interval, 1 s) of samples, as main.c's feed_and_drain
 * does; every generated token id is printed to stdout (the tokenizer is out of scope), and
 * the reference's stderr lines ("Audio:", "Encoder:", "Decoder:") are kept so its
 * benchmark.py regexes parse this program's output too.
 */
#include "../../include/vox_hip_host.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define DEFAULT_FEED_CHUNK 16000  /* main.c: 1 s of samples */

static void drain(vh_stream_t *s, int *text_tokens) {
    int ids[256], n;
    while ((n = vh_stream_get(s, ids, 256)) > 0)
        for (int i = 0; i < n; i++) {
            printf("%d ", ids[i]);
            if (ids[i] >= 1000) (*text_tokens)++;  /* TOKEN_TEXT_MIN (voxtral.c:399) */
        }
    fflush(stdout);
}

int main(int argc, char **argv) {
    const char *model = NULL, *wav = NULL;
    float interval = -1.0f;
    int delay_ms = -1;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-d") && i + 1 < argc) model = argv[++i];
        else if (!strcmp(argv[i], "-i") && i + 1 < argc) wav = argv[++i];
        else if (!strcmp(argv[i], "-I") && i + 1 < argc) interval = (float)atof(argv[++i]);
        else if (!strcmp(argv[i], "--delay") && i + 1 < argc) delay_ms = atoi(argv[++i]);
        else {
            fprintf(stderr, "usage: %s -d consolidated.safetensors -i audio.wav [-I secs] [--delay ms]\n", argv[0]);
            return 2;
        }
    }
    if (!model || !wav) {
        fprintf(stderr, "usage: %s -d consolidated.safetensors -i audio.wav [-I secs] [--delay ms]\n", argv[0]);
        return 2;
    }
    vh_ctx_t *ctx = vh_load(model);
    if (!ctx) return 1;
    if (delay_ms > 0 && vh_set_delay(ctx, delay_ms)) return 1;
    vh_stream_t *s = vh_stream_init(ctx);
    if (!s) return 1;
    int feed_chunk = DEFAULT_FEED_CHUNK;
    if (interval > 0) {
        vh_set_processing_interval(s, interval);
        feed_chunk = (int)(interval * 16000);
        if (feed_chunk < 160) feed_chunk = 160;
        if (feed_chunk > DEFAULT_FEED_CHUNK) feed_chunk = DEFAULT_FEED_CHUNK;
    }
    int n = 0;
    float *samples = vh_load_wav(wav, &n);
    if (!samples) return 1;
    fprintf(stderr, "Audio: %d samples (%.1f seconds)\n", n, (float)n / 16000.0f);
    int text_tokens = 0, rc = 0;
    for (int off = 0; off < n && !rc; off += feed_chunk) {
        const int chunk = n - off < feed_chunk ? n - off : feed_chunk;
        rc = vh_stream_feed(s, samples + off, chunk);
        drain(s, &text_tokens);
    }
    free(samples);
    if (!rc) rc = vh_stream_finish(s);
    drain(s, &text_tokens);
    printf("\n");
    vh_stats_t st;
    vh_stream_stats(s, &st);
    /* the lines vox_stream_free prints (voxtral.c:1358-1370) */
    fprintf(stderr, "Encoder: %d mel -> %d tokens (%.0f ms)\n", st.mel_frames, st.adapter_tokens, st.encoder_ms);
    if (st.generated > 0) {
        const double gen_ms = st.decoder_ms - st.prefill_ms;
        fprintf(stderr, "Decoder: %d text tokens (%d steps) in %.0f ms (prefill %.0f ms + %.1f ms/step)\n",
                text_tokens, st.generated, st.decoder_ms, st.prefill_ms,
                st.generated > 1 ? gen_ms / (st.generated - 1) : 0.0);
    }
    vh_stream_free(s);
    vh_free(ctx);
    return rc ? 1 : 0;
}
