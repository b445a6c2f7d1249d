/*
 * vox_hip_transcribe -- main.c's file mode (main.c:107-118, 126-210, 383-410) on the
 * MI355X backend through the C host API (include/vox_hip_host.h):
 *
 *   vox_hip_transcribe -d consolidated.safetensors -i audio.wav [-I secs] [--delay ms]
 *                      [--alt cutoff] [--continuous]
 *
 * The audio is fed in pieces of min(interval, 1 s) of samples, as main.c's feed_and_drain
 * does; every generated token id is printed to stdout (the tokenizer is out of scope) --
 * with --alt (main.c:149-154, 3 candidates) as id|alt|alt for the accepted alternatives.
 * --continuous turns on live mode (vox_stream_set_continuous, which main.c sets for --stdin
 * and the microphone, main.c:208-209) on the file's samples.  The
 * the reference's stderr lines ("Audio:", "Encoder:", "Decoder:") are kept so its
 * benchmark.py regexes parse this program's output too.
 */
#include "../../include/vox_hip_host.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define DEFAULT_FEED_CHUNK 16000  /* main.c: 1 s of samples */

static void drain(vh_stream_t *s, int *text_tokens, int alt) {
    int rec[256 * VH_MAX_ALT], n;
    while ((n = vh_stream_get_alt(s, rec, 256)) > 0)
        for (int i = 0; i < n; i++) {
            const int *r = rec + i * VH_MAX_ALT;
            printf("%d", r[0]);
            for (int a = 1; alt && a < VH_MAX_ALT && r[a] >= 0; a++) printf("|%d", r[a]);
            printf(" ");
            if (vh_token_class(r[0]) == VH_TOK_TEXT) (*text_tokens)++;
        }
    fflush(stdout);
}

int main(int argc, char **argv) {
    const char *model = NULL, *wav = NULL;
    float interval = -1.0f, alt_cutoff = -1.0f;
    int delay_ms = -1, continuous = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-d") && i + 1 < argc) model = argv[++i];
        else if (!strcmp(argv[i], "-i") && i + 1 < argc) wav = argv[++i];
        else if (!strcmp(argv[i], "-I") && i + 1 < argc) interval = (float)atof(argv[++i]);
        else if (!strcmp(argv[i], "--delay") && i + 1 < argc) delay_ms = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--alt") && i + 1 < argc) alt_cutoff = (float)atof(argv[++i]);
        else if (!strcmp(argv[i], "--continuous")) continuous = 1;
        else {
            model = NULL;
            break;
        }
    }
    if (!model || !wav || (alt_cutoff != -1.0f && (alt_cutoff < 0 || alt_cutoff > 1))) {
        fprintf(stderr, "usage: %s -d consolidated.safetensors -i audio.wav [-I secs] [--delay ms] "
                        "[--alt 0..1] [--continuous]\n", argv[0]);
        return 2;
    }
    vh_ctx_t *ctx = vh_load(model);
    if (!ctx) return 1;
    if (delay_ms > 0 && vh_set_delay(ctx, delay_ms)) return 1;
    vh_stream_t *s = vh_stream_init(ctx);
    if (!s) return 1;
    if (alt_cutoff >= 0 && vh_stream_set_alt(s, 3, alt_cutoff)) return 1;  /* main.c:197-198 */
    vh_stream_set_continuous(s, continuous);
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
        drain(s, &text_tokens, alt_cutoff >= 0);
    }
    free(samples);
    if (!rc) rc = vh_stream_finish(s);
    drain(s, &text_tokens, alt_cutoff >= 0);
    printf("\n");
    vh_stats_t st;
    vh_stream_stats(s, &st);
    /* the lines vox_stream_free prints (voxtral.c:1358-1370) */
    fprintf(stderr, "Encoder: %d mel -> %d tokens (%.0f ms)\n", st.mel_frames, st.adapter_tokens, st.encoder_ms);
    if (continuous) fprintf(stderr, "Restarts: %d (%d full)\n", st.restarts, st.full_resets);
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
