/*
 * vox_hip_host.c -- the reference's loader and streaming driver in C99 over the MI355X C
 * ABI (include/voxtral_hip.h).  See include/vox_hip_host.h.
 *
 * Model load: voxtral.c:131-284 + voxtral_safetensors.c (header parse, bf16 / Q8 / F32
 * tensors).  Streaming: stream_run_encoder gating (voxtral.c:827-851), stream_run_decoder
 * draining (1013-1145, non-continuous), vox_stream_feed / flush / finish (1288-1316,
 * 1640-1667).  The mel front-end, encoder and decoder all run on the device
 * (vox_hip_mel_*, vox_hip_stream_encode_mel, vox_hip_stream_decode).
 */
#define _POSIX_C_SOURCE 200809L
#include "../../include/vox_hip_host.h"

#include <fcntl.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define STREAM_FIRST_CHUNK_MIN_MEL 312  /* voxtral.c:405 */
#define STREAM_DEFAULT_INTERVAL 2.0f    /* voxtral.c:408 */
#define RAW_AUDIO_LENGTH_PER_TOK 1280   /* voxtral.c:400 */
#define OFFLINE_STREAMING_BUFFER_TOKENS 10 /* voxtral.c:401 */
#define ENC_PREFIX "mm_streams_embeddings.embedding_module.whisper_encoder"
#define EMB_PREFIX "mm_streams_embeddings.embedding_module"

static char g_err[512];

static int fail(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    fprintf(stderr, "vox_hip_host: %s\n", g_err);
    return -1;
}

const char *vh_last_error(void) { return g_err; }

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

/* ------------------------------------------------------------------------
 * safetensors: 8-byte little-endian header length, JSON object
 * {name: {"dtype": s, "shape": [..], "data_offsets": [begin, end]}, "__metadata__": {..}}
 * ------------------------------------------------------------------------ */
enum { DT_BF16, DT_F32, DT_Q8, DT_OTHER };
typedef struct {
    char name[160];
    int dtype, ndim;
    long long shape[4];
    size_t begin, end;
} st_tensor_t;

typedef struct {
    int fd;
    uint8_t *map;
    size_t size, base;
    st_tensor_t *t;
    int n;
} st_file_t;

static void ws(const char **p) {
    while (**p == ' ' || **p == '\n' || **p == '\r' || **p == '\t') (*p)++;
}

/* a JSON string into buf (no escapes occur in tensor names or dtypes) */
static int jstr(const char **p, char *buf, size_t cap) {
    ws(p);
    if (**p != '"') return -1;
    (*p)++;
    size_t n = 0;
    while (**p && **p != '"') {
        if (**p == '\\' && (*p)[1]) (*p)++;
        if (n + 1 < cap) buf[n++] = **p;
        (*p)++;
    }
    if (**p != '"') return -1;
    (*p)++;
    buf[n] = 0;
    return 0;
}

static int jskip(const char **p);

static int jskip_container(const char **p, char open, char close) {
    if (**p != open) return -1;
    (*p)++;
    ws(p);
    if (**p == close) {
        (*p)++;
        return 0;
    }
    for (;;) {
        if (open == '{') {
            char k[256];
            if (jstr(p, k, sizeof k)) return -1;
            ws(p);
            if (**p != ':') return -1;
            (*p)++;
        }
        if (jskip(p)) return -1;
        ws(p);
        if (**p == ',') {
            (*p)++;
            continue;
        }
        if (**p == close) {
            (*p)++;
            return 0;
        }
        return -1;
    }
}

static int jskip(const char **p) {
    ws(p);
    if (**p == '{') return jskip_container(p, '{', '}');
    if (**p == '[') return jskip_container(p, '[', ']');
    if (**p == '"') {
        char tmp[512];
        return jstr(p, tmp, sizeof tmp);
    }
    while (**p && **p != ',' && **p != '}' && **p != ']') (*p)++;
    return 0;
}

static int jints(const char **p, long long *out, int cap) {
    ws(p);
    if (**p != '[') return -1;
    (*p)++;
    int n = 0;
    for (;;) {
        ws(p);
        if (**p == ']') {
            (*p)++;
            return n;
        }
        char *e;
        long long v = strtoll(*p, &e, 10);
        if (e == *p) return -1;
        if (n < cap) out[n] = v;
        n++;
        *p = e;
        ws(p);
        if (**p == ',') (*p)++;
    }
}

/* byte length must match shape and dtype: BF16 2 B / F32 4 B per element; Q8 (quantize.py
 * layout, voxtral_safetensors.c:457-468) rows f32 scales + rows * cols int8 */
static int st_check_bytes(const st_tensor_t *t) {
    long long n = 1;
    for (int i = 0; i < t->ndim; i++) {
        if (t->shape[i] < 0 || (t->shape[i] && n > (1LL << 40) / t->shape[i])) return -1;
        n *= t->shape[i];
    }
    const size_t len = t->end - t->begin;
    switch (t->dtype) {
        case DT_BF16: return len == (size_t)n * 2 ? 0 : -1;
        case DT_F32: return len == (size_t)n * 4 ? 0 : -1;
        case DT_Q8: {
            if (t->ndim < 1 || t->shape[0] <= 0) return -1;
            const long long rows = t->shape[0];
            return len == (size_t)rows * 4 + (size_t)n ? 0 : -1;
        }
        default: return 0; /* other dtypes are never read */
    }
}

static void st_close(st_file_t *f) {
    if (f->map && f->map != MAP_FAILED) munmap(f->map, f->size);
    if (f->fd >= 0) close(f->fd);
    free(f->t);
    memset(f, 0, sizeof *f);
    f->fd = -1;
}

static int st_open(st_file_t *f, const char *path) {
    memset(f, 0, sizeof *f);
    f->fd = open(path, O_RDONLY);
    if (f->fd < 0) return fail("cannot open %s", path);
    struct stat sb;
    if (fstat(f->fd, &sb) || sb.st_size < 16) return fail("%s: not a safetensors file", path);
    f->size = (size_t)sb.st_size;
    f->map = mmap(NULL, f->size, PROT_READ, MAP_PRIVATE, f->fd, 0);
    if (f->map == MAP_FAILED) return fail("%s: mmap failed", path);
    uint64_t hl = 0;
    memcpy(&hl, f->map, 8);
    /* overflow-safe (voxtral_safetensors.c:236-240 tests header_size > file_size - 8) */
    if (hl == 0 || hl > f->size - 8) return fail("%s: bad header length", path);
    char *hdr = malloc(hl + 1);
    memcpy(hdr, f->map + 8, hl);
    hdr[hl] = 0;
    f->base = 8 + hl;
    int cap = 1024;
    f->t = calloc(cap, sizeof *f->t);
    const char *p = hdr;
    int rc = -1;
    ws(&p);
    if (*p != '{') goto done;
    p++;
    for (;;) {
        ws(&p);
        if (*p == '}') {
            rc = 0;
            break;
        }
        char name[160];
        if (jstr(&p, name, sizeof name)) goto done;
        ws(&p);
        if (*p != ':') goto done;
        p++;
        ws(&p);
        if (!strcmp(name, "__metadata__")) {
            if (jskip(&p)) goto done;
        } else {
            if (*p != '{') goto done;
            p++;
            if (f->n == cap) {
                cap *= 2;
                f->t = realloc(f->t, cap * sizeof *f->t);
            }
            st_tensor_t *t = &f->t[f->n];
            memset(t, 0, sizeof *t);
            snprintf(t->name, sizeof t->name, "%s", name);
            for (;;) {
                ws(&p);
                if (*p == '}') {
                    p++;
                    break;
                }
                char key[64];
                if (jstr(&p, key, sizeof key)) goto done;
                ws(&p);
                if (*p != ':') goto done;
                p++;
                if (!strcmp(key, "dtype")) {
                    char dt[32];
                    if (jstr(&p, dt, sizeof dt)) goto done;
                    t->dtype = !strcmp(dt, "BF16") ? DT_BF16 : !strcmp(dt, "F32") ? DT_F32 : !strcmp(dt, "Q8") ? DT_Q8 : DT_OTHER;
                } else if (!strcmp(key, "shape")) {
                    t->ndim = jints(&p, t->shape, 4);
                    if (t->ndim < 0 || t->ndim > 4) goto done;
                } else if (!strcmp(key, "data_offsets")) {
                    long long o[2];
                    if (jints(&p, o, 2) != 2) goto done;
                    t->begin = (size_t)o[0];
                    t->end = (size_t)o[1];
                } else if (jskip(&p)) {
                    goto done;
                }
                ws(&p);
                if (*p == ',') p++;
            }
            if (t->end < t->begin || t->end > f->size - f->base) goto done;
            if (st_check_bytes(t)) goto done;
            f->n++;
        }
        ws(&p);
        if (*p == ',') p++;
    }
done:
    free(hdr);
    if (rc) return fail("%s: malformed safetensors header", path);
    return 0;
}

static const st_tensor_t *st_find(const st_file_t *f, const char *name) {
    for (int i = 0; i < f->n; i++)
        if (!strcmp(f->t[i].name, name)) return &f->t[i];
    return NULL;
}

static long long st_numel(const st_tensor_t *t) {
    long long n = 1;
    for (int i = 0; i < t->ndim; i++) n *= t->shape[i];
    return n;
}

/* ------------------------------------------------------------------------
 * Model dimensions from the shapes (voxtral.h:26-50 constants for the rest)
 * ------------------------------------------------------------------------ */
static int count_layers(const st_file_t *f, const char *fmt) {
    char nm[200];
    int n = 0;
    for (;;) {
        snprintf(nm, sizeof nm, fmt, n);
        if (!st_find(f, nm)) return n;
        n++;
    }
}

static int infer_config(const st_file_t *f, vox_hip_config_t *c) {
    memset(c, 0, sizeof *c);
    const st_tensor_t *conv0 = st_find(f, ENC_PREFIX ".conv_layers.0.conv.weight");
    const st_tensor_t *ewq = st_find(f, ENC_PREFIX ".transformer.layers.0.attention.wq.weight");
    const st_tensor_t *ewk = st_find(f, ENC_PREFIX ".transformer.layers.0.attention.wk.weight");
    const st_tensor_t *ew1 = st_find(f, ENC_PREFIX ".transformer.layers.0.feed_forward.w1.weight");
    const st_tensor_t *ad0 = st_find(f, EMB_PREFIX ".audio_language_projection.0.weight");
    const st_tensor_t *emb = st_find(f, EMB_PREFIX ".tok_embeddings.weight");
    const st_tensor_t *dwq = st_find(f, "layers.0.attention.wq.weight");
    const st_tensor_t *dwk = st_find(f, "layers.0.attention.wk.weight");
    const st_tensor_t *dw1 = st_find(f, "layers.0.feed_forward.w1.weight");
    const st_tensor_t *ada = st_find(f, "layers.0.ada_rms_norm_t_cond.0.weight");
    if (!conv0 || !ewq || !ewk || !ew1 || !ad0 || !emb || !dwq || !dwk || !dw1 || !ada || conv0->ndim != 3)
        return fail("checkpoint lacks the Voxtral tensors (voxtral_safetensors.c names)");
    c->enc_dim = (int)conv0->shape[0];
    c->mel_bins = (int)conv0->shape[1];
    c->enc_layers = count_layers(f, ENC_PREFIX ".transformer.layers.%d.attention.wq.weight");
    c->enc_head_dim = 64;                      /* VOX_ENC_HEAD_DIM */
    c->enc_heads = (int)ewq->shape[0] / 64;
    c->enc_kv_heads = (int)ewk->shape[0] / 64;
    c->enc_hidden = (int)ew1->shape[0];
    c->enc_window = 750;                       /* VOX_ENC_WINDOW */
    c->downsample = (int)(ad0->shape[1] / c->enc_dim);
    c->dec_dim = (int)emb->shape[1];
    c->vocab = (int)emb->shape[0];
    c->dec_layers = count_layers(f, "layers.%d.attention.wq.weight");
    c->dec_head_dim = 128;                     /* VOX_DEC_HEAD_DIM */
    c->dec_heads = (int)dwq->shape[0] / 128;
    c->dec_kv_heads = (int)dwk->shape[0] / 128;
    c->dec_hidden = (int)dw1->shape[0];
    c->dec_window = 8192;                      /* VOX_DEC_WINDOW */
    c->ada_dim = (int)ada->shape[0];
    c->rope_theta = 1e6f;
    c->enc_eps = 1e-5f;
    c->dec_eps = 1e-5f;
    c->gelu_erf = 0;
    return 0;
}

int vh_inspect(const char *path, vox_hip_config_t *cfg) {
    st_file_t f;
    if (st_open(&f, path)) {
        st_close(&f);
        return -1;
    }
    int rc = infer_config(&f, cfg);
    st_close(&f);
    return rc;
}

/* ------------------------------------------------------------------------
 * Weight table (voxtral.c:131-284): matrices straight off the mapping (bf16), or int8
 * data + copied f32 row scales (Q8, quantize.py packs them unaligned); small tensors as f32
 * ------------------------------------------------------------------------ */
typedef struct {
    void **allocs;
    int n, cap;
} arena_t;

static void *arena_add(arena_t *a, void *p) {
    if (!p) return NULL;
    if (a->n == a->cap) {
        a->cap = a->cap ? 2 * a->cap : 256;
        a->allocs = realloc(a->allocs, a->cap * sizeof(void *));
    }
    a->allocs[a->n++] = p;
    return p;
}

static void arena_free(arena_t *a) {
    for (int i = 0; i < a->n; i++) free(a->allocs[i]);
    free(a->allocs);
    memset(a, 0, sizeof *a);
}

typedef struct {
    const st_file_t *f;
    arena_t *a;
    int bad;
} loader_t;

/* tensor as f32 (bf16 widened exactly, Q8 dequantised as safetensors_get_f32 does) */
static const float *load_f32(loader_t *L, const char *name) {
    const st_tensor_t *t = st_find(L->f, name);
    if (!t) {
        L->bad = fail("missing tensor %s", name);
        return NULL;
    }
    const uint8_t *src = L->f->map + L->f->base + t->begin;
    const long long n = st_numel(t);
    float *out = arena_add(L->a, malloc((size_t)n * 4));
    if (t->dtype == DT_F32) {
        memcpy(out, src, (size_t)n * 4);
    } else if (t->dtype == DT_BF16) {
        for (long long i = 0; i < n; i++) {
            uint16_t b;
            memcpy(&b, src + 2 * i, 2);
            uint32_t u = (uint32_t)b << 16;
            memcpy(&out[i], &u, 4);
        }
    } else if (t->dtype == DT_Q8 && t->ndim == 2) {
        const long long rows = t->shape[0], cols = t->shape[1];
        for (long long r = 0; r < rows; r++) {
            float sc;
            memcpy(&sc, src + 4 * r, 4);
            const int8_t *q = (const int8_t *)(src + rows * 4 + r * cols);
            for (long long k = 0; k < cols; k++) out[r * cols + k] = (float)q[k] * sc;
        }
    } else {
        L->bad = fail("%s: unsupported dtype", name);
        return NULL;
    }
    return out;
}

/* matrix: bf16 data pointer, or int8 data with its row scales (*scales set) */
static const uint16_t *load_mat(loader_t *L, const char *name, const float **scales) {
    const st_tensor_t *t = st_find(L->f, name);
    *scales = NULL;
    if (!t || t->ndim != 2) {
        L->bad = fail("missing matrix %s", name);
        return NULL;
    }
    const uint8_t *src = L->f->map + L->f->base + t->begin;
    if (t->dtype == DT_BF16) return (const uint16_t *)src;
    if (t->dtype == DT_Q8) {
        const long long rows = t->shape[0];
        float *sc = arena_add(L->a, malloc((size_t)rows * 4));
        memcpy(sc, src, (size_t)rows * 4);
        *scales = sc;
        return (const uint16_t *)(src + rows * 4);
    }
    L->bad = fail("%s: matrices must be BF16 or Q8", name);
    return NULL;
}

struct vh_ctx {
    vox_hip_config_t cfg;
    vox_hip_model_t *model;
    int delay_tokens;
    int owns_model;   /* 0: vh_ctx_wrap of a caller's model */
};

vh_ctx_t *vh_ctx_wrap(vox_hip_model_t *model, const vox_hip_config_t *cfg, int delay_tokens) {
    if (!model || !cfg) {
        fail("vh_ctx_wrap: null model or config");
        return NULL;
    }
    vh_ctx_t *ctx = calloc(1, sizeof *ctx);
    ctx->cfg = *cfg;
    ctx->model = model;
    ctx->delay_tokens = delay_tokens;
    return ctx;
}

const vox_hip_config_t *vh_config(const vh_ctx_t *ctx) { return &ctx->cfg; }

#define NAMEBUF 200

vh_ctx_t *vh_load(const char *path) {
    if (!vox_hip_init()) {
        fail("no HIP device: %s", vox_hip_last_error());
        return NULL;
    }
    st_file_t f;
    if (st_open(&f, path)) {
        st_close(&f);
        return NULL;
    }
    vh_ctx_t *ctx = calloc(1, sizeof *ctx);
    if (infer_config(&f, &ctx->cfg)) {
        st_close(&f);
        free(ctx);
        return NULL;
    }
    const vox_hip_config_t *c = &ctx->cfg;
    arena_t a = {0};
    loader_t L = {&f, &a, 0};
    vox_hip_weights_t w;
    memset(&w, 0, sizeof w);
    const int EL = c->enc_layers, DL = c->dec_layers;
    char nm[NAMEBUF];
    w.conv0_w = load_f32(&L, ENC_PREFIX ".conv_layers.0.conv.weight");
    w.conv0_b = load_f32(&L, ENC_PREFIX ".conv_layers.0.conv.bias");
    w.conv1_w = load_f32(&L, ENC_PREFIX ".conv_layers.1.conv.weight");
    w.conv1_b = load_f32(&L, ENC_PREFIX ".conv_layers.1.conv.bias");
#define PTRS(n) arena_add(&a, calloc((size_t)(n), sizeof(void *)))
    /* per-layer matrices: data pointer array + scale array */
    const char *enc_mats[7] = {"attention.wq.weight", "attention.wk.weight", "attention.wv.weight", "attention.wo.weight",
                               "feed_forward.w1.weight", "feed_forward.w2.weight", "feed_forward.w3.weight"};
    const uint16_t **ed[7];
    const float **es[7];
    for (int m = 0; m < 7; m++) {
        ed[m] = PTRS(EL);
        es[m] = PTRS(EL);
        for (int l = 0; l < EL; l++) {
            snprintf(nm, sizeof nm, ENC_PREFIX ".transformer.layers.%d.%s", l, enc_mats[m]);
            ed[m][l] = load_mat(&L, nm, &es[m][l]);
        }
    }
    const int q8 = es[0][0] != NULL;
    w.enc_wq = ed[0]; w.enc_wk = ed[1]; w.enc_wv = ed[2]; w.enc_wo = ed[3];
    w.enc_w1 = ed[4]; w.enc_w2 = ed[5]; w.enc_w3 = ed[6];
    if (q8) {
        w.enc_wq_s = es[0]; w.enc_wk_s = es[1]; w.enc_wv_s = es[2]; w.enc_wo_s = es[3];
        w.enc_w1_s = es[4]; w.enc_w2_s = es[5]; w.enc_w3_s = es[6];
    }
    const char *enc_vecs[6] = {"attention.wq.bias", "attention.wv.bias", "attention.wo.bias",
                               "feed_forward.w2.bias", "attention_norm.weight", "ffn_norm.weight"};
    const float **ev[6];
    for (int v = 0; v < 6; v++) {
        ev[v] = PTRS(EL);
        for (int l = 0; l < EL; l++) {
            snprintf(nm, sizeof nm, ENC_PREFIX ".transformer.layers.%d.%s", l, enc_vecs[v]);
            ev[v][l] = load_f32(&L, nm);
        }
    }
    w.enc_wq_b = ev[0]; w.enc_wv_b = ev[1]; w.enc_wo_b = ev[2]; w.enc_w2_b = ev[3];
    w.enc_attn_norm = ev[4]; w.enc_ffn_norm = ev[5];
    w.enc_norm = load_f32(&L, ENC_PREFIX ".transformer.norm.weight");
    w.ad0 = load_mat(&L, EMB_PREFIX ".audio_language_projection.0.weight", &w.ad0_s);
    w.ad1 = load_mat(&L, EMB_PREFIX ".audio_language_projection.2.weight", &w.ad1_s);
    w.tok_emb = load_mat(&L, EMB_PREFIX ".tok_embeddings.weight", &w.tok_emb_s);
    const char *dec_mats[7] = {"attention.wq.weight", "attention.wk.weight", "attention.wv.weight", "attention.wo.weight",
                               "feed_forward.w1.weight", "feed_forward.w2.weight", "feed_forward.w3.weight"};
    const uint16_t **dd[7];
    const float **dsc[7];
    for (int m = 0; m < 7; m++) {
        dd[m] = PTRS(DL);
        dsc[m] = PTRS(DL);
        for (int l = 0; l < DL; l++) {
            snprintf(nm, sizeof nm, "layers.%d.%s", l, dec_mats[m]);
            dd[m][l] = load_mat(&L, nm, &dsc[m][l]);
        }
    }
    w.dec_wq = dd[0]; w.dec_wk = dd[1]; w.dec_wv = dd[2]; w.dec_wo = dd[3];
    w.dec_w1 = dd[4]; w.dec_w2 = dd[5]; w.dec_w3 = dd[6];
    if (q8) {
        w.dec_wq_s = dsc[0]; w.dec_wk_s = dsc[1]; w.dec_wv_s = dsc[2]; w.dec_wo_s = dsc[3];
        w.dec_w1_s = dsc[4]; w.dec_w2_s = dsc[5]; w.dec_w3_s = dsc[6];
    }
    const char *dec_vecs[4] = {"attention_norm.weight", "ffn_norm.weight", "ada_rms_norm_t_cond.0.weight",
                               "ada_rms_norm_t_cond.2.weight"};
    const float **dv[4];
    for (int v = 0; v < 4; v++) {
        dv[v] = PTRS(DL);
        for (int l = 0; l < DL; l++) {
            snprintf(nm, sizeof nm, "layers.%d.%s", l, dec_vecs[v]);
            dv[v][l] = load_f32(&L, nm);
        }
    }
    w.dec_attn_norm = dv[0]; w.dec_ffn_norm = dv[1]; w.dec_ada_down = dv[2]; w.dec_ada_up = dv[3];
    w.dec_norm = load_f32(&L, "norm.weight");
#undef PTRS
    ctx->delay_tokens = 6;  /* default 480 ms (voxtral.c:136) */
    if (!L.bad) {
        ctx->model = vox_hip_model_create(c, &w, ctx->delay_tokens);
        ctx->owns_model = 1;
        if (!ctx->model) fail("vox_hip_model_create: %s", vox_hip_last_error());
    }
    arena_free(&a);
    st_close(&f);  /* every weight now lives in HBM */
    if (!ctx->model) {
        free(ctx);
        return NULL;
    }
    return ctx;
}

void vh_free(vh_ctx_t *ctx) {
    if (!ctx) return;
    if (ctx->owns_model) vox_hip_model_free(ctx->model);
    free(ctx);
}

int vh_set_delay(vh_ctx_t *ctx, int delay_ms) {
    if (delay_ms < 80) delay_ms = 80;
    if (delay_ms > 2400) delay_ms = 2400;
    ctx->delay_tokens = delay_ms / 80;
    return vox_hip_model_set_delay(ctx->model, ctx->delay_tokens);
}

/* ------------------------------------------------------------------------
 * Streaming (voxtral.c:827-851, 1013-1145, 1288-1316, 1640-1667)
 * ------------------------------------------------------------------------ */
/* live-mode limits (voxtral.c:410-420) */
#define STREAM_MAX_DECODE_KV 2000
#define STREAM_MAX_NON_TEXT_STREAK 64
#define STREAM_MAX_NO_DECODE_SAMPLES (16000 * 20)
#define STREAM_EMPTY_RESTARTS_FOR_FULL_RESET 2
#define TOKEN_EOS 2
#define TOKEN_TEXT_MIN 1000

struct vh_stream {
    vh_ctx_t *ctx;
    vh_sched_t *sched;          /* non-NULL: decoding is left to vh_sched_run */
    vox_hip_stream_t *st;
    vox_hip_mel_t *mel;
    int mel_cursor, conv_started, finished, min_new_mel;
    long long real_samples, last_decode_sample;
    int *queue;                 /* records of VH_MAX_ALT ids: chosen id, accepted alternatives, -1 */
    int q_head, q_tail, q_cap;
    int *dec_buf, *alt_buf;
    int generated, chunks, started_decoding;
    int continuous, n_alt;
    int pend_first, pend_n;     /* scheduled stream: a chunk waiting for vh_sched_run's batched encoder pass */
    float alt_cutoff;
    int nontext_streak, text_since_restart, empty_restarts, restarts, full_resets;
    double enc_ms, dec_ms, prefill_ms;
};

vh_stream_t *vh_stream_init(vh_ctx_t *ctx) {
    vh_stream_t *s = calloc(1, sizeof *s);
    s->ctx = ctx;
    s->st = vox_hip_stream_create(ctx->model);
    if (!s->st) {
        fail("vox_hip_stream_create: %s", vox_hip_last_error());
        free(s);
        return NULL;
    }
    /* 32 left-pad tokens of silence (voxtral.c:1255) */
    s->mel = vox_hip_mel_create(s->st, 32 * RAW_AUDIO_LENGTH_PER_TOK);
    if (!s->mel) {
        fail("vox_hip_mel_create: %s", vox_hip_last_error());
        vox_hip_stream_free(s->st);
        free(s);
        return NULL;
    }
    s->min_new_mel = (int)(STREAM_DEFAULT_INTERVAL * 100.0f);
    s->q_cap = 4096;
    s->queue = malloc(sizeof(int) * VH_MAX_ALT * s->q_cap);
    s->dec_buf = malloc(sizeof(int) * 4096);
    s->alt_buf = malloc(sizeof(int) * VH_MAX_ALT * 4096);
    s->n_alt = 1;
    return s;
}

void vh_stream_free(vh_stream_t *s) {
    if (!s) return;
    if (s->sched) vh_sched_detach(s->sched, s);
    vox_hip_mel_free(s->mel);
    vox_hip_stream_free(s->st);
    free(s->queue);
    free(s->dec_buf);
    free(s->alt_buf);
    free(s);
}

int vh_stream_reset(vh_stream_t *s) {
    if (!s) return -1;
    if (s->sched) return fail("vh_stream_reset: detach the stream from its scheduler first");
    if (vox_hip_stream_sync(s->st)) return fail("sync: %s", vox_hip_last_error());
    if (vox_hip_mel_reset(s->mel, 32 * RAW_AUDIO_LENGTH_PER_TOK) || vox_hip_stream_reset(s->st))
        return fail("reset: %s", vox_hip_last_error());
    /* everything vh_stream_init leaves zero goes back to zero; buffers and settings stay */
    s->mel_cursor = s->conv_started = s->finished = 0;
    s->real_samples = s->last_decode_sample = 0;
    s->q_head = s->q_tail = 0;
    s->generated = s->chunks = s->started_decoding = 0;
    s->pend_first = s->pend_n = 0;
    s->nontext_streak = s->text_since_restart = s->empty_restarts = s->restarts = s->full_resets = 0;
    s->enc_ms = s->dec_ms = s->prefill_ms = 0.0;
    return 0;
}

void vh_stream_set_continuous(vh_stream_t *s, int on) { s->continuous = on ? 1 : 0; }

int vh_stream_set_alt(vh_stream_t *s, int n_alt, float cutoff) {
    if (n_alt < 1) n_alt = 1;
    if (n_alt > VH_MAX_ALT) n_alt = VH_MAX_ALT;
    if (cutoff < 0) cutoff = 0;
    if (cutoff > 1) cutoff = 1;
    s->n_alt = n_alt;
    s->alt_cutoff = cutoff;
    return vox_hip_stream_set_alt(s->st, n_alt, cutoff);
}

int vh_token_class(int id) {
    /* stream_classify_token (voxtral.c:532-539) without the tokenizer: ids below
     * TOKEN_TEXT_MIN are control tokens; Tekken's id 1000 is the raw byte 0x00, the one text
     * id whose decode is an empty C string (INVALID); every other text id decodes to a
     * non-empty piece */
    if (id == TOKEN_EOS) return VH_TOK_EOS;
    if (id < TOKEN_TEXT_MIN) return VH_TOK_CONTROL;
    if (id == TOKEN_TEXT_MIN) return VH_TOK_INVALID;
    return VH_TOK_TEXT;
}

void vh_set_processing_interval(vh_stream_t *s, float seconds) {
    if (seconds <= 0) seconds = 0;
    s->min_new_mel = (int)(seconds * 100.0f);
    if (s->min_new_mel < 1) s->min_new_mel = 1;
}

/* stream_enqueue_token (voxtral.c:542-567): one record per generated id */
static void queue_push(vh_stream_t *s, const int *recs, int n) {
    for (int i = 0; i < n; i++) {
        const int next = (s->q_tail + 1) % s->q_cap;
        if (next == s->q_head) {  /* full: grow (keeps order) */
            int *nq = malloc(sizeof(int) * VH_MAX_ALT * s->q_cap * 2);
            int k = 0;
            for (int j = s->q_head; j != s->q_tail; j = (j + 1) % s->q_cap, k++)
                memcpy(nq + k * VH_MAX_ALT, s->queue + j * VH_MAX_ALT, sizeof(int) * VH_MAX_ALT);
            free(s->queue);
            s->queue = nq;
            s->q_head = 0;
            s->q_tail = k;
            s->q_cap *= 2;
        }
        memcpy(s->queue + s->q_tail * VH_MAX_ALT, recs + i * VH_MAX_ALT, sizeof(int) * VH_MAX_ALT);
        s->q_tail = (s->q_tail + 1) % s->q_cap;
    }
}

/* the chunk a scheduled stream deferred, encoded alone (before its own decode, before a
 * second chunk, on detach) */
static int flush_pending(vh_stream_t *s) {
    if (s->pend_n <= 0) return 0;
    const double t0 = now_ms();
    const float *p = vox_hip_mel_frame_ptr(s->mel, s->pend_first);
    if (!p || vox_hip_stream_encode_mel(s->st, p, s->pend_n, 1) < 0) return fail("encoder: %s", vox_hip_last_error());
    s->enc_ms += now_ms() - t0;
    s->pend_n = 0;
    s->chunks++;
    return vox_hip_mel_discard_before(s->mel, s->mel_cursor);
}

static int sched_batch_encode(void) {
    /* VOX_HIP_SCHED_BATCH_ENC=0: every scheduled chunk is encoded on its own */
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("VOX_HIP_SCHED_BATCH_ENC");
        v = (e && atoi(e) == 0) ? 0 : 1;
    }
    return v;
}

/* stream_run_encoder (voxtral.c:827-851) */
static int run_encoder(vh_stream_t *s) {
    int off = 0;
    const int frames = vox_hip_mel_frames(s->mel, &off);
    if (frames < 0) return fail("vox_hip_mel_frames failed");
    const int total = off + frames;
    if (s->mel_cursor < off) s->mel_cursor = off;
    const int new_mel = total - s->mel_cursor;
    const int need = s->conv_started ? s->min_new_mel : STREAM_FIRST_CHUNK_MIN_MEL;
    if (new_mel < need && !s->finished) return 0;
    if (new_mel <= 0) return 0;
    if (s->sched && sched_batch_encode()) {
        /* the chunk (same frame range as on the single-stream path) waits for vh_sched_run,
         * which encodes every attached stream's chunk in one batched pass */
        if (flush_pending(s)) return -1;
        s->pend_first = s->mel_cursor;
        s->pend_n = new_mel;
        s->conv_started = 1;
        s->mel_cursor = total;
        return 0;
    }
    /* a chunk deferred for a scheduler the stream has left goes first, in order */
    if (flush_pending(s)) return -1;
    const double t0 = now_ms();
    const float *p = vox_hip_mel_frame_ptr(s->mel, s->mel_cursor);
    /* a scheduled stream's chunk is only enqueued (vox_hip_stream_set_async_encode): the
     * other streams' chunks of this tick overlap it, vh_sched_run's steps wait for it */
    if (!p || vox_hip_stream_encode_mel(s->st, p, new_mel, 1) < 0 ||
        ((!s->sched || (getenv("VOX_HIP_SCHED_ASYNC") && atoi(getenv("VOX_HIP_SCHED_ASYNC")) == 0)) &&
         vox_hip_stream_sync(s->st)))
        return fail("encoder: %s", vox_hip_last_error());
    s->enc_ms += now_ms() - t0;
    s->conv_started = 1;
    s->mel_cursor = total;
    s->chunks++;
    return vox_hip_mel_discard_before(s->mel, s->mel_cursor);
}

/* stream_reset_full_state (voxtral.c:786-814): new mel context, conv stem, encoder and
 * decoder state */
static int reset_full(vh_stream_t *s) {
    vox_hip_mel_t *m = vox_hip_mel_create(s->st, 32 * RAW_AUDIO_LENGTH_PER_TOK);
    if (!m) return fail("vox_hip_mel_create: %s", vox_hip_last_error());
    vox_hip_mel_free(s->mel);
    s->mel = m;
    s->mel_cursor = 0;
    s->conv_started = 0;
    if (vox_hip_stream_reset(s->st)) return fail("reset: %s", vox_hip_last_error());
    return 0;
}

/* stream_enqueue_token for n ids just generated (s->dec_buf; their alternatives records
 * in s->alt_buf): token classes for the live-mode counters (voxtral.c:1116-1139), records
 * queued.  Sets *eos when the ids end with EOS. */
static void consume_tokens(vh_stream_t *s, int n, int *eos) {
    s->generated += n;
    s->last_decode_sample = s->real_samples;
    for (int i = 0; i < n; i++) {
        const int cls = vh_token_class(s->dec_buf[i]);
        if (cls == VH_TOK_TEXT) {
            s->text_since_restart = 1;
            s->empty_restarts = 0;
            s->nontext_streak = 0;
        } else if (cls != VH_TOK_EOS) {
            s->nontext_streak++;
            /* alternatives belong to text tokens only (stream_fill_alts is called for
             * STREAM_TOK_TEXT) */
            for (int a = 1; a < VH_MAX_ALT; a++) s->alt_buf[i * VH_MAX_ALT + a] = -1;
        } else {
            *eos = 1;
        }
    }
    queue_push(s, s->alt_buf, n);
}

/* alternatives records of the n ids in s->dec_buf (generated from step gen0 on) */
static int fill_alt_records(vh_stream_t *s, int gen0, int n) {
    if (s->n_alt > 1) {
        if (vox_hip_stream_read_alts(s->st, gen0, n, s->alt_buf, NULL))
            return fail("alternatives: %s", vox_hip_last_error());
        return 0;
    }
    for (int i = 0; i < n; i++) {
        s->alt_buf[i * VH_MAX_ALT] = s->dec_buf[i];
        for (int a = 1; a < VH_MAX_ALT; a++) s->alt_buf[i * VH_MAX_ALT + a] = -1;
    }
    return 0;
}

/* the live-mode restart checks after a decoder drain (voxtral.c:1189-1239) */
static int after_drain(vh_stream_t *s, int eos) {
    if (!s->continuous) return 0;
    int st6[6];
    vox_hip_stream_state(s->st, st6);
    const int started = st6[3];
    int need = 0;
    if (eos) need = 1;
    else if (started && st6[0] > STREAM_MAX_DECODE_KV) need = 2;
    else if (started && s->nontext_streak >= STREAM_MAX_NON_TEXT_STREAK) need = 3;
    else if (!s->finished && s->real_samples - s->last_decode_sample >= STREAM_MAX_NO_DECODE_SAMPLES) need = 4;
    if (!need) return 0;
    if (s->text_since_restart) s->empty_restarts = 0;
    else s->empty_restarts++;
    const int full = need >= 2 || s->empty_restarts >= STREAM_EMPTY_RESTARTS_FOR_FULL_RESET;
    s->restarts++;
    if (full) {
        s->full_resets++;
        if (reset_full(s) && vox_hip_stream_reset_decoder(s->st)) return fail("reset: %s", vox_hip_last_error());
        s->empty_restarts = 0;
    } else if (vox_hip_stream_reset_decoder(s->st)) {
        return fail("reset: %s", vox_hip_last_error());
    }
    /* stream_reset_decoder_state (voxtral.c:766-783) */
    s->started_decoding = 0;
    s->nontext_streak = 0;
    s->text_since_restart = 0;
    s->last_decode_sample = s->real_samples;
    return 0;
}

/* the prompt's adapter rows are there (or the decoder already runs) */
static int decoder_ready(vh_stream_t *s) {
    int st6[6];
    vox_hip_stream_state(s->st, st6);
    return st6[3] || vox_hip_stream_adapter_tokens(s->st) >= 1 + 32 + s->ctx->delay_tokens;
}

/* stream_run_decoder (voxtral.c:1013-1240): prefill once the prompt's adapter rows exist,
 * then every available row; greedy decoding stops after EOS (token 2).  In continuous
 * (live) mode the decoder restarts afterwards on EOS, KV > 2000, a 64-token non-text
 * streak or 20 s of audio without a decoded token, escalating to a full reset
 * (voxtral.c:1189-1239). */
static int run_decoder(vh_stream_t *s) {
    if (flush_pending(s)) return -1;
    if (!decoder_ready(s)) return 0;  /* waiting for the prompt */
    int eos = 0;
    for (;;) {
        const double t0 = now_ms();
        const int first = !s->started_decoding;
        int st6[6];
        vox_hip_stream_state(s->st, st6);
        const int gen0 = st6[5];
        /* the first call runs the prefill + first token alone, so its time is the
         * reference's prefill_ms */
        const int n = vox_hip_stream_decode(s->st, first ? 1 : 4096, 1, s->dec_buf, NULL);
        if (n < 0) return fail("decoder: %s", vox_hip_last_error());
        const double dt = now_ms() - t0;
        if (n == 0) break;
        if (first) {
            s->prefill_ms += dt;
            s->started_decoding = 1;
        }
        s->dec_ms += dt;
        if (fill_alt_records(s, gen0, n)) return -1;
        consume_tokens(s, n, &eos);
        if (eos) break;
    }
    return after_drain(s, eos);
}

int vh_stream_feed(vh_stream_t *s, const float *samples, int n) {
    if (!s || s->finished || n <= 0) return -1;
    if (vox_hip_mel_feed(s->mel, samples, n) < 0) return fail("mel: %s", vox_hip_last_error());
    s->real_samples += n;
    if (run_encoder(s) || (!s->sched && run_decoder(s))) return -1;
    return 0;
}

int vh_stream_flush(vh_stream_t *s) {
    if (!s || s->finished) return -1;
    /* the right padding vox_stream_flush feeds (voxtral.c:1645-1656) */
    const int align = (int)((RAW_AUDIO_LENGTH_PER_TOK - (s->real_samples % RAW_AUDIO_LENGTH_PER_TOK)) %
                            RAW_AUDIO_LENGTH_PER_TOK);
    const int pad = align + ((s->ctx->delay_tokens + 1) + OFFLINE_STREAMING_BUFFER_TOKENS) * RAW_AUDIO_LENGTH_PER_TOK;
    float *zeros = calloc((size_t)pad, sizeof(float));
    const int rc = vox_hip_mel_feed(s->mel, zeros, pad);
    free(zeros);
    if (rc < 0) return fail("mel: %s", vox_hip_last_error());
    const int saved = s->min_new_mel;
    s->min_new_mel = 1;
    /* a scheduled stream leaves the drain to vh_sched_run, except in live mode: there the
     * restart checks after this drain (voxtral.c:1189-1239) come before the final chunk of
     * vox_stream_finish, so the stream drains here on its own path */
    const int e = run_encoder(s) || ((!s->sched || s->continuous) && run_decoder(s));
    s->min_new_mel = saved;
    return e ? -1 : 0;
}

int vh_stream_finish(vh_stream_t *s) {
    if (!s || s->finished) return -1;
    if (vh_stream_flush(s)) return -1;
    s->finished = 1;
    if (vox_hip_mel_finish(s->mel, 0) < 0) return fail("mel: %s", vox_hip_last_error());
    if (run_encoder(s) || (!s->sched && run_decoder(s))) return -1;
    return 0;
}

int vh_stream_get(vh_stream_t *s, int *ids, int max) {
    int n = 0;
    while (n < max && s->q_head != s->q_tail) {
        ids[n++] = s->queue[s->q_head * VH_MAX_ALT];
        s->q_head = (s->q_head + 1) % s->q_cap;
    }
    return n;
}

int vh_stream_get_alt(vh_stream_t *s, int *recs, int max) {
    int n = 0;
    while (n < max && s->q_head != s->q_tail) {
        memcpy(recs + n * VH_MAX_ALT, s->queue + s->q_head * VH_MAX_ALT, sizeof(int) * VH_MAX_ALT);
        n++;
        s->q_head = (s->q_head + 1) % s->q_cap;
    }
    return n;
}

void vh_stream_stats(const vh_stream_t *s, vh_stats_t *o) {
    memset(o, 0, sizeof *o);
    o->mel_frames = s->mel_cursor;
    o->adapter_tokens = vox_hip_stream_adapter_tokens(s->st);
    o->generated = s->generated;
    o->chunks = s->chunks;
    o->encoder_ms = s->enc_ms;
    o->decoder_ms = s->dec_ms;
    o->prefill_ms = s->prefill_ms;
    o->restarts = s->restarts;
    o->full_resets = s->full_resets;
}

/* ------------------------------------------------------------------------
 * Per-GPU stream scheduler (the per-stream token loop of voxtral.c:
 * 1105-1145 turned into one batched step for every stream that has adapter rows)
 * ------------------------------------------------------------------------ */
#define VH_SCHED_STEPS 4096   /* tokens per stream and vox_hip_batch_decode call */

struct vh_sched {
    vh_ctx_t *ctx;
    int step_cap;             /* vh_sched_set_step_cap: steps per stream and run (<= 0: drain) */
    vox_hip_batch_t *batch;   /* made on the first batched step (fragment-major weight copies) */
    int cap, n;
    vh_stream_t *s[VH_SCHED_MAX];
    int *tok;                 /* [cap][VH_SCHED_STEPS] */
    vh_sched_stats_t stats;
};

vh_sched_t *vh_sched_create(vh_ctx_t *ctx, int max_streams) {
    if (!ctx || max_streams < 1 || max_streams > VH_SCHED_MAX) {
        fail("vh_sched_create: 1..%d streams", VH_SCHED_MAX);
        return NULL;
    }
    vh_sched_t *q = calloc(1, sizeof *q);
    q->ctx = ctx;
    q->cap = max_streams;
    q->tok = malloc(sizeof(int) * (size_t)max_streams * VH_SCHED_STEPS);
    return q;
}

void vh_sched_free(vh_sched_t *q) {
    if (!q) return;
    /* every attached stream leaves as vh_sched_detach does: its deferred chunk encoded, async
     * encoding off (errors are left in vh_last_error) */
    while (q->n > 0) {
        vh_stream_t *s = q->s[q->n - 1];
        if (vh_sched_detach(q, s)) {
            s->sched = NULL;
            q->n--;
        }
    }
    vox_hip_batch_free(q->batch);
    free(q->tok);
    free(q);
}

int vh_sched_attach(vh_sched_t *q, vh_stream_t *s) {
    if (!q || !s || s->ctx->model != q->ctx->model) return fail("vh_sched_attach: stream of another model");
    if (s->sched == q) return 0;
    if (s->sched) return fail("vh_sched_attach: stream already attached to a scheduler");
    if (q->n == q->cap) return fail("vh_sched_attach: scheduler full (%d streams)", q->cap);
    if (q->ctx->model != s->ctx->model) return fail("vh_sched_attach: stream of another model");
    /* VOX_HIP_SCHED_ASYNC=0: each encoder chunk synchronises (the round-2 behaviour) */
    const char *ae = getenv("VOX_HIP_SCHED_ASYNC");
    if (vox_hip_stream_set_async_encode(s->st, !(ae && atoi(ae) == 0)))
        return fail("async encode: %s", vox_hip_last_error());
    q->s[q->n++] = s;
    s->sched = q;
    return 0;
}

int vh_sched_detach(vh_sched_t *q, vh_stream_t *s) {
    for (int i = 0; i < q->n; i++)
        if (q->s[i] == s) {
            const int rc = flush_pending(s);
            q->s[i] = q->s[--q->n];
            s->sched = NULL;
            if (rc) return -1;
            return vox_hip_stream_set_async_encode(s->st, 0) ? fail("async encode: %s", vox_hip_last_error()) : 0;
        }
    return fail("vh_sched_detach: stream not attached");
}

void vh_sched_set_step_cap(vh_sched_t *q, int cap) { q->step_cap = cap > 0 ? cap : 0; }

int vh_stream_pending(vh_stream_t *s) {
    int st6[6];
    vox_hip_stream_state(s->st, st6);
    if (st6[4]) return 0;  /* EOS: nothing more is decoded (non-continuous) */
    const int rows = vox_hip_stream_adapter_tokens(s->st);
    int left;
    if (!st6[3]) left = rows >= 1 + 32 + s->ctx->delay_tokens ? rows - (32 + s->ctx->delay_tokens) : 0;
    else left = rows - st6[1] > 0 ? rows - st6[1] : 0;
    /* a chunk deferred for the scheduler's encoder pass has rows to come */
    return left + (s->pend_n > 0);
}

void vh_sched_stats(const vh_sched_t *q, vh_sched_stats_t *out) {
    *out = q->stats;
    long long b[6] = {0};
    if (q->batch && vox_hip_batch_stats(q->batch, b) == 0) {
        out->steps = b[1];
        out->captures = b[3];
        out->prefill_passes = b[4];
    }
}

static int sched_steps_first(void) {
    /* VOX_HIP_SCHED_STEPS_FIRST=0: the round-5 order (encoder pass enqueued before the steps) */
    const char *e = getenv("VOX_HIP_SCHED_STEPS_FIRST");
    return !(e && atoi(e) == 0);
}

static int sched_overlap(void) {
    /* VOX_HIP_SCHED_OVERLAP=0: the encoder pass completes before the batched steps start
     * (read per run, so one process can serve both ways) */
    const char *e = getenv("VOX_HIP_SCHED_OVERLAP");
    return !(e && atoi(e) == 0);
}

static int sched_tail_sync(void) {
    const char *e = getenv("VOX_HIP_SCHED_TAIL_SYNC");
    return e && atoi(e) == 1;
}

static int sched_encode(vh_sched_t *q, int overlap);

/* the batched steps of one run: every stream whose decoder can run (ran[i]) goes into one
 * vox_hip_batch_decode call per round, another round only when a stream hit the step cap;
 * bounded: stream i reads only its first rows[i] adapter rows (an encoder pass may still be
 * running on its queue).  enc_between: the run's encoder pass is enqueued between the first
 * round's begin and finish (vox_hip_batch_begin_rows / vox_hip_batch_finish), so the steps are
 * on the device before the pass; *enc_done tells whether that happened */
static int sched_steps(vh_sched_t *q, int bounded, const int *rows, const int *ran, int *eos, int *total,
                       int enc_between, int *enc_done) {
    for (int iter = 0;; iter++) {
        vox_hip_stream_t *hs[VH_SCHED_MAX];
        int idx[VH_SCHED_MAX], counts[VH_SCHED_MAX], gen0[VH_SCHED_MAX], brows[VH_SCHED_MAX], nb = 0;
        for (int i = 0; i < q->n; i++) {
            vh_stream_t *s = q->s[i];
            if (!ran[i] || eos[i]) continue;
            /* past a step cap only live-mode streams go on: their restart checks (step 4)
             * belong after a full drain, as in the reference */
            if (iter > 0 && q->step_cap > 0 && !s->continuous) continue;
            int st6[6];
            vox_hip_stream_state(s->st, st6);
            if (st6[4]) continue;
            if (st6[3] && rows[i] - st6[1] <= 0) continue;
            gen0[nb] = st6[5];
            brows[nb] = rows[i];
            hs[nb] = s->st;
            idx[nb++] = i;
        }
        if (!nb) break;
        if (!q->batch) {
            q->batch = vox_hip_batch_create(q->ctx->model, q->cap);
            if (!q->batch) return fail("batch: %s", vox_hip_last_error());
        }
        double t0 = now_ms();
        const int cap = q->step_cap > 0 && q->step_cap < VH_SCHED_STEPS ? q->step_cap : VH_SCHED_STEPS;
        int r;
        if (bounded && enc_between && iter == 0) {
            if (vox_hip_batch_begin_rows(q->batch, hs, nb, brows, cap, 1, q->tok, counts) < 0)
                return fail("batched decoder: %s", vox_hip_last_error());
            const double tb = now_ms();
            if (sched_encode(q, 1)) return -1;
            *enc_done = 1;
            t0 += now_ms() - tb;  /* the pass's enqueue is the encoder's time */
            r = vox_hip_batch_finish(q->batch);
        } else {
            r = bounded ? vox_hip_batch_decode_rows(q->batch, hs, nb, brows, cap, 1, q->tok, counts)
                        : vox_hip_batch_decode(q->batch, hs, nb, cap, 1, q->tok, counts);
        }
        if (r < 0) return fail("batched decoder: %s", vox_hip_last_error());
        const double dt = now_ms() - t0;
        q->stats.batch_calls++;
        q->stats.batch_ms += dt;
        int more = 0;
        for (int k = 0; k < nb; k++) {
            vh_stream_t *s = q->s[idx[k]];
            const int n = counts[k];
            s->dec_ms += dt;
            if (!n) continue;
            if (!s->started_decoding) {
                /* its prefill ran in this call (shared with the other new streams) */
                s->started_decoding = 1;
                s->prefill_ms += dt;
                q->stats.prefills++;
            }
            memcpy(s->dec_buf, q->tok + (size_t)k * cap, sizeof(int) * (size_t)n);
            if (fill_alt_records(s, gen0[k], n)) return -1;
            consume_tokens(s, n, &eos[idx[k]]);
            *total += n;
            more |= n == cap;
        }
        q->stats.tokens += r;
        /* with a step cap, a scheduled stream's rows beyond it wait for the next run */
        if (r == 0 || !more) break;
    }
    return 0;
}

int vh_sched_run(vh_sched_t *q) {
    const double t_run = now_ms();
    int total = 0;
    int eos[VH_SCHED_MAX] = {0}, ran[VH_SCHED_MAX] = {0};
    /* Overlap: the batched steps decode the adapter rows that exist when the run starts while
     * this run's encoder pass (on the streams' queues) computes the next ones.  The steps are
     * begun first and the pass is enqueued behind them, so the run's first steps are on the
     * device before the host spends ~1.4 ms on the pass's eager launches (served 16 streams
     * +3.4 %; the two queues' kernels still take turns on the device).  With a step cap set, the pass's rows
     * are decoded by the next run; with no cap (step_cap <= 0) this run waits for the pass and
     * drains them in a second round of steps.  Greedy ids do not depend on when a row is
     * decoded, so a stream's ids are unchanged.  Live-mode streams keep the sequential order:
     * their restart checks belong after a drain of every row of the chunk (voxtral.c:1189-1239). */
    int overlap = sched_overlap() && sched_batch_encode();
    for (int i = 0; i < q->n; i++) overlap = overlap && !q->s[i]->continuous;
    int rows[VH_SCHED_MAX] = {0};
    if (overlap)
        for (int i = 0; i < q->n; i++) {
            vh_stream_t *s = q->s[i];
            /* every row counted here is complete: nothing is left on the stream's queue */
            if (vox_hip_stream_sync(s->st)) return fail("sync: %s", vox_hip_last_error());
            rows[i] = vox_hip_stream_adapter_tokens(s->st);
            int st6[6];
            vox_hip_stream_state(s->st, st6);
            ran[i] = st6[3] || rows[i] >= 1 + 32 + s->ctx->delay_tokens;
        }
    /* 0. every attached stream's deferred chunk through one batched encoder pass (the layers'
     *    weights read once for all of them); with the overlap it is enqueued after the first
     *    batched steps (below), so those are on the device first */
    int enc_done = 0;
    if (!overlap || !sched_steps_first()) {
        if (sched_encode(q, overlap)) return -1;
        enc_done = 1;
    }
    /* 1-2. every stream whose decoder can run -- its prompt's adapter rows are there, or it
     *      already decodes and has rows left -- goes into the batched steps: the new ones'
     *      prefills share one stacked pass and they take their first token there, streams
     *      stop on the device when their rows run out or at EOS, streams with --alt keep their
     *      candidates (vox_hip_batch_decode); one call per round, another only when a stream
     *      hit the per-call step cap */
    if (!overlap)
        for (int i = 0; i < q->n; i++) {
            ran[i] = decoder_ready(q->s[i]);
            rows[i] = vox_hip_stream_adapter_tokens(q->s[i]->st);
        }
    if (sched_steps(q, overlap, rows, ran, eos, &total, !enc_done, &enc_done)) return -1;
    if (!enc_done && sched_encode(q, overlap)) return -1;  /* no steps ran this time */
    /* 3 (overlap). without a step cap the pass completes before the run returns (its rows are
     *    drained below); with one, the run returns while the pass may still be running: the
     *    caller's feeds and resets queue behind it on the streams' queues, and the next run
     *    syncs every stream before it counts rows (above), so the host work between runs
     *    overlaps the pass instead of leaving the device idle (VOX_HIP_SCHED_TAIL_SYNC=1: wait
     *    here as before round 6) */
    if (overlap) {
        if (q->step_cap <= 0 || sched_tail_sync())
            for (int i = 0; i < q->n; i++)
                if (vox_hip_stream_sync(q->s[i]->st)) return fail("encoder: %s", vox_hip_last_error());
        /* without a step cap a run drains every stream (vh_sched_set_step_cap): the rows this
         * run's pass produced are decoded now, after the pass, instead of by the next run */
        if (q->step_cap <= 0) {
            for (int i = 0; i < q->n; i++) {
                ran[i] = decoder_ready(q->s[i]);
                rows[i] = vox_hip_stream_adapter_tokens(q->s[i]->st);
            }
            if (sched_steps(q, 0, rows, ran, eos, &total, 0, &enc_done)) return -1;
        }
    }
    /* 4. per-stream live-mode restarts (voxtral.c:1189-1239) */
    for (int i = 0; i < q->n; i++)
        if (ran[i] == 1 && after_drain(q->s[i], eos[i])) return -1;
    q->stats.runs++;
    q->stats.run_ms += now_ms() - t_run;
    return total;
}

/* the run's encoder pass over every attached stream's deferred chunk (step 0 of vh_sched_run);
 * overlap: left running on the streams' queues (vh_sched_run syncs them before it returns) */
static int sched_encode(vh_sched_t *q, int overlap) {
    {
        vox_hip_stream_t *hs[VH_SCHED_MAX];
        const float *mp[VH_SCHED_MAX];
        int nf[VH_SCHED_MAX], added[VH_SCHED_MAX], idx[VH_SCHED_MAX], nb = 0;
        for (int i = 0; i < q->n; i++) {
            vh_stream_t *s = q->s[i];
            if (s->pend_n <= 0) continue;
            mp[nb] = vox_hip_mel_frame_ptr(s->mel, s->pend_first);
            if (!mp[nb]) return fail("vox_hip_mel_frame_ptr failed");
            hs[nb] = s->st;
            nf[nb] = s->pend_n;
            idx[nb++] = i;
        }
        if (nb) {
            const double t0 = now_ms();
            if (vox_hip_stream_encode_mel_batch(hs, mp, nf, nb, 1, added) < 0)
                return fail("batched encoder: %s", vox_hip_last_error());
            if (!overlap) {
                /* the pass completes here (the batched decode would wait for it anyway), so its
                 * time is the encoder's, not the decoder's */
                for (int k = 0; k < nb; k++)
                    if (vox_hip_stream_sync(hs[k])) return fail("encoder: %s", vox_hip_last_error());
                const double dt = now_ms() - t0;
                q->stats.enc_ms += dt;
                for (int k = 0; k < nb; k++) q->s[idx[k]]->enc_ms += dt / nb;
            } else {
                /* still running: it completes beside the steps (step 3); enc_ms counts the
                 * enqueue.  (Leaving it running past the run's end, for the next run to wait
                 * for, measured no faster: profiles/r4_serve_overlap_ab.txt.) */
                q->stats.enc_ms += now_ms() - t0;
            }
            q->stats.enc_batches++;
            for (int k = 0; k < nb; k++) {
                vh_stream_t *s = q->s[idx[k]];
                s->pend_n = 0;
                s->chunks++;
                /* safe with the pass in flight: discarding frees no device memory (a later grow
                 * of the mel buffer frees the old one through hipFree, which waits for the
                 * device) and the sample compaction is ordered on the stream's queue */
                if (vox_hip_mel_discard_before(s->mel, s->mel_cursor)) return -1;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * WAV (voxtral_audio.c:49-166): RIFF / WAVE, "fmt " 16-bit PCM, any channel count (mixed
 * down by the mean), any sample rate (linear interpolation to 16 kHz in the reference's f32
 * arithmetic); a "data" size of 0xFFFFFFFF (piped ffmpeg) or past the end means "to the end"
 * ------------------------------------------------------------------------ */
static float *parse_wav(const uint8_t *d, long size, int *n_samples, const char *path) {
    if (size < 44 || memcmp(d, "RIFF", 4) || memcmp(d + 8, "WAVE", 4)) {
        fail("%s: not a RIFF/WAVE file", path);
        return NULL;
    }
    int channels = 0, rate = 0, bits = 0, fmt = 0;
    const uint8_t *pcm = NULL;
    long pcm_size = 0;
    const uint8_t *p = d + 12, *end = d + size;
    while (p + 8 <= end) {
        uint32_t len;
        memcpy(&len, p + 4, 4);
        if (!memcmp(p, "fmt ", 4) && len >= 16 && (long)len <= end - p - 8) {
            fmt = p[8] | p[9] << 8;
            channels = p[10] | p[11] << 8;
            rate = p[12] | p[13] << 8 | p[14] << 16 | p[15] << 24;
            bits = p[22] | p[23] << 8;
        } else if (!memcmp(p, "data", 4)) {
            pcm = p + 8;
            pcm_size = (int32_t)len;
            if (pcm_size <= 0 || pcm_size > end - pcm) pcm_size = end - pcm;
            break;
        }
        if ((long)len > end - p - 8) break;
        p += 8 + (long)len + (len & 1);
    }
    if (fmt != 1 || bits != 16 || !pcm || channels < 1 || rate <= 0) {
        fail("%s: unsupported WAV (need 16-bit PCM; fmt %d, %d bit, %d ch, %d Hz)", path, fmt, bits, channels, rate);
        return NULL;
    }
    const int n = (int)(pcm_size / (channels * 2));
    float *x = malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        if (channels == 1) {
            int16_t v;
            memcpy(&v, pcm + 2 * (size_t)i, 2);
            x[i] = v / 32768.0f;
        } else {
            float sum = 0;
            for (int c = 0; c < channels; c++) {
                int16_t v;
                memcpy(&v, pcm + 2 * ((size_t)i * channels + c), 2);
                sum += v;
            }
            x[i] = (sum / channels) / 32768.0f;
        }
    }
    if (rate == 16000) {
        *n_samples = n;
        return x;
    }
    const int m = (int)((long long)n * 16000 / rate);
    float *y = malloc(sizeof(float) * (size_t)(m > 0 ? m : 1));
    for (int i = 0; i < m; i++) {
        const float pos = (float)i * rate / 16000;
        const int k = (int)pos;
        const float fr = pos - k;
        y[i] = k + 1 < n ? x[k] * (1.0f - fr) + x[k + 1] * fr : (k < n ? x[k] : 0.0f);
    }
    free(x);
    *n_samples = m;
    return y;
}

float *vh_load_wav(const char *path, int *n_samples) {
    FILE *fp = fopen(path, "rb");
    if (!fp) {
        fail("cannot open %s", path);
        return NULL;
    }
    fseek(fp, 0, SEEK_END);
    const long size = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    uint8_t *buf = malloc(size > 0 ? (size_t)size : 1);
    const size_t got = size > 0 ? fread(buf, 1, (size_t)size, fp) : 0;
    fclose(fp);
    float *out = NULL;
    if (size <= 0 || (long)got != size) fail("%s: short read", path);
    else out = parse_wav(buf, size, n_samples, path);
    free(buf);
    return out;
}
