// vox_hip.hip -- host side of the MI355X backend: implements include/voxtral_hip.h.
//
// Replaces voxtral_metal.m (SeungheonOh/voxtral.c) for the hot path.  Model weights are
// uploaded once into HBM and packed (Q|K|V merged, W1|W3 interleaved); each stream owns
// its rolling KV caches, conv-stem tails and adapter buffer in HBM; the decoder step is
// one hipGraph replay whose kernels read the step position from device memory, so a run
// of greedy steps never returns to the host (DESIGN.md "Decoder step").
#include "../../include/voxtral_hip.h"
#include "vox_hip_internal.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <stddef.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

using namespace vox;

#define TOKEN_BOS 1
#define TOKEN_EOS 2
#define TOKEN_STREAMING_PAD 32

static thread_local std::string g_err;
static int g_inited = 0;
static size_t g_mem_used = 0;

static int set_err(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    fprintf(stderr, "voxtral_hip: %s\n", buf);
    return -1;
}

#define CK(expr)                                                                          \
    do {                                                                                  \
        hipError_t e__ = (expr);                                                          \
        if (e__ != hipSuccess)                                                            \
            return set_err("%s failed at %s:%d: %s", #expr, __FILE__, __LINE__, hipGetErrorString(e__)); \
    } while (0)

template <class T>
static hipError_t dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e == hipSuccess) {
        g_mem_used += n * sizeof(T);
        // The streams are non-blocking, so nothing orders a null-stream memset before the
        // kernels a stream enqueues next: wait for the zeroing before handing the buffer out.
        e = hipMemsetAsync(*p, 0, n * sizeof(T), nullptr);
        if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    }
    return e;
}
// Host -> device copy that has landed when it returns (a pageable-source hipMemcpy may
// return once the data is staged, before the DMA that the stream kernels depend on).
static hipError_t h2d(void* dst, const void* src, size_t bytes) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, nullptr);
    return e == hipSuccess ? hipStreamSynchronize(nullptr) : e;
}
template <class T>
static void dfree(T*& p) {
    if (p) hipFree((void*)p);
    p = nullptr;
}

extern "C" const char* vox_hip_last_error(void) { return g_err.c_str(); }
extern "C" void vox_hip_clear_error(void) { g_err.clear(); }

extern "C" int vox_hip_init(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_err("no HIP device");
        return 0;
    }
    g_inited = 1;
    return 1;
}
extern "C" int vox_hip_available(void) { return g_inited; }
extern "C" void vox_hip_shutdown(void) { g_inited = 0; }
extern "C" size_t vox_hip_memory_used(void) { return g_mem_used; }
extern "C" int vox_hip_set_device(int device) {
    CK(hipSetDevice(device));
    return 0;
}

extern "C" void vox_hip_config_voxtral_4b(vox_hip_config_t* c) {
    // voxtral.h:26-50
    c->enc_dim = 1280; c->enc_layers = 32; c->enc_heads = 32; c->enc_kv_heads = 32;
    c->enc_head_dim = 64; c->enc_hidden = 5120; c->enc_window = 750;
    c->dec_dim = 3072; c->dec_layers = 26; c->dec_heads = 32; c->dec_kv_heads = 8;
    c->dec_head_dim = 128; c->dec_hidden = 9216; c->dec_window = 8192;
    c->vocab = 131072; c->mel_bins = 128; c->downsample = 4; c->ada_dim = 32;
    c->rope_theta = 1000000.0f; c->enc_eps = 1e-5f; c->dec_eps = 1e-5f; c->gelu_erf = 0;
}

// ---------------------------------------------------------------------------
// Host math that the reference runs on the CPU once per load (kept bit-identical)
// ---------------------------------------------------------------------------
static float host_gelu(float v, int erf_mode) {
    if (erf_mode) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    float x3 = v * v * v;
    float inner = 0.7978845608028654f * (v + 0.044715f * x3);
    return 0.5f * v * (1.0f + tanhf(inner));
}

// vox_compute_rope_freqs (voxtral_kernels.c:617-629) for positions [p0, p0+n)
static void host_rope(float* out, int p0, int n, int dim, float theta) {
    int half = dim / 2;
    for (int s = 0; s < n; s++) {
        float p = (float)(p0 + s);
        for (int d = 0; d < half; d++) {
            float freq = 1.0f / powf(theta, (float)(2 * d) / (float)dim);
            float ang = p * freq;
            out[(size_t)s * dim + 2 * d] = cosf(ang);
            out[(size_t)s * dim + 2 * d + 1] = sinf(ang);
        }
    }
}

// ---------------------------------------------------------------------------
// Model
// ---------------------------------------------------------------------------
// Weight matrices are raw bytes: bf16 [rows, K], or int8 [rows, K] when the matching
// scale array (Q8 per-row scales, quantize.py) is non-null.
struct EncLayerD {
    uint8_t *wqkv, *wo, *w13, *w2;
    float *sqkv, *so, *s13, *s2;
    float *bqkv, *bo, *b2, *attn_norm, *ffn_norm;
};
struct DecLayerD {
    uint8_t *wqkv, *wo, *w13, *w2;
    float *sqkv, *so, *s13, *s2;
    float *attn_norm, *ffn_norm;
};
// the same matrices in MFMA fragment order for the batched step (k_skf; built on first use)
struct DecFragD {
    uint8_t *wqkv, *wo, *w13, *w2;
};
static int frag_copy(uint8_t** dst, const uint8_t* src, int N, int K, int q8);
struct vox_hip_model;
static int model_frag(vox_hip_model* m);

struct vox_hip_model {
    vox_hip_config_t c;
    int delay_tokens;
    uint16_t *conv0_w, *conv1_w;
    float *conv0_b, *conv1_b, *enc_norm, *dec_norm;
    std::vector<EncLayerD> enc;
    std::vector<DecLayerD> dec;
    uint8_t *ad0, *ad1, *tok_emb;
    float *ad0_s, *ad1_s, *tok_emb_s;  // Q8 scales (null: bf16)
    float* ada_scale;              // device [dec_layers][dec_dim]
    std::vector<float> ada_host;   // host copy
    std::vector<std::vector<float>> ada_down, ada_up;
    float *rope_enc, *rope_dec;    // device tables [rope_positions][hd]
    int rope_positions;
    int rope_gen;                  // bumped when the tables are reallocated (graphs hold the pointer)
    std::vector<DecFragD> dfrag;   // fragment-major decoder matrices (empty until a batch or a bf16 prefill)
    std::vector<DecFragD> efrag;   // fragment-major encoder matrices (empty until a short chunk)
    uint8_t* lm_frag;              // fragment-major LM head (tied embeddings)
    int kv16;                      // decoder KV rings of streams created from now on in IEEE half
};

static int upload(void* dst, const void* src, size_t bytes) {
    if (!src) return set_err("null weight pointer");
    CK(h2d(dst, src, bytes));
    return 0;
}

// f32 tensor that holds bf16 values (the reference's load_f32 of a BF16 tensor) -> bf16
static int upload_f32_as_bf16(uint16_t* dst, const float* src, size_t n) {
    std::vector<uint16_t> tmp(n);
    for (size_t i = 0; i < n; i++) {
        uint32_t u;
        memcpy(&u, &src[i], 4);
        if (u & 0xffffu) return set_err("conv weight is not bf16-representable (element %zu)", i);
        tmp[i] = (uint16_t)(u >> 16);
    }
    return upload(dst, tmp.data(), n * 2);
}

// One device matrix (bf16, or int8 + per-row f32 scales) from a host pointer pair.
static int upload_mat(uint8_t** dst, float** dscale, const void* src, const float* scale, size_t rows,
                      size_t cols) {
    const size_t esz = scale ? 1 : 2;
    CK(dalloc(dst, rows * cols * esz));
    if (upload(*dst, src, rows * cols * esz)) return -1;
    *dscale = nullptr;
    if (scale) {
        CK(dalloc(dscale, rows));
        if (upload(*dscale, scale, rows * 4)) return -1;
    }
    return 0;
}

// merged Q|K|V rows (voxtral_metal.m merged_3 warmup); all three bf16 or all three Q8
static int upload_qkv(uint8_t** dst, float** dscale, const void* wq, const float* sq, const void* wk,
                      const float* sk, const void* wv, const float* sv, int nq, int nkv, int K) {
    if (!sq != !sk || !sq != !sv) return set_err("wq/wk/wv mix bf16 and Q8");
    const size_t esz = sq ? 1 : 2, rows = (size_t)nq + 2 * nkv;
    CK(dalloc(dst, rows * K * esz));
    if (upload(*dst, wq, (size_t)nq * K * esz) || upload(*dst + (size_t)nq * K * esz, wk, (size_t)nkv * K * esz) ||
        upload(*dst + (size_t)(nq + nkv) * K * esz, wv, (size_t)nkv * K * esz))
        return -1;
    *dscale = nullptr;
    if (sq) {
        CK(dalloc(dscale, rows));
        if (upload(*dscale, sq, (size_t)nq * 4) || upload(*dscale + nq, sk, (size_t)nkv * 4) ||
            upload(*dscale + nq + nkv, sv, (size_t)nkv * 4))
            return -1;
    }
    return 0;
}

// rows 32g..32g+15 <- w1 rows 16g..16g+15, rows 32g+16..32g+31 <- w3 rows 16g..
// (Q8: the row scales are interleaved the same way)
static int upload_w13(uint8_t** dst, float** dscale, const void* w1, const float* s1, const void* w3,
                      const float* s3, int hidden, int K) {
    if (!w1 || !w3) return set_err("null w1/w3");
    if (!s1 != !s3) return set_err("w1/w3 mix bf16 and Q8");
    if (hidden % 16) return set_err("hidden %d not a multiple of 16", hidden);
    const size_t esz = s1 ? 1 : 2;
    CK(dalloc(dst, (size_t)2 * hidden * K * esz));
    size_t grp = (size_t)16 * K * esz;
    CK(hipMemcpy2D(*dst, 2 * grp, w1, grp, grp, hidden / 16, hipMemcpyHostToDevice));
    CK(hipMemcpy2D(*dst + grp, 2 * grp, w3, grp, grp, hidden / 16, hipMemcpyHostToDevice));
    *dscale = nullptr;
    if (s1) {
        CK(dalloc(dscale, (size_t)2 * hidden));
        const size_t g4 = 16 * 4;
        CK(hipMemcpy2D(*dscale, 2 * g4, s1, g4, g4, hidden / 16, hipMemcpyHostToDevice));
        CK(hipMemcpy2D((char*)*dscale + g4, 2 * g4, s3, g4, g4, hidden / 16, hipMemcpyHostToDevice));
    }
    return 0;
}

static int model_update_ada(vox_hip_model_t* m) {
    // vox_update_time_conditioning (voxtral.c:31-80)
    const vox_hip_config_t& c = m->c;
    int D = c.dec_dim, A = c.ada_dim;
    std::vector<float> t_cond(D), hidden(A);
    int half = D / 2;
    float log_theta = logf(10000.0f);
    float t = (float)m->delay_tokens;
    for (int i = 0; i < half; i++) {
        float inv_freq = expf(-log_theta * (float)i / (float)half);
        float emb = t * inv_freq;
        t_cond[i] = cosf(emb);
        t_cond[i + half] = sinf(emb);
    }
    m->ada_host.assign((size_t)c.dec_layers * D, 0.f);
    for (int l = 0; l < c.dec_layers; l++) {
        const float* down = m->ada_down[l].data();
        const float* up = m->ada_up[l].data();
        for (int i = 0; i < A; i++) {
            float sum = 0.f;
            for (int j = 0; j < D; j++) sum += down[(size_t)i * D + j] * t_cond[j];
            hidden[i] = host_gelu(sum, c.gelu_erf);
        }
        float* sc = m->ada_host.data() + (size_t)l * D;
        for (int i = 0; i < D; i++) {
            float sum = 0.f;
            for (int j = 0; j < A; j++) sum += up[(size_t)i * A + j] * hidden[j];
            sc[i] = sum;
        }
    }
    CK(h2d(m->ada_scale, m->ada_host.data(), m->ada_host.size() * 4));
    return 0;
}

static int model_rope_tables(vox_hip_model_t* m, int positions) {
    const vox_hip_config_t& c = m->c;
    dfree(m->rope_enc);
    dfree(m->rope_dec);
    std::vector<float> t((size_t)positions * std::max(c.enc_head_dim, c.dec_head_dim));
    CK(dalloc(&m->rope_enc, (size_t)positions * c.enc_head_dim));
    host_rope(t.data(), 0, positions, c.enc_head_dim, c.rope_theta);
    CK(h2d(m->rope_enc, t.data(), (size_t)positions * c.enc_head_dim * 4));
    CK(dalloc(&m->rope_dec, (size_t)positions * c.dec_head_dim));
    host_rope(t.data(), 0, positions, c.dec_head_dim, c.rope_theta);
    CK(h2d(m->rope_dec, t.data(), (size_t)positions * c.dec_head_dim * 4));
    m->rope_positions = positions;
    m->rope_gen++;
    return 0;
}

static int check_config(const vox_hip_config_t* c) {
    if (c->enc_head_dim != 64 && c->enc_head_dim != 128) return set_err("enc_head_dim must be 64/128");
    if (c->dec_head_dim != 64 && c->dec_head_dim != 128) return set_err("dec_head_dim must be 64/128");
    if (c->enc_heads % c->enc_kv_heads || c->dec_heads % c->dec_kv_heads)
        return set_err("heads must be a multiple of kv heads");
    if (c->dec_heads / c->dec_kv_heads > 4 || c->enc_heads / c->enc_kv_heads > 4)
        return set_err("GQA ratio > 4 unsupported");
    int dims[] = {c->enc_dim, c->enc_hidden, c->dec_dim, c->dec_hidden,
                  c->enc_heads * c->enc_head_dim, c->dec_heads * c->dec_head_dim,
                  c->dec_kv_heads * c->dec_head_dim, c->mel_bins * 3};
    for (int d : dims)
        if (d % 64) return set_err("dimension %d not a multiple of 64", d);
    if (c->vocab % 2) return set_err("vocab must be even");
    if (c->downsample != 4) return set_err("downsample must be 4");
    return 0;
}

extern "C" void vox_hip_model_free(vox_hip_model_t* m);

extern "C" vox_hip_model_t* vox_hip_model_create(const vox_hip_config_t* cfg,
                                                 const vox_hip_weights_t* w, int delay_tokens) {
    if (!g_inited && !vox_hip_init()) return nullptr;
    if (check_config(cfg)) return nullptr;
    vox_hip_model_t* m = new vox_hip_model_t();
    memset(&m->c, 0, sizeof m->c);
    m->c = *cfg;
    m->delay_tokens = delay_tokens;
    {
        // the reference's VOX_DECODER_KV_FP16 (voxtral.c:189-190); opt-in here (unset = f32,
        // the CPU reference's cache), vox_hip_model_set_kv_fp16 overrides
        const char* e = getenv("VOX_DECODER_KV_FP16");
        m->kv16 = (e && atoi(e) != 0 && cfg->dec_head_dim == 128) ? 1 : 0;
    }
    m->conv0_w = m->conv1_w = nullptr;
    m->ad0 = m->ad1 = m->tok_emb = nullptr;
    m->ad0_s = m->ad1_s = m->tok_emb_s = nullptr;
    m->conv0_b = m->conv1_b = m->enc_norm = m->dec_norm = m->ada_scale = nullptr;
    m->rope_enc = m->rope_dec = nullptr;
    const vox_hip_config_t& c = *cfg;
    const int ED = c.enc_dim, EQ = c.enc_heads * c.enc_head_dim, EKV = c.enc_kv_heads * c.enc_head_dim;
    const int EH = c.enc_hidden;
    const int DD = c.dec_dim, DQ = c.dec_heads * c.dec_head_dim, DKV = c.dec_kv_heads * c.dec_head_dim;
    const int DH = c.dec_hidden;
    auto fail = [&]() -> vox_hip_model_t* { vox_hip_model_free(m); return nullptr; };
#define TRY(x) do { if ((x) != 0) return fail(); } while (0)
#define TRYH(x) do { hipError_t e__ = (x); if (e__ != hipSuccess) { set_err("%s: %s", #x, hipGetErrorString(e__)); return fail(); } } while (0)
#define SCL(field, l) (w->field ? w->field[l] : nullptr)
    // conv stem
    TRYH(dalloc(&m->conv0_w, (size_t)ED * c.mel_bins * 3));
    TRY(upload_f32_as_bf16(m->conv0_w, w->conv0_w, (size_t)ED * c.mel_bins * 3));
    TRYH(dalloc(&m->conv1_w, (size_t)ED * ED * 3));
    TRY(upload_f32_as_bf16(m->conv1_w, w->conv1_w, (size_t)ED * ED * 3));
    TRYH(dalloc(&m->conv0_b, ED));
    TRY(upload(m->conv0_b, w->conv0_b, ED * 4));
    TRYH(dalloc(&m->conv1_b, ED));
    TRY(upload(m->conv1_b, w->conv1_b, ED * 4));
    // encoder layers
    m->enc.resize(c.enc_layers);
    for (int l = 0; l < c.enc_layers; l++) {
        EncLayerD& L = m->enc[l];
        memset(&L, 0, sizeof L);
        TRY(upload_qkv(&L.wqkv, &L.sqkv, w->enc_wq[l], SCL(enc_wq_s, l), w->enc_wk[l], SCL(enc_wk_s, l),
                       w->enc_wv[l], SCL(enc_wv_s, l), EQ, EKV, ED));
        TRYH(dalloc(&L.bqkv, EQ + 2 * EKV));  // k part stays zero: wk has no bias
        TRY(upload(L.bqkv, w->enc_wq_b[l], EQ * 4));
        TRY(upload(L.bqkv + EQ + EKV, w->enc_wv_b[l], EKV * 4));
        TRY(upload_mat(&L.wo, &L.so, w->enc_wo[l], SCL(enc_wo_s, l), ED, EQ));
        TRYH(dalloc(&L.bo, ED));
        TRY(upload(L.bo, w->enc_wo_b[l], ED * 4));
        TRY(upload_w13(&L.w13, &L.s13, w->enc_w1[l], SCL(enc_w1_s, l), w->enc_w3[l], SCL(enc_w3_s, l), EH, ED));
        TRY(upload_mat(&L.w2, &L.s2, w->enc_w2[l], SCL(enc_w2_s, l), ED, EH));
        TRYH(dalloc(&L.b2, ED));
        TRY(upload(L.b2, w->enc_w2_b[l], ED * 4));
        TRYH(dalloc(&L.attn_norm, ED));
        TRY(upload(L.attn_norm, w->enc_attn_norm[l], ED * 4));
        TRYH(dalloc(&L.ffn_norm, ED));
        TRY(upload(L.ffn_norm, w->enc_ffn_norm[l], ED * 4));
    }
    TRYH(dalloc(&m->enc_norm, ED));
    TRY(upload(m->enc_norm, w->enc_norm, ED * 4));
    // adapter
    TRY(upload_mat(&m->ad0, &m->ad0_s, w->ad0, w->ad0_s, DD, (size_t)ED * c.downsample));
    TRY(upload_mat(&m->ad1, &m->ad1_s, w->ad1, w->ad1_s, DD, DD));
    // decoder
    TRY(upload_mat(&m->tok_emb, &m->tok_emb_s, w->tok_emb, w->tok_emb_s, c.vocab, DD));
    m->dec.resize(c.dec_layers);
    m->ada_down.resize(c.dec_layers);
    m->ada_up.resize(c.dec_layers);
    for (int l = 0; l < c.dec_layers; l++) {
        DecLayerD& L = m->dec[l];
        memset(&L, 0, sizeof L);
        TRY(upload_qkv(&L.wqkv, &L.sqkv, w->dec_wq[l], SCL(dec_wq_s, l), w->dec_wk[l], SCL(dec_wk_s, l),
                       w->dec_wv[l], SCL(dec_wv_s, l), DQ, DKV, DD));
        TRY(upload_mat(&L.wo, &L.so, w->dec_wo[l], SCL(dec_wo_s, l), DD, DQ));
        TRY(upload_w13(&L.w13, &L.s13, w->dec_w1[l], SCL(dec_w1_s, l), w->dec_w3[l], SCL(dec_w3_s, l), DH, DD));
        TRY(upload_mat(&L.w2, &L.s2, w->dec_w2[l], SCL(dec_w2_s, l), DD, DH));
        TRYH(dalloc(&L.attn_norm, DD));
        TRY(upload(L.attn_norm, w->dec_attn_norm[l], DD * 4));
        TRYH(dalloc(&L.ffn_norm, DD));
        TRY(upload(L.ffn_norm, w->dec_ffn_norm[l], DD * 4));
        if (!w->dec_ada_down[l] || !w->dec_ada_up[l]) { set_err("null ada weights"); return fail(); }
        m->ada_down[l].assign(w->dec_ada_down[l], w->dec_ada_down[l] + (size_t)c.ada_dim * DD);
        m->ada_up[l].assign(w->dec_ada_up[l], w->dec_ada_up[l] + (size_t)DD * c.ada_dim);
    }
    TRYH(dalloc(&m->dec_norm, DD));
    TRY(upload(m->dec_norm, w->dec_norm, DD * 4));
    TRYH(dalloc(&m->ada_scale, (size_t)c.dec_layers * DD));
    TRY(model_update_ada(m));
    TRY(model_rope_tables(m, 32768));
#undef TRY
#undef TRYH
#undef SCL
    return m;
}

extern "C" void vox_hip_model_free(vox_hip_model_t* m) {
    if (!m) return;
    dfree(m->conv0_w); dfree(m->conv1_w); dfree(m->conv0_b); dfree(m->conv1_b);
    for (auto& L : m->enc) {
        dfree(L.wqkv); dfree(L.wo); dfree(L.w13); dfree(L.w2);
        dfree(L.sqkv); dfree(L.so); dfree(L.s13); dfree(L.s2);
        dfree(L.bqkv); dfree(L.bo); dfree(L.b2); dfree(L.attn_norm); dfree(L.ffn_norm);
    }
    for (auto& L : m->dec) {
        dfree(L.wqkv); dfree(L.wo); dfree(L.w13); dfree(L.w2);
        dfree(L.sqkv); dfree(L.so); dfree(L.s13); dfree(L.s2);
        dfree(L.attn_norm); dfree(L.ffn_norm);
    }
    for (auto& F : m->dfrag) {
        dfree(F.wqkv); dfree(F.wo); dfree(F.w13); dfree(F.w2);
    }
    for (auto& F : m->efrag) {
        dfree(F.wqkv); dfree(F.wo); dfree(F.w13); dfree(F.w2);
    }
    dfree(m->lm_frag);
    dfree(m->enc_norm); dfree(m->ad0); dfree(m->ad1); dfree(m->tok_emb); dfree(m->dec_norm);
    dfree(m->ad0_s); dfree(m->ad1_s); dfree(m->tok_emb_s);
    dfree(m->ada_scale); dfree(m->rope_enc); dfree(m->rope_dec);
    delete m;
}

extern "C" int vox_hip_model_set_delay(vox_hip_model_t* m, int delay_tokens) {
    m->delay_tokens = delay_tokens;
    return model_update_ada(m);
}

extern "C" int vox_hip_set_gemm_planes(int planes) {
    if (set_gemm_planes(planes)) return set_err("gemm planes: 2 or 3 (got %d)", planes);
    return 0;
}

extern "C" int vox_hip_gemm_planes(void) { return gemm_planes_np(); }
extern "C" int vox_hip_set_gemmf_wait(int ticks) { return set_gemmf_wait(ticks); }

extern "C" int vox_hip_model_set_kv_fp16(vox_hip_model_t* m, int on) {
    if (on && m->c.dec_head_dim != 128) return set_err("16-bit decoder KV: head_dim 128 only (got %d)", m->c.dec_head_dim);
    m->kv16 = on ? 1 : 0;
    return 0;
}

extern "C" int vox_hip_stream_kv_fp16(const vox_hip_stream_t* s);

extern "C" int vox_hip_model_ada_scale(vox_hip_model_t* m, float* out) {
    memcpy(out, m->ada_host.data(), m->ada_host.size() * 4);
    return 0;
}

// ---------------------------------------------------------------------------
// Stream
// ---------------------------------------------------------------------------
static const int ENC_SUB = 1024;      // encoder rows per pass through the 32 layers
static const int DEC_SLACK = 64;      // decoder ring capacity = window + slack
static const int STEP_BATCH = 16;     // graph replays between EOS checks
static const size_t GEMM_WS_ELEMS = (size_t)8 << 20;  // split-K workspace (32 MB)
static const int TOKENS_CAP = 1 << 16;  // per-stream token / alternatives ring entries

struct vox_hip_stream {
    vox_hip_stream() { memset((void*)this, 0, offsetof(vox_hip_stream, pev)); }
    vox_hip_model_t* m;
    unsigned long long uid;  // unique per stream object ever created (batch graph keys)
    hipStream_t st;
    // rolling KV caches [layers][cap][kv_dim]
    float *ek, *ev, *dk, *dv;   // dk / dv: f32 elements, or IEEE half ones when kv16
    int ecap, dcap;
    int kv16;
    long long enc_pos;  // next encoder logical position
    // conv stem
    float *mel_p, *mel_tail, *c0_p, *c0_tail, *c0_res, *im2col;
    int res_count;
    int frames_cap;   // capacity (mel frames) of the conv buffers
    // encoder
    float *x_enc, *xn, *qkv, *q, *att, *gate, *enc_res;
    int x_rows_cap;
    int enc_res_count;
    float *rope_rows;  // per-call rope rows for the boundary twins
    int rope_rows_cap;
    // adapter
    float *adapter, *ad_mid;
    int adapter_cap, total_adapter;
    // decoder
    float *xd, *xnd, *qkvd, *qd_, *attd, *gated, *part, *logits, *pval;
    float *part_alt, *alts;  // stream_fill_alts partials / per-step records [tokens_cap][ALT_REC]
    float* gws;              // split-K GEMM partials (encoder / prefill / adapter)
    size_t gws_n;
    uint16_t* exp_;          // skinny encoder: row planes [4][3][16][max K] (fragment order)
    float* eslab;            // skinny encoder: split-K slabs [4][S][16][N]
    uint16_t* exp2;          // k_sklx: the second planes buffer (wo / w2 inputs)
    int* eticket;            // k_sklx slice tickets [SKX_TICKETS] (zeroed, self-resetting)
    int enc_async;           // vox_hip_stream_encode_mel returns without a stream sync
    float* xbatch;           // stacked encoder rows of a batched pass led by this stream
    float *cs_im, *cs_c0;    // its stacked conv-stem im2col rows / conv0 rows (enc_prefix_batch)
    float *abatch, *abatch_out;  // its stacked adapter input rows (4 x enc_dim) / adapter rows
    float* essq;             // k_sklx row sums of squares per column slice [2][slices][16]
    uint16_t *gpa, *gpc;     // k_gemmf planes: norm / attention rows (K <= max(enc_dim, heads x hd)), gate rows
    int* gflags;             // k_gemmf partial-tile flags + the recompute counter (gemmf_flag_ints())
    int gepoch;              // k_gemmf launch epoch on this stream
    uint16_t *dpa, *dpc;     // decoder prefill planes on k_gemmf: [rb][3][16][max(dim, heads x hd)], [rb][3][16][hidden]
    int dp_rows;             // rows they hold
    int n_alt;               // vox_stream_set_alt (voxtral.c:1329-1337); 1 = off
    float alt_cutoff;
    int graph_alt;           // alt mode the step graphs were captured with
    int graph_rope_gen;      // model rope table generation the step graphs were captured with
    int *pidx, *state, *tokens;   // tokens: ring of tokens_cap ids, index = step % tokens_cap
    int* twin_state;              // decoder_full_step's argmax state (the graph state stays untouched)
    int dec_rows_cap, tokens_cap;
    hipGraphExec_t step_exec[STEP_GRAPHS];  // [g]: attention with 2^g key splits (g = 0: no combine)
    int graph_ready;              // bit mask of built graphs
    int started, eos_seen, n_generated;
    int h_state[4];
    // profiling
    int profiling;
    int graph_prof;               // the last (eager, profiled) steps recorded W1|W3 events
    int capturing;
    hipEvent_t evt[2];
    hipEvent_t sev;               // cross-queue ordering (batched encoder pass), no timing
    std::vector<hipEvent_t> pev;  // [2*dec_layers] start/stop of each layer's W1|W3 GEMV
    double prof_ms, prof_bytes;
    long long prof_launches;
};

static int stream_alloc_frames(vox_hip_stream_t* s, int frames) {
    if (frames <= s->frames_cap) return 0;
    const vox_hip_config_t& c = s->m->c;
    int f = 256;
    while (f < frames) f *= 2;
    dfree(s->mel_p); dfree(s->c0_p); dfree(s->im2col); dfree(s->x_enc);
    CK(dalloc(&s->mel_p, (size_t)(f + 2) * c.mel_bins));
    CK(dalloc(&s->c0_p, (size_t)(f + 3) * c.enc_dim));
    size_t im = std::max((size_t)f * c.mel_bins * 3, (size_t)(f / 2 + 2) * c.enc_dim * 3);
    CK(dalloc(&s->im2col, im));
    CK(dalloc(&s->x_enc, (size_t)(f / 2 + 8) * c.enc_dim));
    s->frames_cap = f;
    return 0;
}

static int stream_alloc_adapter(vox_hip_stream_t* s, int need) {
    if (need <= s->adapter_cap) return 0;
    const int D = s->m->c.dec_dim;
    int nc = s->adapter_cap ? s->adapter_cap : 1024;
    while (nc < need) nc *= 2;
    float* na = nullptr;
    CK(dalloc(&na, (size_t)nc * D));
    if (s->adapter && s->total_adapter > 0)
        CK(hipMemcpyAsync(na, s->adapter, (size_t)s->total_adapter * D * 4, hipMemcpyDeviceToDevice, s->st));
    CK(hipStreamSynchronize(s->st));
    dfree(s->adapter);
    s->adapter = na;
    s->adapter_cap = nc;
    s->graph_ready = 0;  // the step graph captured the old pointer
    return 0;
}

static int stream_alloc_dec_rows(vox_hip_stream_t* s, int rows) {
    if (rows <= s->dec_rows_cap) return 0;
    const vox_hip_config_t& c = s->m->c;
    int r = 64;
    while (r < rows) r *= 2;
    const int DQ = c.dec_heads * c.dec_head_dim, DKV = c.dec_kv_heads * c.dec_head_dim;
    dfree(s->xd); dfree(s->xnd); dfree(s->qkvd); dfree(s->qd_); dfree(s->attd); dfree(s->gated);
    CK(dalloc(&s->xd, (size_t)r * c.dec_dim));
    CK(dalloc(&s->xnd, (size_t)r * c.dec_dim));
    CK(dalloc(&s->qkvd, (size_t)r * (DQ + 2 * DKV)));
    CK(dalloc(&s->qd_, (size_t)r * DQ));
    CK(dalloc(&s->attd, (size_t)r * DQ));
    CK(dalloc(&s->gated, (size_t)r * c.dec_hidden));
    s->dec_rows_cap = r;
    s->graph_ready = 0;
    return 0;
}

extern "C" void vox_hip_stream_free(vox_hip_stream_t* s);

extern "C" vox_hip_stream_t* vox_hip_stream_create(vox_hip_model_t* m) {
    static std::atomic<unsigned long long> next_uid{1};
    vox_hip_stream_t* s = new vox_hip_stream_t();
    s->m = m;
    s->uid = next_uid++;
    const vox_hip_config_t& c = m->c;
    auto fail = [&]() -> vox_hip_stream_t* { vox_hip_stream_free(s); return nullptr; };
#define TRYH(x) do { hipError_t e__ = (x); if (e__ != hipSuccess) { set_err("%s: %s", #x, hipGetErrorString(e__)); return fail(); } } while (0)
#define SCL(field, l) (w->field ? w->field[l] : nullptr)
    TRYH(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
    const int EKV = c.enc_kv_heads * c.enc_head_dim, DKV = c.dec_kv_heads * c.dec_head_dim;
    const int EQ = c.enc_heads * c.enc_head_dim;
    s->ecap = c.enc_window + ENC_SUB + 64;
    s->dcap = c.dec_window + DEC_SLACK;
    s->kv16 = m->kv16;
    TRYH(dalloc(&s->ek, (size_t)c.enc_layers * s->ecap * EKV));
    TRYH(dalloc(&s->ev, (size_t)c.enc_layers * s->ecap * EKV));
    // (dalloc counts floats: a half ring takes half of them; DKV is even)
    TRYH(dalloc(&s->dk, (size_t)c.dec_layers * s->dcap * DKV / (s->kv16 ? 2 : 1)));
    TRYH(dalloc(&s->dv, (size_t)c.dec_layers * s->dcap * DKV / (s->kv16 ? 2 : 1)));
    TRYH(dalloc(&s->mel_tail, (size_t)2 * c.mel_bins));
    TRYH(dalloc(&s->c0_tail, (size_t)2 * c.enc_dim));
    TRYH(dalloc(&s->c0_res, (size_t)c.enc_dim));
    TRYH(dalloc(&s->enc_res, (size_t)4 * c.enc_dim));
    TRYH(dalloc(&s->xn, (size_t)ENC_SUB * c.enc_dim));
    TRYH(dalloc(&s->qkv, (size_t)ENC_SUB * (EQ + 2 * EKV)));
    TRYH(dalloc(&s->q, (size_t)ENC_SUB * EQ));
    TRYH(dalloc(&s->att, (size_t)ENC_SUB * EQ));
    TRYH(dalloc(&s->gate, (size_t)ENC_SUB * c.enc_hidden));
    TRYH(dalloc(&s->ad_mid, (size_t)(ENC_SUB / 4 + 4) * c.dec_dim));
    // decode-attention partials + one arrival count per kv head after them (zeroed here,
    // reset by the merging block after every launch)
    TRYH(dalloc(&s->part, (size_t)c.dec_heads * attn_maxch(c.dec_window) * (c.dec_head_dim + 2) + c.dec_kv_heads));
    TRYH(dalloc(&s->part_alt, (size_t)GEMV_MAX_BLOCKS * ALT_PART));
    s->gws_n = GEMM_WS_ELEMS;
    TRYH(dalloc(&s->gws, s->gws_n));
    TRYH(dalloc(&s->logits, (size_t)c.vocab));
    TRYH(dalloc(&s->pval, GEMV_MAX_BLOCKS));
    TRYH(dalloc(&s->pidx, GEMV_MAX_BLOCKS));
    TRYH(dalloc(&s->state, 4));
    TRYH(dalloc(&s->twin_state, 4));
    s->tokens_cap = TOKENS_CAP;
    TRYH(dalloc(&s->tokens, s->tokens_cap));
    TRYH(dalloc(&s->alts, (size_t)s->tokens_cap * ALT_REC));
    s->n_alt = 1;
    s->alt_cutoff = 0.f;
    TRYH(hipEventCreate(&s->evt[0]));
    TRYH(hipEventCreate(&s->evt[1]));
    TRYH(hipEventCreateWithFlags(&s->sev, hipEventDisableTiming));
#undef TRYH
    if (stream_alloc_frames(s, 2048) || stream_alloc_adapter(s, 1024) || stream_alloc_dec_rows(s, 64))
        return fail();
    if (vox_hip_stream_reset(s)) return fail();
    return s;
}

// the batched steps' queue: the highest stream priority, so beside a cross-stream encoder pass
// (vox_hip_batch_decode_rows) the latency-bound step kernels go first
static hipError_t queue_high_priority(hipStream_t* q) {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) {
        (void)hipGetLastError();  // not left pending for the next launch check
        hi = 0;
    }
    // VOX_HIP_BATCH_PRIORITY=0: a normal-priority batch queue (A/B of the served overlap)
    const char* e = getenv("VOX_HIP_BATCH_PRIORITY");
    if (e && atoi(e) == 0) return hipStreamCreateWithFlags(q, hipStreamNonBlocking);
    return hipStreamCreateWithPriority(q, hipStreamNonBlocking, hi);
}

extern "C" int vox_hip_stream_kv_fp16(const vox_hip_stream_t* s) { return s->kv16; }

// layer l's decoder K or V ring (base = s->dk or s->dv) in the stream's element type
static float* dec_ring(const vox_hip_stream_t* s, float* base, int l) {
    const vox_hip_config_t& c = s->m->c;
    const size_t elems = (size_t)l * s->dcap * c.dec_kv_heads * c.dec_head_dim;
    return reinterpret_cast<float*>(reinterpret_cast<char*>(base) + elems * (s->kv16 ? 2 : 4));
}

extern "C" void vox_hip_stream_free(vox_hip_stream_t* s) {
    if (!s) return;
    if (s->st) hipStreamSynchronize(s->st);
    for (int g = 0; g < STEP_GRAPHS; g++)
        if (s->step_exec[g]) hipGraphExecDestroy(s->step_exec[g]);
    dfree(s->ek); dfree(s->ev); dfree(s->dk); dfree(s->dv);
    dfree(s->mel_p); dfree(s->mel_tail); dfree(s->c0_p); dfree(s->c0_tail); dfree(s->c0_res);
    dfree(s->im2col); dfree(s->x_enc); dfree(s->xn); dfree(s->qkv); dfree(s->q); dfree(s->att);
    dfree(s->gate); dfree(s->enc_res); dfree(s->rope_rows); dfree(s->adapter); dfree(s->ad_mid);
    dfree(s->xd); dfree(s->xnd); dfree(s->qkvd); dfree(s->qd_); dfree(s->attd); dfree(s->gated);
    dfree(s->part); dfree(s->logits); dfree(s->pval); dfree(s->pidx); dfree(s->state); dfree(s->twin_state); dfree(s->tokens);
    dfree(s->part_alt); dfree(s->alts); dfree(s->gws); dfree(s->exp_); dfree(s->eslab); dfree(s->eticket); dfree(s->essq); dfree(s->exp2); dfree(s->xbatch); dfree(s->abatch); dfree(s->abatch_out); dfree(s->cs_im); dfree(s->cs_c0);
    dfree(s->gpa); dfree(s->gpc); dfree(s->gflags); dfree(s->dpa); dfree(s->dpc);
    if (s->evt[0]) hipEventDestroy(s->evt[0]);
    if (s->evt[1]) hipEventDestroy(s->evt[1]);
    if (s->sev) hipEventDestroy(s->sev);
    for (hipEvent_t e : s->pev) hipEventDestroy(e);
    if (s->st) hipStreamDestroy(s->st);
    delete s;
}

extern "C" int vox_hip_stream_reset_decoder(vox_hip_stream_t* s) {
    // stream_reset_decoder_state (voxtral.c:766-783): KV length 0, adapter backlog dropped
    s->total_adapter = 0;
    s->started = 0;
    s->eos_seen = 0;
    s->n_generated = 0;
    int st[4] = {0, 0, TOKEN_BOS, 0};
    memcpy(s->h_state, st, sizeof st);
    CK(hipMemcpyAsync(s->state, st, sizeof st, hipMemcpyHostToDevice, s->st));
    CK(hipStreamSynchronize(s->st));
    return 0;
}

extern "C" int vox_hip_stream_reset(vox_hip_stream_t* s) {
    // stream_reset_full_state (voxtral.c:786-814)
    const vox_hip_config_t& c = s->m->c;
    s->enc_pos = 0;
    s->res_count = 0;
    s->enc_res_count = 0;
    CK(hipMemsetAsync(s->mel_tail, 0, (size_t)2 * c.mel_bins * 4, s->st));
    CK(hipMemsetAsync(s->c0_tail, 0, (size_t)2 * c.enc_dim * 4, s->st));
    return vox_hip_stream_reset_decoder(s);
}

extern "C" int vox_hip_stream_sync(vox_hip_stream_t* s) {
    CK(hipStreamSynchronize(s->st));
    return 0;
}

// ---------------------------------------------------------------------------
// Incremental log-mel on the device: the vox_mel_ctx_t of
// voxtral_audio.c:405-671 with its padded sample buffer and its frames in HBM.  The
// kernels run on the owning stream's queue, ahead of the encoder that reads the frames.
// ---------------------------------------------------------------------------
static const int MEL_FFT = 400, MEL_FREQ = 201, MEL_HOP = 160, MEL_BINS = 128, MEL_SR = 16000;
static const float MEL_LOG_MAX = 1.5f;                // LOG_MEL_MAX (voxtral_audio.c:25)
static const long long MEL_COMPACT_MIN = 16000;       // MEL_SAMPLE_COMPACT_MIN (:429)

struct vox_hip_mel {
    vox_hip_stream_t* s;
    float *window, *dcosT, *dsinT, *filtT;  // device tables (built on the host as the reference does)
    float* samples;                         // padded audio; samples[0] = global sample sample_offset
    long long n_samples, samples_cap, sample_offset;
    float* mel;                             // frames; mel[0] = global frame mel_phys0
    int mel_cap, mel_phys0;
    int frame_offset, n_frames;             // live frames: global [frame_offset, frame_offset + n_frames)
    int finished;
};

// hertz_to_mel / mel_to_hertz / build_mel_filters (voxtral_audio.c:223-285), f32 as there
static float mel_hz_to_mel(float f) {
    const float logstep = 27.0f / logf(6.4f);
    float m = 3.0f * f / 200.0f;
    if (f >= 1000.0f) m = 15.0f + logf(f / 1000.0f) * logstep;
    return m;
}
static float mel_mel_to_hz(float m) {
    const float logstep = logf(6.4f) / 27.0f;
    float f = 200.0f * m / 3.0f;
    if (m >= 15.0f) f = 1000.0f * expf(logstep * (m - 15.0f));
    return f;
}

extern "C" void vox_hip_mel_free(vox_hip_mel_t* m) {
    if (!m) return;
    if (m->s) hipStreamSynchronize(m->s->st);
    dfree(m->window); dfree(m->dcosT); dfree(m->dsinT); dfree(m->filtT); dfree(m->samples); dfree(m->mel);
    delete m;
}

extern "C" vox_hip_mel_t* vox_hip_mel_create(vox_hip_stream_t* s, int left_pad_samples) {
    if (!s || left_pad_samples < 0) {
        set_err("vox_hip_mel_create: bad arguments");
        return nullptr;
    }
    vox_hip_mel_t* m = new vox_hip_mel_t();
    memset((void*)m, 0, sizeof *m);
    m->s = s;
    auto fail = [&]() -> vox_hip_mel_t* { vox_hip_mel_free(m); return nullptr; };
    std::vector<float> win(MEL_FFT), dc((size_t)MEL_FFT * MEL_FREQ), ds((size_t)MEL_FFT * MEL_FREQ),
        ft((size_t)MEL_FREQ * MEL_BINS, 0.f);
    // DFT tables and periodic Hann window (voxtral_audio.c:531-545)
    for (int k = 0; k < MEL_FREQ; k++)
        for (int n = 0; n < MEL_FFT; n++) {
            const float ang = 2.0f * (float)M_PI * (float)k * (float)n / (float)MEL_FFT;
            dc[(size_t)n * MEL_FREQ + k] = cosf(ang);
            ds[(size_t)n * MEL_FREQ + k] = sinf(ang);
        }
    for (int i = 0; i < MEL_FFT; i++) win[i] = 0.5f * (1.0f - cosf(2.0f * (float)M_PI * (float)i / (float)MEL_FFT));
    // Slaney filters (voxtral_audio.c:248-285), stored [freq][bin]
    float fft_freqs[MEL_FREQ], ffq[MEL_BINS + 2], fdf[MEL_BINS + 1];
    for (int i = 0; i < MEL_FREQ; i++) fft_freqs[i] = (float)i * ((float)MEL_SR / 2.0f) / (float)(MEL_FREQ - 1);
    const float mmin = mel_hz_to_mel(0.0f), mmax = mel_hz_to_mel((float)MEL_SR / 2.0f);
    for (int i = 0; i < MEL_BINS + 2; i++) ffq[i] = mel_mel_to_hz(mmin + (mmax - mmin) * (float)i / (float)(MEL_BINS + 1));
    for (int i = 0; i < MEL_BINS + 1; i++) {
        fdf[i] = ffq[i + 1] - ffq[i];
        if (fdf[i] == 0.0f) fdf[i] = 1e-6f;
    }
    for (int b = 0; b < MEL_BINS; b++) {
        const float enorm = 2.0f / (ffq[b + 2] - ffq[b]);
        for (int f = 0; f < MEL_FREQ; f++) {
            const float down = (fft_freqs[f] - ffq[b]) / fdf[b];
            const float up = (ffq[b + 2] - fft_freqs[f]) / fdf[b + 1];
            float v = fminf(down, up);
            if (v < 0.0f) v = 0.0f;
            ft[(size_t)f * MEL_BINS + b] = v * enorm;
        }
    }
#define TRYH(x) do { hipError_t e__ = (x); if (e__ != hipSuccess) { set_err("%s: %s", #x, hipGetErrorString(e__)); return fail(); } } while (0)
    TRYH(dalloc(&m->window, win.size()));
    TRYH(dalloc(&m->dcosT, dc.size()));
    TRYH(dalloc(&m->dsinT, ds.size()));
    TRYH(dalloc(&m->filtT, ft.size()));
    TRYH(h2d(m->window, win.data(), win.size() * 4));
    TRYH(h2d(m->dcosT, dc.data(), dc.size() * 4));
    TRYH(h2d(m->dsinT, ds.data(), ds.size() * 4));
    TRYH(h2d(m->filtT, ft.data(), ft.size() * 4));
    // left padding: 200 (center reflect over silence) + left_pad_samples zeros (:547-557)
    m->n_samples = 200 + (long long)left_pad_samples;
    m->samples_cap = m->n_samples + 16000;
    TRYH(dalloc(&m->samples, (size_t)m->samples_cap));   // zeroed
    m->mel_cap = 1024;
    TRYH(dalloc(&m->mel, (size_t)m->mel_cap * MEL_BINS));
#undef TRYH
    return m;
}

static int mel_reserve_samples(vox_hip_mel_t* m, long long need) {
    if (need <= m->samples_cap) return 0;
    long long nc = m->samples_cap;
    while (nc < need) nc *= 2;
    float* nb = nullptr;
    CK(dalloc(&nb, (size_t)nc));
    CK(hipMemcpyAsync(nb, m->samples, (size_t)m->n_samples * 4, hipMemcpyDeviceToDevice, m->s->st));
    CK(hipStreamSynchronize(m->s->st));
    dfree(m->samples);
    m->samples = nb;
    m->samples_cap = nc;
    return 0;
}

// mel_compute_available (voxtral_audio.c:454-513): every frame whose window fits
static int mel_compute(vox_hip_mel_t* m) {
    const long long next = (long long)m->frame_offset + m->n_frames;  // global index of the next frame
    long long nf = 0;
    while ((next + nf) * MEL_HOP - m->sample_offset + MEL_FFT <= m->n_samples) nf++;
    if (nf == 0) return 0;
    const long long need = next + nf - m->mel_phys0;  // physical frames after this call
    if (need > m->mel_cap) {
        // grow, keeping only the live frames (discarded ones are dropped here)
        int nc = m->mel_cap;
        while (nc < need - (m->frame_offset - m->mel_phys0)) nc *= 2;
        float* nb = nullptr;
        CK(dalloc(&nb, (size_t)nc * MEL_BINS));
        if (m->n_frames)
            CK(hipMemcpyAsync(nb, m->mel + (size_t)(m->frame_offset - m->mel_phys0) * MEL_BINS,
                              (size_t)m->n_frames * MEL_BINS * 4, hipMemcpyDeviceToDevice, m->s->st));
        CK(hipStreamSynchronize(m->s->st));
        dfree(m->mel);
        m->mel = nb;
        m->mel_cap = nc;
        m->mel_phys0 = m->frame_offset;
    }
    CK(launch_mel_frames(m->samples, next * MEL_HOP - m->sample_offset, (int)nf, m->window, m->dcosT, m->dsinT,
                         m->filtT, MEL_LOG_MAX - 8.0f, m->mel + (size_t)(next - m->mel_phys0) * MEL_BINS, m->s->st));
    m->n_frames += (int)nf;
    return (int)nf;
}

// mel_compact_samples (voxtral_audio.c:432-451): samples no future frame reads are dropped
// once they reach 1 s (and never overlap the kept tail, so one device copy moves it)
static int mel_compact(vox_hip_mel_t* m) {
    const long long needed_from = ((long long)m->frame_offset + m->n_frames) * MEL_HOP;
    long long discard = needed_from - m->sample_offset;
    if (discard <= 0) return 0;
    if (discard > m->n_samples) discard = m->n_samples;
    const long long remain = m->n_samples - discard;
    if (discard < MEL_COMPACT_MIN || remain > discard) return 0;
    if (remain > 0)
        CK(hipMemcpyAsync(m->samples, m->samples + discard, (size_t)remain * 4, hipMemcpyDeviceToDevice, m->s->st));
    m->n_samples = remain;
    m->sample_offset += discard;
    return 0;
}

extern "C" int vox_hip_mel_reset(vox_hip_mel_t* m, int left_pad_samples) {
    if (!m || left_pad_samples < 0) return set_err("vox_hip_mel_reset: bad arguments");
    const long long n0 = 200 + (long long)left_pad_samples;
    if (mel_reserve_samples(m, n0)) return -1;
    CK(hipMemsetAsync(m->samples, 0, (size_t)n0 * 4, m->s->st));
    m->n_samples = n0;
    m->sample_offset = 0;
    m->mel_phys0 = 0;
    m->frame_offset = 0;
    m->n_frames = 0;
    m->finished = 0;
    return 0;
}

extern "C" int vox_hip_mel_feed(vox_hip_mel_t* m, const float* samples, int n) {
    if (!m || m->finished) return set_err("vox_hip_mel_feed: no context or already finished");
    if (n <= 0) return 0;
    if (mel_reserve_samples(m, m->n_samples + n)) return -1;
    CK(hipMemcpyAsync(m->samples + m->n_samples, samples, (size_t)n * 4, hipMemcpyHostToDevice, m->s->st));
    m->n_samples += n;
    const int nf = mel_compute(m);
    if (nf < 0 || mel_compact(m)) return -1;
    return nf;
}

extern "C" int vox_hip_mel_finish(vox_hip_mel_t* m, int right_pad) {
    if (!m) return set_err("vox_hip_mel_finish: no context");
    if (m->finished) return m->n_frames;
    if (right_pad < 0) right_pad = 0;
    if (mel_reserve_samples(m, m->n_samples + right_pad + 200)) return -1;
    if (right_pad > 0)
        CK(hipMemsetAsync(m->samples + m->n_samples, 0, (size_t)right_pad * 4, m->s->st));
    m->n_samples += right_pad;
    // right reflect over the last real samples (voxtral_audio.c:609-624)
    CK(launch_mel_reflect(m->samples, m->n_samples, m->n_samples - right_pad, 200, m->s->st));
    m->n_samples += 200;
    if (mel_compute(m) < 0) return -1;
    if (m->n_frames > 0) m->n_frames--;  // the last frame is dropped (:629-630)
    m->finished = 1;
    return m->n_frames;
}

extern "C" int vox_hip_mel_frames(const vox_hip_mel_t* m, int* frame_offset) {
    if (!m) return -1;
    if (frame_offset) *frame_offset = m->frame_offset;
    return m->n_frames;
}

extern "C" const float* vox_hip_mel_frame_ptr(const vox_hip_mel_t* m, int global_frame) {
    if (!m || global_frame < m->frame_offset || global_frame > m->frame_offset + m->n_frames) {
        set_err("vox_hip_mel_frame_ptr: frame %d outside the live range", global_frame);
        return nullptr;
    }
    return m->mel + (size_t)(global_frame - m->mel_phys0) * MEL_BINS;
}

// vox_mel_discard_before (voxtral_audio.c:645-662): frames before keep_from_frame leave the
// live range (their memory is reclaimed at the next growth)
extern "C" int vox_hip_mel_discard_before(vox_hip_mel_t* m, int keep_from_frame) {
    if (!m) return -1;
    if (keep_from_frame <= m->frame_offset) return 0;
    int d = keep_from_frame - m->frame_offset;
    if (d > m->n_frames) d = m->n_frames;
    m->frame_offset += d;
    m->n_frames -= d;
    return mel_compact(m);
}

extern "C" int vox_hip_mel_read(vox_hip_mel_t* m, int global_first, int n, float* out) {
    if (!m || n < 0 || global_first < m->frame_offset || global_first + n > m->frame_offset + m->n_frames)
        return set_err("vox_hip_mel_read: range outside the live frames");
    if (n == 0) return 0;
    CK(hipMemcpyAsync(out, m->mel + (size_t)(global_first - m->mel_phys0) * MEL_BINS, (size_t)n * MEL_BINS * 4,
                      hipMemcpyDeviceToHost, m->s->st));
    CK(hipStreamSynchronize(m->s->st));
    return 0;
}

// ---------------------------------------------------------------------------
// Encoder: 32 layers on rows [0, n) of x (logical positions pos0..), in place.
// voxtral_encoder.c:562-686.  rope: rows for these positions (table slice or per-call).
// ---------------------------------------------------------------------------
// Short encoder chunks (streaming -I: ~25 rows per 0.5 s) sit far below the MFMA ridge:
// their projections run as skinny GEMMs over fragment-major encoder weights (k_skl, the
// batched decoder's kernel: rows = up to 2 B fragments of 16, every weight byte streamed
// once per row block) with the consumers fused (residual + bias + RMSNorm into planes,
// SwiGLU into planes, bias into the QKV rows).  Longer chunks keep k_gemm2.
static const int ENC_SKINNY_MAX = SK_MAX_ROWS;  // buffers: up to SK_MAX_ROWS / 16 row blocks
static int enc_skinny_rows() {
    // chunks of up to this many rows take the skinny path (VOX_HIP_ENC_SKINNY_ROWS, <= 96).
    // 80: the ~70-row flush chunk of a one-shot clip too (jfk encoder RTF 0.00129 -> 0.00118:
    // five 16-row blocks re-reading each weight slice from the XCD's L2 beat a mostly empty
    // 128-row k_gemm2 tile)
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("VOX_HIP_ENC_SKINNY_ROWS");
        v = e ? std::max(0, std::min(ENC_SKINNY_MAX, atoi(e))) : 80;
    }
    return v;
}

static int model_enc_frag(vox_hip_model_t* m) {
    if (!m->efrag.empty()) return 0;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, EQ = c.enc_heads * c.enc_head_dim, EKV = c.enc_kv_heads * c.enc_head_dim;
    const int EH = c.enc_hidden;
    std::vector<DecFragD> F(c.enc_layers, DecFragD{});
    for (int l = 0; l < c.enc_layers; l++) {
        const EncLayerD& L = m->enc[l];
        if (frag_copy(&F[l].wqkv, L.wqkv, EQ + 2 * EKV, ED, L.sqkv != nullptr) ||
            frag_copy(&F[l].wo, L.wo, ED, EQ, L.so != nullptr) ||
            frag_copy(&F[l].w13, L.w13, 2 * EH, ED, L.s13 != nullptr) ||
            frag_copy(&F[l].w2, L.w2, ED, EH, L.s2 != nullptr)) {
            for (auto& f : F) { dfree(f.wqkv); dfree(f.wo); dfree(f.w13); dfree(f.w2); }
            return -1;
        }
    }
    m->efrag.swap(F);
    return 0;
}

static bool enc_skinny_ok(const vox_hip_config_t& c) {
    const int ED = c.enc_dim, EQ = c.enc_heads * c.enc_head_dim, EKV = c.enc_kv_heads * c.enc_head_dim;
    const int EH = c.enc_hidden;
    return skl_splits(ED) && skl_splits(EQ) && skl_splits(EH) && ED % 64 == 0 && (EQ + 2 * EKV) % 64 == 0 &&
           (2 * EH) % 64 == 0 && ED <= 8 * 512;
}

static int enc_fused_env() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("VOX_HIP_ENC_FUSED");
        v = (e && atoi(e) == 0) ? 0 : 1;
    }
    return v;
}

static int run_encoder_rows_skinny(vox_hip_stream_t* s, float* x, int n, long long pos0, const float* rope) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, H = c.enc_heads, KVH = c.enc_kv_heads, hd = c.enc_head_dim;
    const int EQ = H * hd, EKV = KVH * hd, EH = c.enc_hidden, NQKV = EQ + 2 * EKV;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t st = s->st;
    if (model_enc_frag(m)) return -1;
    if (!s->exp_) {
        const int kmax = std::max(ED, std::max(EQ, EH));
        const size_t slab = std::max(std::max((size_t)skl_splits(ED, NQKV) * NQKV, (size_t)skl_splits(EQ, ED) * ED),
                                     std::max((size_t)skl_splits(ED, 2 * EH) * 2 * EH, (size_t)skl_splits(EH, ED) * ED));
        const int RB = ENC_SKINNY_MAX / SK_ROWS;
        CK(dalloc(&s->exp_, (size_t)RB * 3 * SK_ROWS * kmax));
        CK(dalloc(&s->eslab, (size_t)RB * SK_ROWS * slab));
        CK(dalloc(&s->eticket, (size_t)SKX_TICKETS));
        CK(dalloc(&s->essq, (size_t)RB * SK_ROWS * (ED / 64)));
    }
    uint16_t* xp = s->exp_;
    float* sl = s->eslab;
    if (enc_fused_env() && !m->enc[0].sqkv) {
        // bf16: the row kernels folded into the projections (k_sklx): 5 launches per layer.
        // Planes alternate between two buffers so that no launch overwrites its own input:
        // xa = the QKV / W1|W3 inputs (x * norm weight), xq = the wo / w2 inputs.
        if (!s->exp2)
            CK(dalloc(&s->exp2, (size_t)(ENC_SKINNY_MAX / SK_ROWS) * 3 * SK_ROWS * std::max(ED, std::max(EQ, EH))));
        uint16_t *xa = xp, *xq = s->exp2;
        SklFused f;
        f.part = sl;
        f.ticket = s->eticket;
        f.eps = c.enc_eps;
        const int nsl_wo = sklx_slices(ED, EQ), nsl_w2 = sklx_slices(ED, EH);
        CK(launch_rmsnorm_fplanes(x, n, ED, m->enc[0].attn_norm, nullptr, c.enc_eps, xa, nullptr, 0, st));
        for (int l = 0; l < c.enc_layers; l++) {
            const EncLayerD& L = m->enc[l];
            const DecFragD& F = m->efrag[l];
            float* Kc = s->ek + (size_t)l * s->ecap * EKV;
            float* Vc = s->ev + (size_t)l * s->ecap * EKV;
            // QKV (attention RMSNorm: layer 0 normalised planes, then x * w planes scaled by
            // the inverse RMS), bias + RoPE + K/V append epilogue (encoder.c:562-607)
            SklFused q = f;
            q.ssq_in = s->essq;
            q.nsl = nsl_w2;
            q.bias = L.bqkv;
            q.rope = rope;
            q.qd = EQ;
            q.kvd = EKV;
            q.hd = hd;
            q.pos0 = (int)pos0;
            q.cap = s->ecap;
            q.q = s->q;
            q.Kc = Kc;
            q.Vc = Vc;
            CK(launch_gemm_sklx(l ? SKX_PRO_SCALE : SKX_PRO_PLANES, SKX_EPI_QKV, xa, ED, F.wqkv, NQKV, n, q, st));
            CK(launch_attn_rows_mf(hd, s->q, EQ, Kc, Vc, s->ecap, s->att, EQ, n, H, KVH, (int)pos0, 0, c.enc_window, scale,
                                 st, s->gws, s->gws_n, xq));
            // wo + bias residual (encoder.c:640-644); the FFN norm's planes and row sums of squares
            SklFused o = f;
            o.x = x;
            o.bias = L.bo;
            o.ssq_out = s->essq;
            o.planes = xa;
            o.nw = L.ffn_norm;
            CK(launch_gemm_sklx(SKX_PRO_PLANES, SKX_EPI_RESID, xq, EQ, F.wo, ED, n, o, st));
            // W1|W3 (FFN RMSNorm), SwiGLU epilogue into the w2 planes (encoder.c:646-676)
            SklFused u = f;
            u.ssq_in = s->essq;
            u.nsl = nsl_wo;
            u.planes = xq;
            CK(launch_gemm_sklx(SKX_PRO_SCALE, SKX_EPI_SWIGLU, xa, ED, F.w13, 2 * EH, n, u, st));
            // w2 + bias residual (encoder.c:678-684); the next layer's attention-norm planes
            SklFused d = f;
            d.x = x;
            d.bias = L.b2;
            d.ssq_out = s->essq;
            if (l + 1 < c.enc_layers) {
                d.planes = xa;
                d.nw = m->enc[l + 1].attn_norm;
            }
            CK(launch_gemm_sklx(SKX_PRO_PLANES, SKX_EPI_RESID, xq, EH, F.w2, ED, n, d, st));
        }
        CK(launch_rmsnorm_rows(x, ED, x, ED, m->enc_norm, nullptr, n, ED, c.enc_eps, st));
        return 0;
    }
    for (int l = 0; l < c.enc_layers; l++) {
        const EncLayerD& L = m->enc[l];
        const DecFragD& F = m->efrag[l];
        float* Kc = s->ek + (size_t)l * s->ecap * EKV;
        float* Vc = s->ev + (size_t)l * s->ecap * EKV;
        // previous layer's w2 residual (+ bias) then RMSNorm -> planes (encoder.c:562-566, 680-684)
        CK(launch_rmsnorm_fplanes(x, n, ED, L.attn_norm, nullptr, c.enc_eps, xp, l ? sl : nullptr,
                                  l ? skl_splits(EH, ED) : 0, st, l ? m->enc[l - 1].b2 : nullptr));
        CK(launch_gemm_skl(xp, ED, F.wqkv, L.sqkv, NQKV, n, sl, st));
        // QKV slabs + biases -> RoPE -> K/V append (one pass), attention with its output
        // merged straight into the wo planes
        CK(launch_slabs_rope_kv(sl, skl_splits(ED, NQKV), n, L.bqkv, EQ, EKV, hd, rope, (int)pos0, s->q, Kc, Vc, s->ecap, st));
        CK(launch_attn_rows_mf(hd, s->q, EQ, Kc, Vc, s->ecap, s->att, EQ, n, H, KVH, (int)pos0, 0, c.enc_window, scale, st,
                             s->gws, s->gws_n, xp));
        CK(launch_gemm_skl(xp, EQ, F.wo, L.so, ED, n, sl, st));
        // wo residual (+ bias) then the FFN RMSNorm -> planes (encoder.c:640-650)
        CK(launch_rmsnorm_fplanes(x, n, ED, L.ffn_norm, nullptr, c.enc_eps, xp, sl, skl_splits(EQ, ED), st, L.bo));
        CK(launch_gemm_skl(xp, ED, F.w13, L.s13, 2 * EH, n, sl, st));
        CK(launch_swiglu_fplanes(sl, skl_splits(ED, 2 * EH), EH, n, xp, st));
        CK(launch_gemm_skl(xp, EH, F.w2, L.s2, ED, n, sl, st));
    }
    CK(launch_resid_slabs(x, n, ED, sl, skl_splits(EH, ED), m->enc[c.enc_layers - 1].b2, st));
    CK(launch_rmsnorm_rows(x, ED, x, ED, m->enc_norm, nullptr, n, ED, c.enc_eps, st));
    return 0;
}

// Encoder passes of more rows (one-shot chunks: 677 rows for jfk, 1024-row passes of long
// clips): the projections on k_gemmf (stream-K MFMA over fragment-major weights), their
// inputs written as planes by the producers (RMSNorm rows, the attention output, the W1|W3
// SwiGLU epilogue), so no GEMM re-splits f32 activations per column tile.
static int enc_gemmf_env() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("VOX_HIP_GEMMF");
        v = (e && atoi(e) == 0) ? 0 : 1;
    }
    return v;
}

static bool enc_gemmf_ok(const vox_hip_model_t* m, int n) {
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, EQ = c.enc_heads * c.enc_head_dim, EKV = c.enc_kv_heads * c.enc_head_dim;
    return enc_gemmf_env() && !m->enc[0].sqkv && gemmf_ok(n, EQ + 2 * EKV, ED) && gemmf_ok(n, ED, EQ) &&
           gemmf_ok(n, 2 * c.enc_hidden, ED) && gemmf_ok(n, ED, c.enc_hidden) && c.enc_hidden % 64 == 0 &&
           ED <= 4 * 512;
}

// one k_gemmf launch on queue st with its split workspace, partial-tile flags and epoch
// counter (a queue's own: two k_gemmf launches in flight on two queues must not share flags)
struct GemmfQ {
    hipStream_t st;
    float* ws;
    size_t ws_n;
    int* flags;
    int* epoch;
};

static int gemmf_on(const GemmfQ& q, int epi, const uint16_t* xs, int K, int n, const uint8_t* W, int N,
                    const float* bias, float* C, int ldc, uint16_t* xo) {
    // the hand-off epoch is a host counter baked into the launch: a captured (replayed)
    // k_gemmf would reuse it and read stale partial tiles, so capture is refused
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    CK(hipStreamIsCapturing(q.st, &cs));
    if (cs != hipStreamCaptureStatusNone) return set_err("k_gemmf launch while the stream is capturing");
    if (++*q.epoch <= 0) *q.epoch = 1;
    // the launcher's shape / workspace checks, reported with the shape (launch_gemmf has one
    // error code for all of them), and an error an earlier unchecked call left pending (the
    // launcher's hipGetLastError would report it as this launch's)
    if (!gemmf_ok(n, N, K) || !q.ws || !q.flags)
        return set_err("k_gemmf: unsupported shape M %d N %d K %d (ws %p flags %p)", n, N, K, (void*)q.ws, (void*)q.flags);
    {
        const hipError_t pend = hipGetLastError();
        if (pend != hipSuccess) return set_err("k_gemmf: HIP error pending before the launch: %s", hipGetErrorString(pend));
    }
    CK(launch_gemmf(epi, gemm_planes_np(), xs, K, n, W, N, bias, C, ldc, xo, q.ws, q.ws_n, q.flags, *q.epoch, q.st));
    return 0;
}

static int gemmf(vox_hip_stream_t* s, int epi, const uint16_t* xs, int K, int n, const uint8_t* W, int N,
                 const float* bias, float* C, int ldc, uint16_t* xo) {
    return gemmf_on(GemmfQ{s->st, s->gws, s->gws_n, s->gflags, &s->gepoch}, epi, xs, K, n, W, N, bias, C, ldc,
                    xo);
}

static int run_encoder_rows_gemmf(vox_hip_stream_t* s, float* x, int n, long long pos0, const float* rope) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, H = c.enc_heads, KVH = c.enc_kv_heads, hd = c.enc_head_dim;
    const int EQ = H * hd, EKV = KVH * hd, EH = c.enc_hidden, NQKV = EQ + 2 * EKV;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t st = s->st;
    if (model_enc_frag(m)) return -1;
    if (!s->gpa) {
        const size_t rb = PLANE_MAX_ROWS / SK_ROWS;
        CK(dalloc(&s->gpa, rb * 3 * SK_ROWS * std::max(ED, EQ)));
        CK(dalloc(&s->gpc, rb * 3 * SK_ROWS * EH));
    }
    if (!s->gflags) CK(dalloc(&s->gflags, gemmf_flag_ints()));
    for (int l = 0; l < c.enc_layers; l++) {
        const EncLayerD& L = m->enc[l];
        const DecFragD& F = m->efrag[l];
        float* Kc = s->ek + (size_t)l * s->ecap * EKV;
        float* Vc = s->ev + (size_t)l * s->ecap * EKV;
        // RMSNorm -> planes, QKV (+ bias), RoPE + K/V append (encoder.c:562-607)
        CK(launch_rmsnorm_fplanes(x, n, ED, L.attn_norm, nullptr, c.enc_eps, s->gpa, nullptr, 0, st));
        if (gemmf(s, EPI_STORE, s->gpa, ED, n, F.wqkv, NQKV, L.bqkv, s->qkv, NQKV, nullptr)) return -1;
        CK(launch_rope_kv(s->qkv, n, EQ, EKV, hd, rope, (int)pos0, s->q, Kc, Vc, s->ecap, st));
        // windowed attention, output as the wo input planes (encoder.c:609-638)
        CK(launch_attn_rows_mf(hd, s->q, EQ, Kc, Vc, s->ecap, s->att, EQ, n, H, KVH, (int)pos0, 0, c.enc_window, scale, st,
                             s->gws, s->gws_n, s->gpa));
        // wo + bias residual (encoder.c:640-644)
        if (gemmf(s, EPI_RESID, s->gpa, EQ, n, F.wo, ED, L.bo, x, ED, nullptr)) return -1;
        // FFN RMSNorm -> planes, W1|W3 with SwiGLU into the w2 planes, w2 + bias residual (:646-684)
        CK(launch_rmsnorm_fplanes(x, n, ED, L.ffn_norm, nullptr, c.enc_eps, s->gpa, nullptr, 0, st));
        if (gemmf(s, EPI_SWIGLU, s->gpa, ED, n, F.w13, 2 * EH, nullptr, nullptr, EH, s->gpc)) return -1;
        if (gemmf(s, EPI_RESID, s->gpc, EH, n, F.w2, ED, L.b2, x, ED, nullptr)) return -1;
    }
    CK(launch_rmsnorm_rows(x, ED, x, ED, m->enc_norm, nullptr, n, ED, c.enc_eps, st));
    return 0;
}

// A single new encoder row (the 1-frame final chunk of a one-shot clip, a live stream's odd
// frame): the decode GEMVs -- every weight byte read once at the weight-streaming rate, with
// the RMSNorm prologues and the bias / RoPE + K/V append / SwiGLU / residual epilogues
// (encoder.c:562-684) -- and the M > 1 attention kernel for the one query row.  Five
// launches per layer instead of the skinny chain's row blocks of 16.
static bool enc_gemv_ok(const vox_hip_model_t* m) {
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, EQ = c.enc_heads * c.enc_head_dim, EKV = c.enc_kv_heads * c.enc_head_dim;
    const bool q8 = m->enc[0].sqkv != nullptr;
    return gemv_ok(EQ + 2 * EKV, ED, q8) && gemv_ok(ED, EQ, q8) && gemv_ok(2 * c.enc_hidden, ED, q8) &&
           gemv_ok(ED, c.enc_hidden, q8) && c.enc_head_dim % 2 == 0 && c.enc_hidden % 16 == 0;
}

static int run_encoder_row_gemv(vox_hip_stream_t* s, float* x, long long pos0, const float* rope) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, H = c.enc_heads, KVH = c.enc_kv_heads, hd = c.enc_head_dim;
    const int EQ = H * hd, EKV = KVH * hd, EH = c.enc_hidden;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t st = s->st;
    for (int l = 0; l < c.enc_layers; l++) {
        const EncLayerD& L = m->enc[l];
        float* Kc = s->ek + (size_t)l * s->ecap * EKV;
        float* Vc = s->ev + (size_t)l * s->ecap * EKV;
        GemvArgs a;
        // RMSNorm -> QKV + bias -> RoPE -> K/V append (encoder.c:562-607)
        memset(&a, 0, sizeof a);
        a.x = x; a.K = ED; a.W = L.wqkv; a.wscale = L.sqkv; a.rows = EQ + 2 * EKV; a.bias = L.bqkv;
        a.norm_w = L.attn_norm; a.eps = c.enc_eps; a.y = s->q;
        a.qd = EQ; a.kvd = EKV; a.hd = hd; a.pos = (int)pos0; a.rope = rope - (size_t)pos0 * hd;
        a.Kc = Kc; a.Vc = Vc; a.cap = s->ecap;
        CK(launch_gemv(PRO_NORM, EPI_QKV_BIAS, a, st));
        // windowed attention of the one query (encoder.c:609-638)
        CK(launch_attn_rows_mf(hd, s->q, EQ, Kc, Vc, s->ecap, s->att, EQ, 1, H, KVH, (int)pos0, 0, c.enc_window, scale,
                               st, s->gws, s->gws_n));
        // wo + bias residual (encoder.c:640-644)
        memset(&a, 0, sizeof a);
        a.x = s->att; a.K = EQ; a.W = L.wo; a.wscale = L.so; a.rows = ED; a.bias = L.bo; a.y = x;
        CK(launch_gemv(PRO_NONE, EPI_RESID, a, st));
        // RMSNorm -> W1|W3 -> silu * up (encoder.c:646-676)
        memset(&a, 0, sizeof a);
        a.x = x; a.K = ED; a.W = L.w13; a.wscale = L.s13; a.rows = 2 * EH; a.norm_w = L.ffn_norm; a.eps = c.enc_eps;
        a.y = s->gate;
        CK(launch_gemv(PRO_NORM, EPI_SWIGLU, a, st));
        // w2 + bias residual (encoder.c:678-684)
        memset(&a, 0, sizeof a);
        a.x = s->gate; a.K = EH; a.W = L.w2; a.wscale = L.s2; a.rows = ED; a.bias = L.b2; a.y = x;
        CK(launch_gemv(PRO_NONE, EPI_RESID, a, st));
    }
    CK(launch_rmsnorm_rows(x, ED, x, ED, m->enc_norm, nullptr, 1, ED, c.enc_eps, st));
    return 0;
}

static int enc_skinny_env() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("VOX_HIP_ENC_SKINNY");
        v = (e && atoi(e) == 0) ? 0 : 1;
    }
    return v;
}

static int run_encoder_rows(vox_hip_stream_t* s, float* x, int n, long long pos0, const float* rope) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, H = c.enc_heads, KVH = c.enc_kv_heads, hd = c.enc_head_dim;
    const int EQ = H * hd, EKV = KVH * hd, EH = c.enc_hidden;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t st = s->st;
    if (n > ENC_SUB) return set_err("encoder pass of %d rows > %d", n, ENC_SUB);
    if (n == 1 && enc_gemv_ok(m)) return run_encoder_row_gemv(s, x, pos0, rope);
    if (n <= enc_skinny_rows() && enc_skinny_env() && enc_skinny_ok(c)) return run_encoder_rows_skinny(s, x, n, pos0, rope);
    if (enc_gemmf_ok(m, n)) return run_encoder_rows_gemmf(s, x, n, pos0, rope);
    for (int l = 0; l < c.enc_layers; l++) {
        const EncLayerD& L = m->enc[l];
        float* Kc = s->ek + (size_t)l * s->ecap * EKV;
        float* Vc = s->ev + (size_t)l * s->ecap * EKV;
        CK(launch_rmsnorm_rows(x, ED, s->xn, ED, L.attn_norm, nullptr, n, ED, c.enc_eps, st));
        CK(launch_gemm(EPI_STORE, 3, s->xn, ED, L.wqkv, L.sqkv, ED, n, EQ + 2 * EKV, L.bqkv, s->qkv, EQ + 2 * EKV, st, s->gws, s->gws_n));
        CK(launch_rope_kv(s->qkv, n, EQ, EKV, hd, rope, (int)pos0, s->q, Kc, Vc, s->ecap, st));
        CK(launch_attn_rows_mf(hd, s->q, EQ, Kc, Vc, s->ecap, s->att, EQ, n, H, KVH, (int)pos0, 0, c.enc_window, scale, st,
                             s->gws, s->gws_n));
        CK(launch_gemm(EPI_RESID, 3, s->att, EQ, L.wo, L.so, EQ, n, ED, L.bo, x, ED, st, s->gws, s->gws_n));
        CK(launch_rmsnorm_rows(x, ED, s->xn, ED, L.ffn_norm, nullptr, n, ED, c.enc_eps, st));
        CK(launch_gemm(EPI_SWIGLU, 3, s->xn, ED, L.w13, L.s13, ED, n, 2 * EH, nullptr, s->gate, EH, st, s->gws, s->gws_n));
        CK(launch_gemm(EPI_RESID, 3, s->gate, EH, L.w2, L.s2, EH, n, ED, L.b2, x, ED, st, s->gws, s->gws_n));
    }
    CK(launch_rmsnorm_rows(x, ED, x, ED, m->enc_norm, nullptr, n, ED, c.enc_eps, st));
    return 0;
}

static int ensure_rope(vox_hip_stream_t* s, long long last_pos) {
    vox_hip_model_t* m = s->m;
    if (last_pos < m->rope_positions) return 0;
    int p = m->rope_positions;
    while (p <= last_pos) p *= 2;
    CK(hipDeviceSynchronize());
    if (model_rope_tables(m, p)) return -1;
    s->graph_ready = 0;
    return 0;
}

// stream_run_encoder in three phases, so a batch of streams can share the layer passes
// (vox_hip_stream_encode_mel_batch): (1) conv stem of n new mel frames on the stream's queue,
// *T1 encoder rows left at *xin (-1 error); (2) the 32 layers over those rows; (3) 4x
// downsample + adapter, returning the adapter rows added.
static int enc_prefix(vox_hip_stream_t* s, const float* mel, int n, int mel_on_device, int* T1o, float** xino) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int MB = c.mel_bins, ED = c.enc_dim;
    hipStream_t st = s->st;
    *T1o = 0;
    *xino = nullptr;
    if (n <= 0) return 0;
    if (stream_alloc_frames(s, n + 4)) return -1;
    // ---- conv0 over [mel_tail(2) | new n] (voxtral.c:594-651) ----
    CK(hipMemcpyAsync(s->mel_p, s->mel_tail, (size_t)2 * MB * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemcpyAsync(s->mel_p + (size_t)2 * MB, mel, (size_t)n * MB * 4,
                      mel_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    CK(launch_mel_tail(s->mel_p, n, MB, s->mel_tail, st));
    // c0_p rows: [c0_tail(2) | residual(res_count) | conv0 new (n)]
    CK(hipMemcpyAsync(s->c0_p, s->c0_tail, (size_t)2 * ED * 4, hipMemcpyDeviceToDevice, st));
    if (s->res_count)
        CK(hipMemcpyAsync(s->c0_p + (size_t)2 * ED, s->c0_res, (size_t)ED * 4, hipMemcpyDeviceToDevice, st));
    float* c0_new = s->c0_p + (size_t)(2 + s->res_count) * ED;
    CK(launch_im2col3(s->mel_p, MB, n, 1, 0, s->im2col, st));
    CK(launch_gemm(c.gelu_erf ? EPI_GELU_ERF : EPI_GELU, 3, s->im2col, MB * 3, m->conv0_w, nullptr, MB * 3, n, ED,
                   m->conv0_b, c0_new, ED, st, s->gws, s->gws_n));
    // ---- stride alignment (voxtral.c:653-692) ----
    const int total = s->res_count + n;
    const int new_res = total & 1;
    const int feed = total - new_res;
    if (new_res)
        CK(hipMemcpyAsync(s->c0_res, s->c0_p + (size_t)(2 + total - 1) * ED, (size_t)ED * 4,
                          hipMemcpyDeviceToDevice, st));
    s->res_count = new_res;
    if (feed <= 0) return 0;
    // ---- conv1 over [c0_tail(2) | feed], first output discarded (voxtral.c:694-756) ----
    const int T1 = feed / 2;
    float* xin = s->x_enc + (size_t)4 * ED;  // 4 spare rows in front for the downsample residual
    CK(launch_im2col3(s->c0_p, ED, T1, 2, 1, s->im2col, st));
    CK(launch_gemm(c.gelu_erf ? EPI_GELU_ERF : EPI_GELU, 3, s->im2col, ED * 3, m->conv1_w, nullptr, ED * 3, T1, ED,
                   m->conv1_b, xin, ED, st, s->gws, s->gws_n));
    CK(hipMemcpyAsync(s->c0_tail, s->c0_p + (size_t)(2 + feed - 2) * ED, (size_t)2 * ED * 4,
                      hipMemcpyDeviceToDevice, st));
    if (ensure_rope(s, s->enc_pos + T1 + 1)) return -1;
    *T1o = T1;
    *xino = xin;
    return 0;
}

// enc_prefix for several streams at once, on lead's queue, the two conv GEMMs run once over
// every stream's rows (the conv weights read once per pass; 2 launches instead of 2 per
// stream).  Stream b's conv0 rows form segment [c0_tail(2) | residual (res) | new (n)] of one
// stacked buffer, laid out as enc_prefix's c0_p: the GEMM also computes the tail / residual
// rows (from stale im2col rows; rows are independent) and the true ones are copied over them;
// conv1 writes stream b's T1[b] encoder rows straight to X at its stacked offset.  Per row the
// same products as enc_prefix (voxtral.c:594-756).  Returns the stacked rows N (-1 error).
static const int CS_ROWS = 2 * ENC_SUB + 5 * VOX_MAX_BATCH;  // conv0 rows of a batched pass
static bool enc_prefix_batch_fits(vox_hip_stream_t* const* ss, const int* n, int B) {
    long long r0 = 0, r1 = 0;
    for (int b = 0; b < B; b++)
        if (n[b] > 0) {
            r0 += 2 + ss[b]->res_count + n[b];
            r1 += (ss[b]->res_count + n[b]) / 2;
        }
    return r0 <= CS_ROWS && r1 <= ENC_SUB;
}

static int enc_prefix_batch(vox_hip_stream_t* lead, vox_hip_stream_t* const* ss, const float* const* mels,
                            const int* n, int B, int mel_on_device, float* X, int* T1, int* off) {
    vox_hip_model_t* m = lead->m;
    const vox_hip_config_t& c = m->c;
    const int MB = c.mel_bins, ED = c.enc_dim;
    hipStream_t st = lead->st;
    if (!lead->cs_im) {
        CK(dalloc(&lead->cs_im, std::max((size_t)CS_ROWS * MB * 3, (size_t)ENC_SUB * ED * 3)));
        CK(dalloc(&lead->cs_c0, (size_t)CS_ROWS * ED));
    }
    std::vector<int> seg(B, 0), res(B, 0), tot(B, 0);
    int R0 = 0, N = 0;
    for (int b = 0; b < B; b++) {
        T1[b] = 0;
        off[b] = N;
        if (n[b] <= 0) continue;
        vox_hip_stream_t* s = ss[b];
        if (stream_alloc_frames(s, n[b] + 4)) return -1;
        seg[b] = R0;
        res[b] = s->res_count;
        tot[b] = s->res_count + n[b];
        R0 += 2 + s->res_count + n[b];
        const int feed = tot[b] - (tot[b] & 1);
        T1[b] = feed > 0 ? feed / 2 : 0;
        N += T1[b];
    }
    // the members' queues (their mel frames) before the lead's
    for (int b = 0; b < B; b++)
        if (ss[b] != lead && n[b] > 0) {
            CK(hipEventRecord(ss[b]->sev, ss[b]->st));
            CK(hipStreamWaitEvent(st, ss[b]->sev, 0));
        }
    // ---- conv0 (voxtral.c:594-651) over every stream's [mel_tail(2) | new n] ----
    for (int b = 0; b < B; b++) {
        if (n[b] <= 0) continue;
        vox_hip_stream_t* s = ss[b];
        CK(hipMemcpyAsync(s->mel_p, s->mel_tail, (size_t)2 * MB * 4, hipMemcpyDeviceToDevice, st));
        CK(hipMemcpyAsync(s->mel_p + (size_t)2 * MB, mels[b], (size_t)n[b] * MB * 4,
                          mel_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
        CK(launch_mel_tail(s->mel_p, n[b], MB, s->mel_tail, st));
        CK(launch_im2col3(s->mel_p, MB, n[b], 1, 0, lead->cs_im + (size_t)(seg[b] + 2 + res[b]) * MB * 3, st));
    }
    CK(launch_gemm(c.gelu_erf ? EPI_GELU_ERF : EPI_GELU, 3, lead->cs_im, MB * 3, m->conv0_w, nullptr, MB * 3, R0, ED,
                   m->conv0_b, lead->cs_c0, ED, st, lead->gws, lead->gws_n));
    // the true tail / residual rows over the computed ones; the new residual row kept
    for (int b = 0; b < B; b++) {
        if (n[b] <= 0) continue;
        vox_hip_stream_t* s = ss[b];
        float* c0p = lead->cs_c0 + (size_t)seg[b] * ED;
        CK(hipMemcpyAsync(c0p, s->c0_tail, (size_t)2 * ED * 4, hipMemcpyDeviceToDevice, st));
        if (res[b]) CK(hipMemcpyAsync(c0p + (size_t)2 * ED, s->c0_res, (size_t)ED * 4, hipMemcpyDeviceToDevice, st));
        const int new_res = tot[b] & 1;
        if (new_res)
            CK(hipMemcpyAsync(s->c0_res, c0p + (size_t)(2 + tot[b] - 1) * ED, (size_t)ED * 4, hipMemcpyDeviceToDevice, st));
        s->res_count = new_res;
        // ---- conv1 im2col over [c0_tail(2) | feed], first output discarded (voxtral.c:694-756) ----
        if (T1[b] > 0) {
            const int feed = 2 * T1[b];
            CK(launch_im2col3(c0p, ED, T1[b], 2, 1, lead->cs_im + (size_t)off[b] * ED * 3, st));
            CK(hipMemcpyAsync(s->c0_tail, c0p + (size_t)feed * ED, (size_t)2 * ED * 4, hipMemcpyDeviceToDevice, st));
        }
    }
    if (N > 0)
        CK(launch_gemm(c.gelu_erf ? EPI_GELU_ERF : EPI_GELU, 3, lead->cs_im, ED * 3, m->conv1_w, nullptr, ED * 3, N, ED,
                       m->conv1_b, X, ED, st, lead->gws, lead->gws_n));
    for (int b = 0; b < B; b++)
        if (T1[b] > 0 && ensure_rope(ss[b], ss[b]->enc_pos + T1[b] + 1)) return -1;
    return N;
}

static int enc_suffix(vox_hip_stream_t* s, float* xin, int T1) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, D = c.dec_dim;
    hipStream_t st = s->st;
    s->enc_pos += T1;
    // ---- 4x downsample with residual + adapter (voxtral.c:868-934, encoder.c:699-737) ----
    const int R = s->enc_res_count;
    const int tot = R + T1;
    const int usable = (tot / 4) * 4;
    const int left = tot - usable;
    int added = 0;
    if (usable > 0) {
        if (R) CK(hipMemcpyAsync(xin - (size_t)R * ED, s->enc_res, (size_t)R * ED * 4, hipMemcpyDeviceToDevice, st));
        const float* ain = xin - (size_t)R * ED;
        const int n4 = usable / 4;
        if (stream_alloc_adapter(s, s->total_adapter + n4)) return -1;
        for (int r0 = 0; r0 < n4; r0 += ENC_SUB / 4) {
            int nr = std::min(ENC_SUB / 4, n4 - r0);
            CK(launch_gemm(c.gelu_erf ? EPI_GELU_ERF : EPI_GELU, 3, ain + (size_t)r0 * 4 * ED, 4 * ED, m->ad0, m->ad0_s,
                           4 * ED, nr, D, nullptr, s->ad_mid, D, st, s->gws, s->gws_n));
            CK(launch_gemm(EPI_STORE, 3, s->ad_mid, D, m->ad1, m->ad1_s, D, nr, D, nullptr,
                           s->adapter + (size_t)(s->total_adapter + r0) * D, D, st, s->gws, s->gws_n));
        }
        s->total_adapter += n4;
        added = n4;
        if (left)
            CK(hipMemcpyAsync(s->enc_res, ain + (size_t)usable * ED, (size_t)left * ED * 4, hipMemcpyDeviceToDevice, st));
    } else if (T1 > 0) {
        // fewer than 4 rows in total: keep all of them (old residual followed by new rows)
        CK(hipMemcpyAsync(s->enc_res + (size_t)R * ED, xin, (size_t)T1 * ED * 4, hipMemcpyDeviceToDevice, st));
    }
    s->enc_res_count = left;
    return added;
}

// enc_suffix for several streams at once, on lead's queue: stream b's new encoder rows are
// X[off[b] ..+ T1[b]); its 4-row groups (residual rows first) are stacked into one adapter
// input, the two adapter projections run once over all of them (the adapter weights read once
// per pass instead of once per stream), and each stream's rows are copied to its adapter
// buffer.  Per row the same products as enc_suffix (voxtral.c:868-934).
static int enc_suffix_batch(vox_hip_stream_t* lead, const float* X, vox_hip_stream_t* const* ss, const int* T1,
                            const int* off, int B, int* added) {
    vox_hip_model_t* m = lead->m;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, D = c.dec_dim;
    hipStream_t st = lead->st;
    const size_t ain_rows = (size_t)ENC_SUB + 4 * VOX_MAX_BATCH;  // encoder rows (+ residuals)
    if (!lead->abatch) {
        CK(dalloc(&lead->abatch, ain_rows * ED));
        CK(dalloc(&lead->abatch_out, ain_rows / 4 * D));
    }
    std::vector<int> aoff(B, 0), n4v(B, 0);
    int NA = 0;  // stacked adapter rows
    // the stacked rows are bounded before any copy is queued; every adapter buffer was sized
    // before the pass was enqueued (vox_hip_stream_encode_mel_batch), so nothing here waits on a queue
    for (int b = 0; b < B; b++)
        if (T1[b] > 0) {
            const int tot = ss[b]->enc_res_count + T1[b];
            if (ss[b]->total_adapter + tot / 4 > ss[b]->adapter_cap) return set_err("enc_suffix_batch: adapter buffer");
            NA += tot / 4;
        }
    if ((size_t)NA * 4 > ain_rows) return set_err("enc_suffix_batch: %d adapter rows", NA);
    NA = 0;
    for (int b = 0; b < B; b++) {
        added[b] = 0;
        if (T1[b] <= 0) continue;
        vox_hip_stream_t* s = ss[b];
        s->enc_pos += T1[b];
        const int R = s->enc_res_count, tot = R + T1[b], usable = (tot / 4) * 4, left = tot - usable;
        const float* xb = X + (size_t)off[b] * ED;
        if (usable > 0) {
            float* dst = lead->abatch + (size_t)NA * 4 * ED;
            if (R) CK(hipMemcpyAsync(dst, s->enc_res, (size_t)R * ED * 4, hipMemcpyDeviceToDevice, st));
            CK(hipMemcpyAsync(dst + (size_t)R * ED, xb, (size_t)(usable - R) * ED * 4, hipMemcpyDeviceToDevice, st));
            if (left)
                CK(hipMemcpyAsync(s->enc_res, xb + (size_t)(usable - R) * ED, (size_t)left * ED * 4,
                                  hipMemcpyDeviceToDevice, st));
            aoff[b] = NA;
            n4v[b] = usable / 4;
            NA += usable / 4;
        } else {
            CK(hipMemcpyAsync(s->enc_res + (size_t)R * ED, xb, (size_t)T1[b] * ED * 4, hipMemcpyDeviceToDevice, st));
        }
        s->enc_res_count = left;
    }
    for (int r0 = 0; r0 < NA; r0 += ENC_SUB / 4) {
        const int nr = std::min(ENC_SUB / 4, NA - r0);
        CK(launch_gemm(c.gelu_erf ? EPI_GELU_ERF : EPI_GELU, 3, lead->abatch + (size_t)r0 * 4 * ED, 4 * ED, m->ad0,
                       m->ad0_s, 4 * ED, nr, D, nullptr, lead->ad_mid, D, st, lead->gws, lead->gws_n));
        CK(launch_gemm(EPI_STORE, 3, lead->ad_mid, D, m->ad1, m->ad1_s, D, nr, D, nullptr,
                       lead->abatch_out + (size_t)r0 * D, D, st, lead->gws, lead->gws_n));
    }
    for (int b = 0; b < B; b++) {
        if (!n4v[b]) continue;
        vox_hip_stream_t* s = ss[b];
        CK(hipMemcpyAsync(s->adapter + (size_t)s->total_adapter * D, lead->abatch_out + (size_t)aoff[b] * D,
                          (size_t)n4v[b] * D * 4, hipMemcpyDeviceToDevice, st));
        s->total_adapter += n4v[b];
        added[b] = n4v[b];
    }
    return 0;
}

// The 32 encoder layers over the stacked new rows of several streams (row block b = rows
// [off[b], off[b] + nr[b]) of X belongs to ss[b], at its logical positions from pos0[b]):
// RMSNorm and the four projections run once over all rows (every weight byte read once for
// the batch), RoPE + K/V append and the windowed attention per stream against its own ring.
// Launched on lead->st with lead's scratch (ENC_SUB rows); the caller orders the streams.
static int run_encoder_rows_batch(vox_hip_stream_t* lead, float* X, int N, vox_hip_stream_t* const* ss,
                                  const int* off, const int* nr, const long long* pos0, int B) {
    vox_hip_model_t* m = lead->m;
    const vox_hip_config_t& c = m->c;
    const int ED = c.enc_dim, H = c.enc_heads, KVH = c.enc_kv_heads, hd = c.enc_head_dim;
    const int EQ = H * hd, EKV = KVH * hd, EH = c.enc_hidden, NQKV = EQ + 2 * EKV;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t st = lead->st;
    const bool gf = enc_gemmf_ok(m, N);
    if (gf) {
        if (model_enc_frag(m)) return -1;
        if (!lead->gpa) {
            const size_t rb = PLANE_MAX_ROWS / SK_ROWS;
            CK(dalloc(&lead->gpa, rb * 3 * SK_ROWS * std::max(ED, EQ)));
            CK(dalloc(&lead->gpc, rb * 3 * SK_ROWS * EH));
        }
        if (!lead->gflags) CK(dalloc(&lead->gflags, gemmf_flag_ints()));
    }
    for (int l = 0; l < c.enc_layers; l++) {
        const EncLayerD& L = m->enc[l];
        if (gf) {
            const DecFragD& F = m->efrag[l];
            CK(launch_rmsnorm_fplanes(X, N, ED, L.attn_norm, nullptr, c.enc_eps, lead->gpa, nullptr, 0, st));
            if (gemmf(lead, EPI_STORE, lead->gpa, ED, N, F.wqkv, NQKV, L.bqkv, lead->qkv, NQKV, nullptr)) return -1;
        } else {
            CK(launch_rmsnorm_rows(X, ED, lead->xn, ED, L.attn_norm, nullptr, N, ED, c.enc_eps, st));
            CK(launch_gemm(EPI_STORE, 3, lead->xn, ED, L.wqkv, L.sqkv, ED, N, NQKV, L.bqkv, lead->qkv, NQKV, st,
                           lead->gws, lead->gws_n));
        }
        // every stream's RoPE + K/V append and attention in one launch each (row offsets)
        EncRows er;
        memset(&er, 0, sizeof er);
        er.B = B;
        for (int b = 0; b < B; b++) {
            er.off[b] = off[b];
            er.nr[b] = nr[b];
            er.pos0[b] = (int)pos0[b];
            er.Kc[b] = ss[b]->ek + (size_t)l * ss[b]->ecap * EKV;
            er.Vc[b] = ss[b]->ev + (size_t)l * ss[b]->ecap * EKV;
        }
        CK(launch_rope_kv_rows(lead->qkv, N, EQ, EKV, hd, m->rope_enc, er, lead->q, lead->ecap, st));
        // (k_gemmf's wo reads planes: the attention writes them itself)
        CK(launch_attn_rows(hd, lead->q, er, N, lead->ecap, lead->att, H, KVH, c.enc_window, scale, lead->gws,
                            lead->gws_n, st, gf ? lead->gpa : nullptr));
        if (gf) {
            const DecFragD& F = m->efrag[l];
            if (gemmf(lead, EPI_RESID, lead->gpa, EQ, N, F.wo, ED, L.bo, X, ED, nullptr)) return -1;
            CK(launch_rmsnorm_fplanes(X, N, ED, L.ffn_norm, nullptr, c.enc_eps, lead->gpa, nullptr, 0, st));
            if (gemmf(lead, EPI_SWIGLU, lead->gpa, ED, N, F.w13, 2 * EH, nullptr, nullptr, EH, lead->gpc)) return -1;
            if (gemmf(lead, EPI_RESID, lead->gpc, EH, N, F.w2, ED, L.b2, X, ED, nullptr)) return -1;
        } else {
            CK(launch_gemm(EPI_RESID, 3, lead->att, EQ, L.wo, L.so, EQ, N, ED, L.bo, X, ED, st, lead->gws, lead->gws_n));
            CK(launch_rmsnorm_rows(X, ED, lead->xn, ED, L.ffn_norm, nullptr, N, ED, c.enc_eps, st));
            CK(launch_gemm(EPI_SWIGLU, 3, lead->xn, ED, L.w13, L.s13, ED, N, 2 * EH, nullptr, lead->gate, EH, st,
                           lead->gws, lead->gws_n));
            CK(launch_gemm(EPI_RESID, 3, lead->gate, EH, L.w2, L.s2, EH, N, ED, L.b2, X, ED, st, lead->gws, lead->gws_n));
        }
    }
    CK(launch_rmsnorm_rows(X, ED, X, ED, m->enc_norm, nullptr, N, ED, c.enc_eps, st));
    return 0;
}

// Several streams' new mel frames through one encoder pass (SURVEY 8f#1's batching applied
// to the encoder): each stream's conv stem on its own queue, then the stacked rows through the
// 32 layers once on ss[0]'s queue (weights read once for the batch), then each stream's
// downsample + adapter on its own queue; HIP events order the queues.  Falls back to one
// stream at a time when the stacked rows exceed one pass (ENC_SUB).  added[b] = adapter rows
// appended to stream b.  Synchronous unless every stream is in async-encode mode.
extern "C" int vox_hip_stream_encode_mel_batch(vox_hip_stream_t* const* ss, const float* const* mels, const int* n,
                                               int B, int mel_on_device, int* added) {
    if (B < 1 || !ss || !mels || !n || !added) return set_err("encode_mel_batch: bad arguments");
    if (B > VOX_MAX_BATCH) return set_err("encode_mel_batch: at most %d streams", VOX_MAX_BATCH);
    for (int b = 0; b < B; b++) {
        if (!ss[b] || ss[b]->m != ss[0]->m || ss[b]->ecap != ss[0]->ecap)
            return set_err("encode_mel_batch: streams of one model");
        for (int j = 0; j < b; j++)
            if (ss[j] == ss[b]) return set_err("encode_mel_batch: stream listed twice");
    }
    vox_hip_stream_t* lead = ss[0];
    const vox_hip_config_t& c = lead->m->c;
    const int ED = c.enc_dim;
    std::vector<int> T1(B), off(B);
    std::vector<float*> xin(B);
    std::vector<long long> pos0(B);
    int N = 0;
    bool all_async = true;
    // encoder rows each stream's frames complete (enc_prefix's stride alignment, on the host)
    int active = 0;
    for (int b = 0; b < B; b++) {
        all_async = all_async && ss[b]->enc_async;
        if (n[b] > 0) {
            const int tot = ss[b]->res_count + n[b];
            active += tot - (tot & 1) > 0;
        }
    }
    // several streams with rows: the conv stems stacked on the lead's queue (one GEMM per
    // conv for all of them, VOX_HIP_ENC_STEM_BATCH=0: one stream at a time), rows straight
    // into the stacked layer input
    static int stem_batch = -1;
    if (stem_batch < 0) {
        const char* e = getenv("VOX_HIP_ENC_STEM_BATCH");
        stem_batch = (e && atoi(e) == 0) ? 0 : 1;
    }
    const bool stacked = stem_batch && active > 1 && enc_prefix_batch_fits(ss, n, B);
    if (stacked) {
        if (!lead->xbatch) CK(dalloc(&lead->xbatch, (size_t)ENC_SUB * ED));
        N = enc_prefix_batch(lead, ss, mels, n, B, mel_on_device, lead->xbatch, T1.data(), off.data());
        if (N < 0) return -1;
        for (int b = 0; b < B; b++) pos0[b] = ss[b]->enc_pos;
    } else {
        for (int b = 0; b < B; b++) {
            if (enc_prefix(ss[b], mels[b], n[b], mel_on_device, &T1[b], &xin[b])) return -1;
            off[b] = N;
            pos0[b] = ss[b]->enc_pos;
            N += T1[b];
        }
    }
    if (!stacked && (N > ENC_SUB || active <= 1)) {
        // one stream at a time: rows beyond one pass, or a single stream with rows (its own
        // path keeps the skinny fused kernels for a short chunk)
        for (int b = 0; b < B; b++) {
            added[b] = 0;
            if (T1[b] <= 0) continue;
            for (int r0 = 0; r0 < T1[b]; r0 += ENC_SUB) {
                const int nrr = std::min(ENC_SUB, T1[b] - r0);
                const long long p0 = ss[b]->enc_pos + r0;
                if (run_encoder_rows(ss[b], xin[b] + (size_t)r0 * ED, nrr, p0, lead->m->rope_enc + (size_t)p0 * c.enc_head_dim))
                    return -1;
            }
            added[b] = enc_suffix(ss[b], xin[b], T1[b]);
            if (added[b] < 0) return -1;
        }
    } else {
        if (!stacked) {
            if (!lead->xbatch) CK(dalloc(&lead->xbatch, (size_t)ENC_SUB * ED));
            // the lead's queue waits for every member's conv stem (each stream's own reusable
            // event), stacks the rows, runs the layers
            for (int b = 1; b < B; b++) {
                CK(hipEventRecord(ss[b]->sev, ss[b]->st));
                CK(hipStreamWaitEvent(lead->st, ss[b]->sev, 0));
            }
            for (int b = 0; b < B; b++)
                if (T1[b] > 0)
                    CK(hipMemcpyAsync(lead->xbatch + (size_t)off[b] * ED, xin[b], (size_t)T1[b] * ED * 4,
                                      hipMemcpyDeviceToDevice, lead->st));
        }
        // adapter buffers sized now, before the pass is on the lead's queue: growing one later
        // (stream_alloc_adapter synchronises the stream's queue) would wait for the whole pass
        for (int b = 0; b < B; b++)
            if (T1[b] > 0 && stream_alloc_adapter(ss[b], ss[b]->total_adapter + (ss[b]->enc_res_count + T1[b]) / 4))
                return -1;
        if (run_encoder_rows_batch(lead, lead->xbatch, N, ss, off.data(), T1.data(), pos0.data(), B)) return -1;
        // downsample + adapter of every stream in one pass on the lead's queue; the members'
        // queues then wait for it
        if (enc_suffix_batch(lead, lead->xbatch, ss, T1.data(), off.data(), B, added)) return -1;
        CK(hipEventRecord(lead->sev, lead->st));
        for (int b = 1; b < B; b++) CK(hipStreamWaitEvent(ss[b]->st, lead->sev, 0));
    }
    if (!all_async)
        for (int b = 0; b < B; b++) CK(hipStreamSynchronize(ss[b]->st));
    return 0;
}

extern "C" int vox_hip_stream_encode_mel(vox_hip_stream_t* s, const float* mel, int n, int mel_on_device) {
    const vox_hip_config_t& c = s->m->c;
    int T1 = 0;
    float* xin = nullptr;
    if (enc_prefix(s, mel, n, mel_on_device, &T1, &xin)) return -1;
    int added = 0;
    if (T1 > 0) {
        // ---- encoder (voxtral_encoder.c:495-693), sub-chunks through all layers ----
        for (int r0 = 0; r0 < T1; r0 += ENC_SUB) {
            int nr = std::min(ENC_SUB, T1 - r0);
            long long p0 = s->enc_pos + r0;
            if (run_encoder_rows(s, xin + (size_t)r0 * c.enc_dim, nr, p0,
                                 s->m->rope_enc + (size_t)p0 * c.enc_head_dim))
                return -1;
        }
        added = enc_suffix(s, xin, T1);
        if (added < 0) return -1;
    }
    if (!s->enc_async) CK(hipStreamSynchronize(s->st));
    return added;
}

extern "C" int vox_hip_stream_set_async_encode(vox_hip_stream_t* s, int on) {
    if (!s) return set_err("null stream");
    if (s->enc_async && !on) CK(hipStreamSynchronize(s->st));
    s->enc_async = on ? 1 : 0;
    return 0;
}

extern "C" int vox_hip_stream_adapter_tokens(vox_hip_stream_t* s) { return s->total_adapter; }

extern "C" int vox_hip_stream_read_adapter(vox_hip_stream_t* s, int first, int n, float* out) {
    const int D = s->m->c.dec_dim;
    if (first < 0 || first + n > s->total_adapter) return set_err("adapter rows out of range");
    CK(hipMemcpyAsync(out, s->adapter + (size_t)first * D, (size_t)n * D * 4, hipMemcpyDeviceToHost, s->st));
    CK(hipStreamSynchronize(s->st));
    return 0;
}

// ---------------------------------------------------------------------------
// Decoder
// ---------------------------------------------------------------------------
// device state after the prompt's prefill rows 0..np-1: the next step reads row np with the
// streaming pad token (voxtral.c:1036-1061)
static int stream_prefilled(vox_hip_stream_t* s, hipStream_t q) {
    const int np = 32 + s->m->delay_tokens;
    const int st4[4] = {np, np, TOKEN_STREAMING_PAD, s->n_generated};
    CK(hipMemcpyAsync(s->state, st4, sizeof st4, hipMemcpyHostToDevice, q));
    s->h_state[0] = np;
    s->h_state[1] = np;
    s->h_state[2] = TOKEN_STREAMING_PAD;
    s->h_state[3] = s->n_generated;
    s->started = 1;
    return 0;
}

// Decoder prefill rows on k_gemmf (bf16 weights): the projections read the fragment-major
// decoder copies of the batched path (model_frag) once per 64-row tile -- the 38-row prompt is
// one tile, where k_gemm2's 128 x 128 tiles were mostly padding and split K eight ways --, with
// the inputs written as planes by their producers (RMSNorm rows, the attention output, the
// W1|W3 SwiGLU epilogue), as the encoder's long passes do.
static int dec_gemmf_env() {
    // VOX_HIP_PREFILL_GEMMF=0: decoder prefills on k_gemm2 over the row-major weights (A/B, and
    // no fragment-major copies for a process that never batches)
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("VOX_HIP_PREFILL_GEMMF");
        v = (e && atoi(e) == 0) ? 0 : 1;
    }
    return v;
}

static bool dec_gemmf_ok(const vox_hip_model_t* m, int n) {
    const vox_hip_config_t& c = m->c;
    const int DD = c.dec_dim, DQ = c.dec_heads * c.dec_head_dim, DKV = c.dec_kv_heads * c.dec_head_dim;
    return enc_gemmf_env() && dec_gemmf_env() && !m->dec[0].sqkv && n >= 1 && n <= PLANE_MAX_ROWS && gemmf_ok(n, DQ + 2 * DKV, DD) &&
           gemmf_ok(n, DD, DQ) && gemmf_ok(n, 2 * c.dec_hidden, DD) && gemmf_ok(n, DD, c.dec_hidden) &&
           c.dec_hidden % 64 == 0;
}

static int stream_dec_planes(vox_hip_stream_t* s, int rows) {
    if (rows <= s->dp_rows) return 0;
    const vox_hip_config_t& c = s->m->c;
    const int DD = c.dec_dim, DQ = c.dec_heads * c.dec_head_dim;
    // whole 128-row tiles: k_gemmf reads every row block of a tile (rows past n are computed
    // and dropped)
    const int r = (rows + 127) / 128 * 128;
    dfree(s->dpa);
    dfree(s->dpc);
    s->dp_rows = 0;
    CK(dalloc(&s->dpa, (size_t)r * 3 * std::max(DD, DQ)));
    CK(dalloc(&s->dpc, (size_t)r * 3 * c.dec_hidden));
    if (!s->gflags) CK(dalloc(&s->gflags, gemmf_flag_ints()));
    s->dp_rows = r;
    return 0;
}

// the prefill layers of rows x[0..n) with planes / scratch of s on queue q; attn(l) runs the
// layer's RoPE + K/V append + attention into s->attd
template <class Attn>
static int dec_layers_gemmf(vox_hip_stream_t* s, const GemmfQ& q, float* x, int n, Attn attn) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int DD = c.dec_dim, DQ = c.dec_heads * c.dec_head_dim, DKV = c.dec_kv_heads * c.dec_head_dim;
    const int DH = c.dec_hidden;
    if (model_frag(m) || stream_dec_planes(s, n)) return -1;
    for (int l = 0; l < c.dec_layers; l++) {
        const DecLayerD& L = m->dec[l];
        const DecFragD& F = m->dfrag[l];
        // RMSNorm -> planes, QKV (decoder.c:509-530)
        CK(launch_rmsnorm_fplanes(x, n, DD, L.attn_norm, nullptr, c.dec_eps, s->dpa, nullptr, 0, q.st));
        if (gemmf_on(q, EPI_STORE, s->dpa, DD, n, F.wqkv, DQ + 2 * DKV, nullptr, s->qkvd, DQ + 2 * DKV, nullptr)) return -1;
        // RoPE + K/V append + attention, its rows as the wo planes in s->dpa (attn's job)
        if (attn(l)) return -1;
        // wo + residual (decoder.c:552-560)
        if (gemmf_on(q, EPI_RESID, s->dpa, DQ, n, F.wo, DD, nullptr, x, DD, nullptr)) return -1;
        // RMSNorm * (1 + ada) -> planes, W1|W3 with SwiGLU into the w2 planes, w2 + residual (:562-606)
        CK(launch_rmsnorm_fplanes(x, n, DD, L.ffn_norm, m->ada_scale + (size_t)l * DD, c.dec_eps, s->dpa, nullptr, 0,
                                  q.st));
        if (gemmf_on(q, EPI_SWIGLU, s->dpa, DD, n, F.w13, 2 * DH, nullptr, nullptr, DH, s->dpc)) return -1;
        if (gemmf_on(q, EPI_RESID, s->dpc, DH, n, F.w2, DD, nullptr, x, DD, nullptr)) return -1;
    }
    return 0;
}

// M>1 rows (prefill) at logical positions pos0.. (voxtral_decoder.c:496-606)
static int run_decoder_rows(vox_hip_stream_t* s, float* x, int n, int pos0, const float* rope) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int DD = c.dec_dim, H = c.dec_heads, KVH = c.dec_kv_heads, hd = c.dec_head_dim;
    const int DQ = H * hd, DKV = KVH * hd, DH = c.dec_hidden;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t st = s->st;
    if (stream_alloc_dec_rows(s, n)) return -1;
    if (n > DEC_SLACK + 1 && pos0 > 0) return set_err("prefill of %d rows on a non-empty cache", n);
    // k_gemmf needs the fragment-major decoder copies (6.86 GB, made here on the first
    // prefill unless a batch made them) and the stream's plane buffers; when either cannot be
    // allocated the prefill takes the k_gemm2 layers below (same arithmetic, row-major weights)
    bool gf = n > 1 && dec_gemmf_ok(m, n);
    if (gf && (model_frag(m) || stream_dec_planes(s, n))) {
        vox_hip_clear_error();
        (void)hipGetLastError();  // the failed hipMalloc, so no later launch check reports it
        gf = false;
    }
    if (gf) {
        // the hand-off flags before the queue descriptor copies the pointer (a stream whose
        // encoder never ran a k_gemmf pass has none yet)
        if (!s->gflags) CK(dalloc(&s->gflags, gemmf_flag_ints()));
        return dec_layers_gemmf(s, GemmfQ{st, s->gws, s->gws_n, s->gflags, &s->gepoch}, x, n, [&](int l) -> int {
            float* Kc = dec_ring(s, s->dk, l);
            float* Vc = dec_ring(s, s->dv, l);
            CK(launch_rope_kv(s->qkvd, n, DQ, DKV, hd, rope, pos0, s->qd_, Kc, Vc, s->dcap, st, s->kv16));
            CK(launch_attn_rows_mf(hd, s->qd_, DQ, Kc, Vc, s->dcap, s->attd, DQ, n, H, KVH, pos0, 0, c.dec_window, scale,
                                   st, s->gws, s->gws_n, s->dpa, s->kv16));
            return 0;
        });
    }
    for (int l = 0; l < c.dec_layers; l++) {
        const DecLayerD& L = m->dec[l];
        float* Kc = dec_ring(s, s->dk, l);
        float* Vc = dec_ring(s, s->dv, l);
        CK(launch_rmsnorm_rows(x, DD, s->xnd, DD, L.attn_norm, nullptr, n, DD, c.dec_eps, st));
        CK(launch_gemm(EPI_STORE, 3, s->xnd, DD, L.wqkv, L.sqkv, DD, n, DQ + 2 * DKV, nullptr, s->qkvd, DQ + 2 * DKV, st, s->gws, s->gws_n));
        CK(launch_rope_kv(s->qkvd, n, DQ, DKV, hd, rope, pos0, s->qd_, Kc, Vc, s->dcap, st, s->kv16));
        CK(launch_attn_rows_mf(hd, s->qd_, DQ, Kc, Vc, s->dcap, s->attd, DQ, n, H, KVH, pos0, 0, c.dec_window, scale, st,
                             s->gws, s->gws_n, nullptr, s->kv16));
        CK(launch_gemm(EPI_RESID, 3, s->attd, DQ, L.wo, L.so, DQ, n, DD, nullptr, x, DD, st, s->gws, s->gws_n));
        CK(launch_rmsnorm_rows(x, DD, s->xnd, DD, L.ffn_norm, m->ada_scale + (size_t)l * DD, n, DD, c.dec_eps, st));
        CK(launch_gemm(EPI_SWIGLU, 3, s->xnd, DD, L.w13, L.s13, DD, n, 2 * DH, nullptr, s->gated, DH, st, s->gws, s->gws_n));
        CK(launch_gemm(EPI_RESID, 3, s->gated, DH, L.w2, L.s2, DH, n, DD, nullptr, x, DD, st, s->gws, s->gws_n));
    }
    return 0;
}

// One decoder step for the token whose input is already in s->xd[0..D).
// state != nullptr: positions come from device state (graph mode);
// otherwise pos/rope_row are host values (boundary twin).
static int enqueue_lm_head(vox_hip_stream_t* s, const int* state);

static int enqueue_step_layers(vox_hip_stream_t* s, const int* state, int pos, const float* rope_row,
                               int splits) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int DD = c.dec_dim, H = c.dec_heads, KVH = c.dec_kv_heads, hd = c.dec_head_dim;
    const int DQ = H * hd, DKV = KVH * hd, DH = c.dec_hidden;
    const float scale = 1.0f / sqrtf((float)hd);
    hipStream_t st = s->st;
    for (int l = 0; l < c.dec_layers; l++) {
        const DecLayerD& L = m->dec[l];
        float* Kc = dec_ring(s, s->dk, l);
        float* Vc = dec_ring(s, s->dv, l);
        GemvArgs a;
        memset(&a, 0, sizeof a);
        // norm -> QKV -> RoPE -> KV append (decoder.c:709-722)
        a.x = s->xd; a.K = DD; a.W = L.wqkv; a.wscale = L.sqkv; a.rows = DQ + 2 * DKV;
        a.norm_w = L.attn_norm; a.eps = c.dec_eps; a.y = s->qd_;
        a.qd = DQ; a.kvd = DKV; a.hd = hd;
        a.state = state; a.pos = pos;
        a.rope = state ? m->rope_dec : rope_row - (size_t)pos * hd;
        a.Kc = Kc; a.Vc = Vc; a.cap = s->dcap; a.kv16 = s->kv16;
        CK(launch_gemv(PRO_NORM, EPI_QKV, a, st));
        // attention over the last min(pos+1, window) keys (decoder.c:724-733)
        CK(launch_attn_decode(hd, s->qd_, Kc, Vc, s->dcap, state, pos, c.dec_window, scale, H, KVH,
                              s->part, s->attd, splits, st, s->kv16));
        // wo + residual (decoder.c:735-740)
        memset(&a, 0, sizeof a);
        a.x = s->attd; a.K = DQ; a.W = L.wo; a.wscale = L.so; a.rows = DD; a.y = s->xd;
        CK(launch_gemv(PRO_NONE, EPI_RESID, a, st));
        // norm * (1 + ada) -> W1|W3 -> silu * up (decoder.c:742-758)
        memset(&a, 0, sizeof a);
        a.x = s->xd; a.K = DD; a.W = L.w13; a.wscale = L.s13; a.rows = 2 * DH; a.norm_w = L.ffn_norm;
        a.ada = m->ada_scale + (size_t)l * DD; a.eps = c.dec_eps; a.y = s->gated;
        // profiling: HIP events recorded by the W1|W3 launch's own dispatch (eager steps)
        const bool gprof = s->profiling && state && !s->capturing && (int)s->pev.size() == 2 * c.dec_layers;
        if (gprof) CK(launch_gemv_timed(PRO_NORM_ADA, EPI_SWIGLU, a, s->pev[2 * l], s->pev[2 * l + 1], st));
        else CK(launch_gemv(PRO_NORM_ADA, EPI_SWIGLU, a, st));
        // W2 + residual (decoder.c:758-760)
        memset(&a, 0, sizeof a);
        a.x = s->gated; a.K = DH; a.W = L.w2; a.wscale = L.s2; a.rows = DD; a.y = s->xd;
        CK(launch_gemv(PRO_NONE, EPI_RESID, a, st));
    }
    return enqueue_lm_head(s, state);
}

// final norm + LM head (tied embeddings) + argmax partials (decoder.c:762-779)
static int enqueue_lm_head(vox_hip_stream_t* s, const int* state) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    hipStream_t st = s->st;
    GemvArgs a;
    memset(&a, 0, sizeof a);
    a.x = s->xd; a.K = c.dec_dim; a.W = m->tok_emb; a.wscale = m->tok_emb_s; a.rows = c.vocab; a.norm_w = m->dec_norm;
    a.eps = c.dec_eps; a.y = s->logits; a.part_val = s->pval; a.part_idx = s->pidx;
    a.part_alt = s->part_alt;
    CK(launch_gemv(PRO_NORM, (state && s->n_alt > 1) ? EPI_LOGITS_ALT : EPI_LOGITS, a, st));
    return 0;
}

// Step graph g serves contexts of up to 2^g * ATT_BLOCK_KEYS keys (the last one: the whole
// window); graph 0 runs one attention block per query head and no combine kernel.
static int graph_splits(const vox_hip_stream_t* s, int g) {
    return std::min(1 << g, attn_maxsplits(s->m->c.dec_window));
}

static int graph_index(const vox_hip_stream_t* s, int ctx) {
    const int need = (ctx + ATT_BLOCK_KEYS - 1) / ATT_BLOCK_KEYS;
    int g = 0;
    while ((1 << g) < need && (1 << g) < attn_maxsplits(s->m->c.dec_window)) g++;
    return g;
}

static int enqueue_graph_step(vox_hip_stream_t* s, int splits) {
    const vox_hip_config_t& c = s->m->c;
    if (enqueue_step_layers(s, s->state, 0, nullptr, splits)) return -1;
    CK(launch_argmax_final(s->pval, s->pidx, gemv_grid(c.vocab), s->state, s->tokens, s->tokens_cap,
                           s->adapter, s->adapter_cap, s->m->tok_emb, s->m->tok_emb_s, c.dec_dim, s->xd,
                           s->part_alt, s->n_alt > 1 ? s->alts : nullptr, s->st));
    return 0;
}

static int build_step_graph(vox_hip_stream_t* s, int gi) {
    if (s->step_exec[gi]) {
        hipGraphExecDestroy(s->step_exec[gi]);
        s->step_exec[gi] = nullptr;
    }
    hipGraph_t g = nullptr;
    CK(hipStreamBeginCapture(s->st, hipStreamCaptureModeThreadLocal));
    s->capturing = 1;
    int rc = enqueue_graph_step(s, graph_splits(s, gi));
    s->capturing = 0;
    hipError_t e = hipStreamEndCapture(s->st, &g);
    if (rc || e != hipSuccess) {
        if (g) hipGraphDestroy(g);
        return set_err("graph capture failed: %s", hipGetErrorString(e));
    }
    e = hipGraphInstantiate(&s->step_exec[gi], g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    if (e != hipSuccess) return set_err("graph instantiate failed: %s", hipGetErrorString(e));
    s->graph_ready |= 1 << gi;
    s->graph_alt = s->n_alt > 1;
    s->graph_rope_gen = s->m->rope_gen;
    return 0;
}

// Sampled kernel timing: after a batch of profiled steps, each layer's W1|W3 event pair
// (recorded by the kernel's dispatch packet) holds the last step's kernel duration.
static int collect_graph_profile(vox_hip_stream_t* s) {
    if (!s->profiling || !s->graph_prof) return 0;
    const vox_hip_config_t& c = s->m->c;
    for (int l = 0; l < c.dec_layers; l++) {
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, s->pev[2 * l], s->pev[2 * l + 1]));
        s->prof_ms += ms;
        s->prof_bytes += (double)2 * c.dec_hidden * c.dec_dim * 2;
        s->prof_launches++;
    }
    return 0;
}

static int use_graphs() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("VOX_HIP_GRAPH");
        v = (e && atoi(e) == 0) ? 0 : 1;
    }
    return v;
}

// n steps starting at logical kv position pos0 (host mirror): the replayed graph is the one
// with the fewest attention key splits that covers the longest context of the n steps.
static int run_steps(vox_hip_stream_t* s, int n, int pos0) {
    const vox_hip_config_t& c = s->m->c;
    const int gi = graph_index(s, std::min(pos0 + n, c.dec_window));
    const int splits = graph_splits(s, gi);
    if (s->profiling && use_graphs() && n > 1) {
        // profiled batch: the first n - 1 steps replay the graph, the last one (whose W1|W3
        // events collect_graph_profile reads) runs eagerly below
        s->profiling = 0;
        const int rc = run_steps(s, n - 1, pos0);
        s->profiling = 1;
        if (rc) return -1;
        pos0 += n - 1;
        n = 1;
    }
    if (!use_graphs() || s->profiling) {
        // eager launches of the same device-state kernels: profiling (the W1|W3 launches
        // carry dispatch-recorded HIP events, which a graph cannot hold), profilers that
        // cannot follow graph replays (VOX_HIP_GRAPH=0).
        if (s->profiling && s->pev.empty()) {
            s->pev.resize(2 * c.dec_layers);
            for (auto& e : s->pev) CK(hipEventCreate(&e));
        }
        s->graph_prof = s->profiling;
        for (int i = 0; i < n; i++)
            if (enqueue_graph_step(s, splits)) return -1;
        return 0;
    }
    if (s->graph_ready && (s->graph_alt != (s->n_alt > 1) || s->graph_rope_gen != s->m->rope_gen)) s->graph_ready = 0;
    if (!(s->graph_ready & (1 << gi)) && build_step_graph(s, gi)) return -1;
    for (int i = 0; i < n; i++) CK(hipGraphLaunch(s->step_exec[gi], s->st));
    return 0;
}

// copy ring entries [first, first + n) of a per-step device log (rec ints / floats per entry)
template <class T>
static int ring_read(const T* ring, int cap, int rec, long long first, int n, T* out, hipStream_t st) {
    while (n > 0) {
        const int slot = (int)(first % cap);
        const int k = std::min(n, cap - slot);
        CK(hipMemcpyAsync(out, ring + (size_t)slot * rec, (size_t)k * rec * sizeof(T), hipMemcpyDeviceToHost, st));
        out += (size_t)k * rec;
        first += k;
        n -= k;
    }
    return 0;
}

// prompt embeds + prefill rows 0..prompt_len-2 (voxtral.c:1036-1057) on the stream's queue;
// the first generated token then comes from row prompt_len-1 through a regular step
static int stream_prefill(vox_hip_stream_t* s) {
    vox_hip_model_t* m = s->m;
    const int np = 32 + m->delay_tokens;
    if (stream_alloc_dec_rows(s, np)) return -1;
    if (ensure_rope(s, np + 2)) return -1;
    CK(launch_embed_rows(s->adapter, m->tok_emb, m->tok_emb_s, 0, np, TOKEN_BOS, TOKEN_STREAMING_PAD, m->c.dec_dim,
                         s->xd, s->st));
    if (run_decoder_rows(s, s->xd, np, 0, m->rope_dec)) return -1;
    return stream_prefilled(s, s->st);
}

extern "C" int vox_hip_stream_decode(vox_hip_stream_t* s, int max_steps, int stop_at_eos,
                                     int* tokens_out, float* logits_out) {
    vox_hip_model_t* m = s->m;
    const vox_hip_config_t& c = m->c;
    const int D = c.dec_dim, V = c.vocab, hd = c.dec_head_dim;
    const int prompt_len = 1 + 32 + m->delay_tokens;
    int produced = 0;
    if (max_steps <= 0 || s->eos_seen) return 0;
    if (!s->started) {
        if (s->total_adapter < prompt_len) return 0;
        if (stream_prefill(s)) return -1;
    }
    const int step_base = s->n_generated;
    int avail = s->total_adapter - (s->h_state[1] > 0 ? s->h_state[1] : prompt_len - 1);
    {
        // host mirror of the device state (positions advance by exactly one per step)
        int st4[4];
        CK(hipMemcpyAsync(st4, s->state, sizeof st4, hipMemcpyDeviceToHost, s->st));
        CK(hipStreamSynchronize(s->st));
        memcpy(s->h_state, st4, sizeof st4);
        avail = s->total_adapter - st4[1];
    }
    if (ensure_rope(s, (long long)s->h_state[0] + avail + 1)) return -1;
    // step input for the first step of this call (later inputs are built by the previous
    // step's argmax kernel)
    if (avail > 0) CK(launch_embed_step(s->adapter, m->tok_emb, m->tok_emb_s, s->state, D, s->xd, s->st));
    int todo = std::min(max_steps, avail);
    std::vector<int> tok;
    while (produced < todo) {
        int b = std::min(STEP_BATCH, todo - produced);
        if (logits_out) b = 1;
        if (run_steps(s, b, s->h_state[0] + produced)) return -1;
        tok.resize(produced + b);
        if (ring_read(s->tokens, s->tokens_cap, 1, (long long)step_base + produced, b, tok.data() + produced, s->st))
            return -1;
        if (logits_out)
            CK(hipMemcpyAsync(logits_out + (size_t)produced * V, s->logits, (size_t)V * 4, hipMemcpyDeviceToHost, s->st));
        CK(hipStreamSynchronize(s->st));
        if (collect_graph_profile(s)) return -1;
        int eos_at = -1;
        if (stop_at_eos)
            for (int i = produced; i < produced + b; i++)
                if (tok[i] == TOKEN_EOS) { eos_at = i; break; }
        if (eos_at >= 0) {
            produced = eos_at + 1;
            s->eos_seen = 1;
            break;
        }
        produced += b;
    }
    if (tokens_out) memcpy(tokens_out, tok.data(), (size_t)produced * 4);
    s->n_generated += produced;
    // host mirror; after an EOS the device ran ahead by at most one batch (never read again
    // in non-continuous mode, voxtral.c:1140-1144)
    s->h_state[0] += produced;
    s->h_state[1] += produced;
    if (produced) s->h_state[2] = tok[produced - 1];
    s->h_state[3] = s->n_generated;
    (void)hd;
    return produced;
}

// vox_stream_set_alt (voxtral.c:1329-1337)
extern "C" int vox_hip_stream_set_alt(vox_hip_stream_t* s, int n_alt, float cutoff) {
    if (!s) return -1;
    if (n_alt < 1) n_alt = 1;
    if (n_alt > VOX_HIP_MAX_ALT) n_alt = VOX_HIP_MAX_ALT;
    if (cutoff < 0) cutoff = 0;
    if (cutoff > 1) cutoff = 1;
    s->n_alt = n_alt;
    s->alt_cutoff = cutoff;
    return 0;
}

// stream_fill_alts (voxtral.c:955-1010) for generated steps [first, first+n): the device
// left, per step, p_best and the three most probable text tokens other than the chosen
// one; the reference's acceptance rule is applied here.  ids_out [n][VOX_HIP_MAX_ALT]:
// [0] = the chosen token, then accepted alternatives, -1 after the first rejection (or
// beyond n_alt).  probs_out (optional) holds the matching softmax probabilities.
extern "C" int vox_hip_stream_read_alts(vox_hip_stream_t* s, int first, int n, int* ids_out,
                                        float* probs_out) {
    if (!s || first < 0 || n < 0 || first + n > s->n_generated || first < s->n_generated - s->tokens_cap)
        return set_err("alt range out of bounds (the last %d steps are kept)", s->tokens_cap);
    if (n == 0) return 0;
    std::vector<float> rec((size_t)n * ALT_REC);
    std::vector<int> tok(n);
    if (ring_read(s->alts, s->tokens_cap, ALT_REC, first, n, rec.data(), s->st) ||
        ring_read(s->tokens, s->tokens_cap, 1, first, n, tok.data(), s->st))
        return -1;
    CK(hipStreamSynchronize(s->st));
    for (int i = 0; i < n; i++) {
        int* ids = ids_out + (size_t)i * VOX_HIP_MAX_ALT;
        float* pr = probs_out ? probs_out + (size_t)i * VOX_HIP_MAX_ALT : nullptr;
        const float* r = rec.data() + (size_t)i * ALT_REC;
        for (int k = 0; k < VOX_HIP_MAX_ALT; k++) {
            ids[k] = -1;
            if (pr) pr[k] = 0.f;
        }
        ids[0] = tok[i];
        if (s->n_alt <= 1) continue;
        const float best_prob = r[0];
        if (pr) pr[0] = best_prob;
        if (best_prob <= 0) continue;
        for (int k = 1; k < s->n_alt; k++) {
            int id;
            memcpy(&id, &r[1 + 2 * (k - 1)], 4);
            const float p = r[2 + 2 * (k - 1)];
            if (id < 0) break;
            const float rr = 1.0f - p / best_prob;
            if (rr > s->alt_cutoff) break;
            ids[k] = id;
            if (pr) pr[k] = p;
        }
    }
    return 0;
}

extern "C" int vox_hip_stream_state(vox_hip_stream_t* s, int* out6) {
    out6[0] = s->h_state[0];
    out6[1] = s->h_state[1];
    out6[2] = s->h_state[2];
    out6[3] = s->started;
    out6[4] = s->eos_seen;
    out6[5] = s->n_generated;
    return 0;
}

extern "C" int vox_hip_stream_set_profiling(vox_hip_stream_t* s, int enable) {
    s->profiling = enable;
    s->prof_ms = 0;
    s->prof_bytes = 0;
    s->prof_launches = 0;
    return 0;
}

extern "C" int vox_hip_stream_profile(vox_hip_stream_t* s, double* out8) {
    out8[0] = s->prof_ms;
    out8[1] = s->prof_bytes;
    out8[2] = (double)s->prof_launches;
    out8[3] = s->prof_launches ? s->prof_ms / s->prof_launches : 0.0;
    out8[4] = 0;  // what the events bracket: the W1|W3 GEMV of every layer
    out8[5] = s->prof_launches ? s->prof_bytes / s->prof_launches : 0.0;
    // k_gemmf stage ranges an owner recomputed because a partial did not arrive in time
    int rec = 0;
    if (s->gflags) {
        CK(hipMemcpyAsync(&rec, s->gflags + gemmf_grid(), sizeof rec, hipMemcpyDeviceToHost, s->st));
        CK(hipStreamSynchronize(s->st));
    }
    out8[6] = rec;
    out8[7] = 0.0;
    return 0;
}

// ---------------------------------------------------------------------------
// Reference-boundary twins (host pointers; voxtral_metal.h)
//
// Any M, N, K: a weight is uploaded once per (host pointer, N, K) into a zero-padded
// [Np, Kp] device copy (Np a multiple of 128, Kp of 64: the k_gemm2 tile), the activation
// rows go into [M, Kp] with zero columns, and C comes back through a pitched copy, so the
// padding never reaches the caller.  M = 1 takes the GEMV when the padded shape suits it.
// Every HIP call is checked; the void functions report through vox_hip_last_error().
// ---------------------------------------------------------------------------
struct TwinW {
    uint8_t* w;   // [Np, Kp] bf16 or int8
    float* s;     // Q8 row scales [Np] (null: bf16)
    int N, K, Np, Kp;
};
struct TwinKey {
    const void* p;
    int n, k;
    bool operator==(const TwinKey& o) const { return p == o.p && n == o.n && k == o.k; }
};
struct TwinKeyHash {
    size_t operator()(const TwinKey& t) const {
        return std::hash<const void*>()(t.p) ^ ((size_t)t.n * 0x9e3779b97f4a7c15ull) ^ ((size_t)t.k << 1);
    }
};
static std::mutex g_twin_mu;
static std::unordered_map<TwinKey, TwinW, TwinKeyHash> g_wcache;  // (host ptr, N, K) -> device copy
static hipStream_t g_twin_st = nullptr;
static float* g_twin_ws = nullptr;  // split-K partials of the twin GEMMs
static float *g_tA = nullptr, *g_tC = nullptr, *g_tQ = nullptr, *g_tK = nullptr, *g_tV = nullptr, *g_tO = nullptr;
static size_t g_tA_n = 0, g_tC_n = 0, g_tQ_n = 0, g_tK_n = 0, g_tV_n = 0, g_tO_n = 0;
static float* g_tWs = nullptr;  // attention key-range partials
static size_t g_tWs_n = 0;

static int pad_to(int v, int a) { return (v + a - 1) / a * a; }

static int twin_buf(float** p, size_t* cap, size_t n) {
    if (n <= *cap) return 0;
    dfree(*p);
    *cap = 0;
    CK(dalloc(p, n));
    *cap = n;
    return 0;
}

// device copy of a host weight [N, K] (+ Q8 row scales), zero-padded to the GEMM tile
static const TwinW* twin_weight(const void* host, const float* scales, int N, int K) {
    if (!host || N <= 0 || K <= 0) {
        set_err("twin weight: null pointer or empty shape (%d x %d)", N, K);
        return nullptr;
    }
    const TwinKey key{host, N, K};
    auto it = g_wcache.find(key);
    if (it != g_wcache.end()) return &it->second;
    TwinW t{nullptr, nullptr, N, K, pad_to(N, 128), pad_to(K, 64)};
    const size_t esz = scales ? 1 : 2;
    hipError_t e = dalloc(&t.w, (size_t)t.Np * t.Kp * esz);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(t.w, (size_t)t.Kp * esz, host, (size_t)K * esz, (size_t)K * esz, N,
                             hipMemcpyHostToDevice, g_twin_st);
    if (e == hipSuccess && scales) {
        e = dalloc(&t.s, (size_t)t.Np);
        if (e == hipSuccess) e = hipMemcpyAsync(t.s, scales, (size_t)N * 4, hipMemcpyHostToDevice, g_twin_st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(g_twin_st);
    if (e != hipSuccess) {
        dfree(t.w);
        dfree(t.s);
        set_err("twin weight upload (%d x %d): %s", N, K, hipGetErrorString(e));
        return nullptr;
    }
    return &(g_wcache[key] = t);
}

static int twin_init() {
    if (!g_inited && !vox_hip_init()) return -1;
    if (!g_twin_st) CK(hipStreamCreateWithFlags(&g_twin_st, hipStreamNonBlocking));
    if (!g_twin_ws) CK(dalloc(&g_twin_ws, GEMM_WS_ELEMS));
    return 0;
}

// host rows [M, K] -> device [M, Kp] (zero columns past K)
static int twin_put_rows(float** buf, size_t* cap, const float* host, int M, int K, int Kp) {
    if (!host) return set_err("twin: null input");
    if (twin_buf(buf, cap, (size_t)M * Kp)) return -1;
    if (Kp != K) {
        CK(hipMemsetAsync(*buf, 0, (size_t)M * Kp * 4, g_twin_st));
        CK(hipMemcpy2DAsync(*buf, (size_t)Kp * 4, host, (size_t)K * 4, (size_t)K * 4, M, hipMemcpyHostToDevice,
                            g_twin_st));
    } else {
        CK(hipMemcpyAsync(*buf, host, (size_t)M * K * 4, hipMemcpyHostToDevice, g_twin_st));
    }
    return 0;
}

// device [M, Np] -> host [M, N]
static int twin_get_rows(float* host, const float* dev, int M, int N, int Np) {
    if (!host) return set_err("twin: null output");
    CK(hipMemcpy2DAsync(host, (size_t)N * 4, dev, (size_t)Np * 4, (size_t)N * 4, M, hipMemcpyDeviceToHost, g_twin_st));
    return 0;
}

// dC[M, W.Np] = dA[M, W.Kp] . W^T on the twin stream
static int twin_gemm_dev(int M, const float* dA, const TwinW& W, float* dC) {
    if (M == 1 && gemv_ok(W.Np, W.Kp, W.s != nullptr)) {
        GemvArgs a;
        memset(&a, 0, sizeof a);
        a.x = dA; a.K = W.Kp; a.W = W.w; a.wscale = W.s; a.rows = W.Np; a.y = dC;
        CK(launch_gemv(PRO_NONE, EPI_STORE, a, g_twin_st));
        return 0;
    }
    CK(launch_gemm(EPI_STORE, 3, dA, W.Kp, W.w, W.s, W.Kp, M, W.Np, nullptr, dC, W.Np, g_twin_st, g_twin_ws,
                   GEMM_WS_ELEMS));
    return 0;
}

static int twin_sgemm(int M, int N, int K, const float* A, const void* B, const float* scales, float* C) {
    if (M <= 0 || N <= 0 || K <= 0) return M == 0 ? 0 : set_err("sgemm: bad shape %d x %d x %d", M, N, K);
    if (twin_init()) return -1;
    const TwinW* W = twin_weight(B, scales, N, K);
    if (!W) return -1;
    if (twin_put_rows(&g_tA, &g_tA_n, A, M, K, W->Kp) || twin_buf(&g_tC, &g_tC_n, (size_t)M * W->Np) ||
        twin_gemm_dev(M, g_tA, *W, g_tC) || twin_get_rows(C, g_tC, M, N, W->Np))
        return -1;
    CK(hipStreamSynchronize(g_twin_st));
    return 0;
}

extern "C" void vox_hip_sgemm_bf16(int M, int N, int K, const float* A, const uint16_t* B, float* C) {
    std::lock_guard<std::mutex> lk(g_twin_mu);
    twin_sgemm(M, N, K, A, B, nullptr, C);
}

extern "C" void vox_hip_sgemm_q8(int M, int N, int K, const float* A, const int8_t* B, const float* scales,
                                 float* C) {
    std::lock_guard<std::mutex> lk(g_twin_mu);
    if (!scales) { set_err("sgemm_q8: null scales"); return; }
    twin_sgemm(M, N, K, A, B, scales, C);
}

// voxtral_metal.m:1274-1414: the input uploaded once, three projections into three arrays
extern "C" void vox_hip_fused_qkv_bf16(int M, int K, const float* input, const uint16_t* wq, int Nq,
                                       const uint16_t* wk, int Nk, const uint16_t* wv, int Nv,
                                       float* q, float* k, float* v) {
    std::lock_guard<std::mutex> lk(g_twin_mu);
    if (M <= 0) return;
    if (twin_init()) return;
    const TwinW* W[3] = {twin_weight(wq, nullptr, Nq, K), twin_weight(wk, nullptr, Nk, K),
                         twin_weight(wv, nullptr, Nv, K)};
    if (!W[0] || !W[1] || !W[2]) return;
    float* outs[3] = {q, k, v};
    float* dO[3] = {nullptr, nullptr, nullptr};
    size_t* caps[3] = {&g_tQ_n, &g_tK_n, &g_tV_n};
    float** bufs[3] = {&g_tQ, &g_tK, &g_tV};
    if (twin_put_rows(&g_tA, &g_tA_n, input, M, K, W[0]->Kp)) return;
    for (int i = 0; i < 3; i++) {
        if (twin_buf(bufs[i], caps[i], (size_t)M * W[i]->Np) || twin_gemm_dev(M, g_tA, *W[i], *bufs[i])) return;
        dO[i] = *bufs[i];
    }
    for (int i = 0; i < 3; i++)
        if (twin_get_rows(outs[i], dO[i], M, W[i]->N, W[i]->Np)) return;
    if (hipStreamSynchronize(g_twin_st) != hipSuccess) set_err("fused_qkv: sync failed");
}

__global__ void k_silu_mul(float* g, const float* u, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        float v = g[i];
        g[i] = v / (1.0f + expf(-v)) * u[i];
    }
}

// voxtral_metal.m:1416-1572: (silu(x w1^T) * x w3^T) w2^T; the caller adds the w2 bias
extern "C" void vox_hip_fused_ffn_bf16(int M, int dim, int hidden, const float* input,
                                       const uint16_t* w1, const uint16_t* w3, const uint16_t* w2,
                                       float* output) {
    std::lock_guard<std::mutex> lk(g_twin_mu);
    if (M <= 0) return;
    if (twin_init()) return;
    const TwinW* d1 = twin_weight(w1, nullptr, hidden, dim);
    const TwinW* d3 = twin_weight(w3, nullptr, hidden, dim);
    const TwinW* d2 = twin_weight(w2, nullptr, dim, hidden);
    if (!d1 || !d3 || !d2) return;
    // gate / up rows [M, Hp]; the padded hidden columns are silu(0) * 0 = 0 and meet the
    // zero K padding of w2
    const int Hp = d1->Np;
    if (d2->Kp != Hp) { set_err("fused_ffn: padded hidden %d != %d", d2->Kp, Hp); return; }
    if (twin_put_rows(&g_tA, &g_tA_n, input, M, dim, d1->Kp) || twin_buf(&g_tQ, &g_tQ_n, (size_t)M * Hp) ||
        twin_buf(&g_tK, &g_tK_n, (size_t)M * Hp) || twin_buf(&g_tC, &g_tC_n, (size_t)M * d2->Np) ||
        twin_gemm_dev(M, g_tA, *d1, g_tQ) || twin_gemm_dev(M, g_tA, *d3, g_tK))
        return;
    const size_t n = (size_t)M * Hp;
    hipLaunchKernelGGL(k_silu_mul, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, g_twin_st, g_tQ, g_tK, n);
    if (hipGetLastError() != hipSuccess) { set_err("fused_ffn: silu_mul launch failed"); return; }
    if (twin_gemm_dev(M, g_tQ, *d2, g_tC) || twin_get_rows(output, g_tC, M, dim, d2->Np)) return;
    if (hipStreamSynchronize(g_twin_st) != hipSuccess) set_err("fused_ffn: sync failed");
}

static int twin_attention(float* out, const float* Q, const float* K, const float* V, int seq_q, int seq_k,
                          int n_heads, int n_kv_heads, int head_dim, float scale, int window_size, int q_offset) {
    if (twin_init()) return -1;
    if (seq_q <= 0) return 0;
    if (!out || !Q || !K || !V) return set_err("encoder_attention: null pointer");
    if (q_offset < 0 || q_offset + seq_q > seq_k) return set_err("encoder_attention: queries beyond keys");
    if (n_kv_heads <= 0 || n_heads % n_kv_heads) return set_err("encoder_attention: heads %d / kv heads %d", n_heads, n_kv_heads);
    const size_t qn = (size_t)seq_q * n_heads * head_dim, kn = (size_t)seq_k * n_kv_heads * head_dim;
    if (twin_buf(&g_tQ, &g_tQ_n, qn) || twin_buf(&g_tK, &g_tK_n, kn) || twin_buf(&g_tV, &g_tV_n, kn) ||
        twin_buf(&g_tO, &g_tO_n, qn))
        return -1;
    CK(hipMemcpyAsync(g_tQ, Q, qn * 4, hipMemcpyHostToDevice, g_twin_st));
    CK(hipMemcpyAsync(g_tK, K, kn * 4, hipMemcpyHostToDevice, g_twin_st));
    CK(hipMemcpyAsync(g_tV, V, kn * 4, hipMemcpyHostToDevice, g_twin_st));
    const int W = window_size > 0 ? window_size : (1 << 30);
    // few query rows: the key-range split + combine path the streaming encoder takes
    float* ws = nullptr;
    size_t wsn = 0;
    if (n_heads * ((seq_q + 15) / 16) < 256) {
        wsn = (size_t)n_heads * seq_q * 16 * (head_dim + 2);
        if (twin_buf(&g_tWs, &g_tWs_n, wsn)) return -1;
        ws = g_tWs;
    }
    CK(launch_attn_rows_mf(head_dim, g_tQ, n_heads * head_dim, g_tK, g_tV, seq_k, g_tO, n_heads * head_dim, seq_q,
                         n_heads, n_kv_heads, q_offset, 0, W, scale, g_twin_st, ws, wsn));
    CK(hipMemcpyAsync(out, g_tO, qn * 4, hipMemcpyDeviceToHost, g_twin_st));
    CK(hipStreamSynchronize(g_twin_st));
    return 0;
}

extern "C" void vox_hip_encoder_attention(float* out, const float* Q, const float* K, const float* V,
                                          int seq_q, int seq_k, int n_heads, int n_kv_heads,
                                          int head_dim, float scale, int window_size, int q_offset) {
    std::lock_guard<std::mutex> lk(g_twin_mu);
    twin_attention(out, Q, K, V, seq_q, seq_k, n_heads, n_kv_heads, head_dim, scale, window_size, q_offset);
}

static int upload_rope_rows(vox_hip_stream_t* s, const float* rope, size_t n) {
    if (n > (size_t)s->rope_rows_cap) {
        dfree(s->rope_rows);
        CK(dalloc(&s->rope_rows, n));
        s->rope_rows_cap = (int)n;
    }
    CK(hipMemcpyAsync(s->rope_rows, rope, n * 4, hipMemcpyHostToDevice, s->st));
    return 0;
}

extern "C" int vox_hip_encoder_full_step(vox_hip_stream_t* s, float* x, int new_len,
                                         const float* rope_freqs, int logical_start) {
    const vox_hip_config_t& c = s->m->c;
    const int ED = c.enc_dim;
    if (stream_alloc_frames(s, 2 * new_len + 8)) return -1;
    float* xin = s->x_enc + (size_t)4 * ED;
    CK(hipMemcpyAsync(xin, x, (size_t)new_len * ED * 4, hipMemcpyHostToDevice, s->st));
    if (upload_rope_rows(s, rope_freqs, (size_t)new_len * c.enc_head_dim)) return -1;
    for (int r0 = 0; r0 < new_len; r0 += ENC_SUB) {
        int nr = std::min(ENC_SUB, new_len - r0);
        if (run_encoder_rows(s, xin + (size_t)r0 * ED, nr, (long long)logical_start + r0,
                             s->rope_rows + (size_t)r0 * c.enc_head_dim))
            return -1;
    }
    CK(hipMemcpyAsync(x, xin, (size_t)new_len * ED * 4, hipMemcpyDeviceToHost, s->st));
    CK(hipStreamSynchronize(s->st));
    return 0;
}

extern "C" int vox_hip_decoder_prefill_step(vox_hip_stream_t* s, float* x, int seq_len,
                                            const float* rope_freqs, int logical_start) {
    const vox_hip_config_t& c = s->m->c;
    if (stream_alloc_dec_rows(s, seq_len)) return -1;
    CK(hipMemcpyAsync(s->xd, x, (size_t)seq_len * c.dec_dim * 4, hipMemcpyHostToDevice, s->st));
    if (upload_rope_rows(s, rope_freqs, (size_t)seq_len * c.dec_head_dim)) return -1;
    if (run_decoder_rows(s, s->xd, seq_len, logical_start, s->rope_rows)) return -1;
    CK(hipMemcpyAsync(x, s->xd, (size_t)seq_len * c.dec_dim * 4, hipMemcpyDeviceToHost, s->st));
    CK(hipStreamSynchronize(s->st));
    return 0;
}

extern "C" void vox_hip_decoder_start(vox_hip_stream_t* s, const float* x, int dim) {
    if (!s || !x || dim != s->m->c.dec_dim) {
        set_err("decoder_start: dim %d != dec_dim", dim);
        return;
    }
    if (hipMemcpyAsync(s->xd, x, (size_t)dim * 4, hipMemcpyHostToDevice, s->st) != hipSuccess)
        set_err("decoder_start upload failed");
}

extern "C" void vox_hip_decoder_end(vox_hip_stream_t* s) {
    if (s && hipStreamSynchronize(s->st) != hipSuccess) set_err("decoder_end: stream sync failed");
}

extern "C" int vox_hip_decoder_full_step(vox_hip_stream_t* s, const float* rope_freqs, int logical_pos,
                                         float* logits) {
    const vox_hip_config_t& c = s->m->c;
    if (upload_rope_rows(s, rope_freqs, (size_t)c.dec_head_dim)) return -1;
    const int ctx = std::min(logical_pos + 1, c.dec_window);
    if (enqueue_step_layers(s, nullptr, logical_pos, s->rope_rows, (ctx + ATT_BLOCK_KEYS - 1) / ATT_BLOCK_KEYS))
        return -1;
    // argmax into the twin's own state so the graph-mode device state is untouched
    int* tmp_state = s->twin_state;
    int st4[4] = {0, 0, 0, 0};
    CK(hipMemcpyAsync(tmp_state, st4, sizeof st4, hipMemcpyHostToDevice, s->st));
    CK(launch_argmax_final(s->pval, s->pidx, gemv_grid(c.vocab), tmp_state, nullptr, 0, nullptr, 0,
                           nullptr, nullptr, c.dec_dim, nullptr, nullptr, nullptr, s->st));
    CK(hipMemcpyAsync(st4, tmp_state, sizeof st4, hipMemcpyDeviceToHost, s->st));
    if (logits) CK(hipMemcpyAsync(logits, s->logits, (size_t)c.vocab * 4, hipMemcpyDeviceToHost, s->st));
    CK(hipStreamSynchronize(s->st));
    return st4[2];
}

extern "C" void* vox_hip_device_upload(const void* host, size_t bytes) {
    void* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) { set_err("device_upload: hipMalloc(%zu) failed", bytes); return nullptr; }
    if (h2d(d, host, bytes) != hipSuccess) { hipFree(d); set_err("device_upload: copy failed"); return nullptr; }
    return d;
}

extern "C" int vox_hip_device_free(void* dev) {
    CK(hipFree(dev));
    return 0;
}

// ---------------------------------------------------------------------------
// Cross-stream batched greedy decoding (C4).  Row i of every batch
// activation buffer belongs to stream i; the weight GEMMs run once per step for all rows
// (M = streams), attention / RoPE / KV append / argmax use each stream's own state, rings
// and adapter rows.  Each stream's device state and token log advance exactly as in
// vox_hip_stream_decode, so streams can switch between the two paths.
// ---------------------------------------------------------------------------
struct vox_hip_batch {
    vox_hip_model_t* m;
    int cap;
    hipStream_t st;
    float *x, *q, *att, *logits, *pval, *palt;
    float* part;     // split-K slabs of the current projection (k_skl), consumed by the next kernel
    float* ssq;      // row sums of squares per 256-column slice (k_resid_xw_fplanes -> k_skl)
    int* ticket;     // k_sklx slice tickets (W1|W3 with the SwiGLU folded in; VOX_HIP_BATCH_SWX=0: off)
    int* pidx;
    uint16_t *xp_d, *xp_q, *xp_h;  // skinny-GEMM inputs: [3][16][K] bf16 planes of the rows (fragment order)
    float* apart;    // decode-attention partials + arrival counters, apart_n floats per slot
    size_t apart_n;
    // the slot table (VOX_MAX_BATCH BatchSlot) followed by the token log [VOX_MAX_BATCH][BATCH_TOKLOG],
    // in device memory and mirrored in pinned host memory (one copy each way per step chunk)
    BatchSlot* slots;
    BatchSlot* hslots;
    // step graphs [kv16][slot bucket 1, 2, 4, 8, 16, 32][attention splits bucket]: their kernel
    // arguments point at the slot table and the batch's buffers only, so they stay valid as
    // streams come and go; captured again only when the model's rope table moves
    hipGraphExec_t gexec[2][6][STEP_GRAPHS];
    int grope_gen;
    // rows of the last call (b->logits row i = stream luid[i], from its last step when llive[i])
    unsigned long long luid[VOX_MAX_BATCH];
    int llive[VOX_MAX_BATCH];
    int lnb;
    long long n_calls, n_replays, n_rows, n_captures, n_prefill_passes, n_prefilled;
    // split-K workspace of the stacked prefills (not the lead stream's: with an encoder pass
    // running beside the batched steps, that stream's queue may be using its own), and the
    // k_gemmf partial-tile flags + epoch of the batch queue's prefill launches
    float* pgws;
    int* gflags;
    int gepoch;
    // a call begun by batch_begin and not yet finished (vox_hip_batch_begin_rows /
    // vox_hip_batch_finish): its streams, outputs and the steps left after the chunk in flight
    struct {
        int active, n, max_steps, stop_at_eos, K, nb, gb, gi, splits, kv16, done, k;
        vox_hip_stream_t* streams[VOX_MAX_BATCH];
        int* tokens_out;
        int* counts_out;
    } call;
};

static int* slot_toklog(BatchSlot* slots) { return reinterpret_cast<int*>(slots + VOX_MAX_BATCH); }
static const size_t SLOT_BYTES = sizeof(BatchSlot) * VOX_MAX_BATCH + sizeof(int) * VOX_MAX_BATCH * BATCH_TOKLOG;

// pack one [N, K] matrix (bf16, or int8 when q8) into fragment order (k_frag_pack)
static int frag_copy(uint8_t** dst, const uint8_t* src, int N, int K, int q8) {
    CK(dalloc(dst, (size_t)N * K * (q8 ? 1 : 2)));
    CK(launch_frag_pack(src, N, K, q8, *dst, nullptr));
    CK(hipStreamSynchronize(nullptr));
    return 0;
}

// fragment-major copies of the decoder matrices and the LM head, made once per model, on the
// first batch or the first bf16 prefill of more than one row (6.86 GB bf16 / 3.83 GB Q8 beside
// the row-major weights the single-stream GEMVs read).  All or nothing: a failed copy frees
// what it had made, so the model holds either every copy or none.
static int model_frag(vox_hip_model_t* m) {
    if (m->lm_frag) return 0;
    const vox_hip_config_t& c = m->c;
    const int DD = c.dec_dim, DQ = c.dec_heads * c.dec_head_dim, DKV = c.dec_kv_heads * c.dec_head_dim;
    const int DH = c.dec_hidden;
    std::vector<DecFragD> F(c.dec_layers, DecFragD{});
    uint8_t* lm = nullptr;
    bool ok = true;
    for (int l = 0; l < c.dec_layers && ok; l++) {
        const DecLayerD& L = m->dec[l];
        ok = !frag_copy(&F[l].wqkv, L.wqkv, DQ + 2 * DKV, DD, L.sqkv != nullptr) &&
             !frag_copy(&F[l].wo, L.wo, DD, DQ, L.so != nullptr) &&
             !frag_copy(&F[l].w13, L.w13, 2 * DH, DD, L.s13 != nullptr) &&
             !frag_copy(&F[l].w2, L.w2, DD, DH, L.s2 != nullptr);
    }
    if (ok) ok = !frag_copy(&lm, m->tok_emb, c.vocab, DD, m->tok_emb_s != nullptr);
    if (!ok) {
        for (auto& f : F) { dfree(f.wqkv); dfree(f.wo); dfree(f.w13); dfree(f.w2); }
        dfree(lm);
        return -1;
    }
    m->dfrag.swap(F);
    m->lm_frag = lm;
    return 0;
}

static void batch_drop_graphs(vox_hip_batch_t* b) {
    for (auto& k : b->gexec)
        for (auto& g : k)
            for (auto& e : g)
                if (e) {
                    hipGraphExecDestroy(e);
                    e = nullptr;
                }
}

extern "C" void vox_hip_batch_free(vox_hip_batch_t* b) {
    if (!b) return;
    if (b->st) hipStreamSynchronize(b->st);
    dfree(b->x); dfree(b->part); dfree(b->ssq); dfree(b->ticket); dfree(b->q); dfree(b->att);
    dfree(b->logits); dfree(b->pval); dfree(b->pidx); dfree(b->palt); dfree(b->apart);
    dfree(b->xp_d); dfree(b->xp_q); dfree(b->xp_h); dfree(b->pgws); dfree(b->gflags);
    if (b->slots) hipFree(b->slots);
    if (b->hslots) hipHostFree(b->hslots);
    batch_drop_graphs(b);
    if (b->st) hipStreamDestroy(b->st);
    delete b;
}

extern "C" vox_hip_batch_t* vox_hip_batch_create(vox_hip_model_t* m, int max_streams) {
    if (!m || max_streams < 1 || max_streams > VOX_MAX_BATCH) {
        set_err("batch size must be 1..%d", VOX_MAX_BATCH);
        return nullptr;
    }
    const vox_hip_config_t& c = m->c;
    if (c.dec_head_dim != 128 || c.dec_heads % c.dec_kv_heads || c.dec_heads / c.dec_kv_heads > 4 ||
        c.dec_dim % 256 || c.dec_dim / 256 > SKL_MAX_SLICES) {
        set_err("batched decode needs head_dim 128, <= 4 query heads per kv head and dec_dim = 256 k <= 3072");
        return nullptr;
    }
    vox_hip_batch_t* b = new vox_hip_batch_t();
    memset((void*)b, 0, sizeof *b);
    b->m = m;
    b->cap = max_streams;
    const size_t D = c.dec_dim, QKV = c.dec_heads * c.dec_head_dim + 2 * c.dec_kv_heads * c.dec_head_dim;
    const size_t S = VOX_MAX_BATCH;  // rows of the slot-indexed buffers (graphs of any bucket)
    auto fail = [&]() -> vox_hip_batch_t* { vox_hip_batch_free(b); return nullptr; };
#define TRYH(x) do { hipError_t e__ = (x); if (e__ != hipSuccess) { set_err("%s: %s", #x, hipGetErrorString(e__)); return fail(); } } while (0)
    TRYH(queue_high_priority(&b->st));
    TRYH(dalloc(&b->x, S * D));
    {
        const size_t DQ = (size_t)c.dec_heads * c.dec_head_dim, DH = c.dec_hidden;
        const size_t n = std::max(std::max(skl_splits(D, (int)QKV) * QKV, skl_splits(DQ, D) * D),
                                  std::max(skl_splits(D, 2 * DH) * 2 * DH, skl_splits(DH, D) * D));
        if (!skl_splits(D) || !skl_splits(DQ) || !skl_splits(DH)) {
            set_err("batched decode needs dec_dim, heads*head_dim and dec_hidden divisible by 256");
            return fail();
        }
        TRYH(dalloc(&b->part, (size_t)S * n));  // [row block][split][16][N] for the S slot rows
    }
    TRYH(dalloc(&b->ssq, (size_t)SK_ROWS * SKX_TICKETS));  // [slices][16], any slice count
    TRYH(dalloc(&b->ticket, (size_t)SKX_TICKETS));
    TRYH(dalloc(&b->q, S * c.dec_heads * c.dec_head_dim));
    TRYH(dalloc(&b->att, S * c.dec_heads * c.dec_head_dim));
    TRYH(dalloc(&b->logits, S * c.vocab));
    TRYH(dalloc(&b->pval, S * ARGB));
    TRYH(dalloc(&b->pidx, S * ARGB));
    TRYH(dalloc(&b->palt, S * ARGB * ALT_PART));
    // attention partials + one arrival count per kv head (zeroed; reset by the merging block)
    b->apart_n = (size_t)c.dec_heads * attn_maxch(c.dec_window) * (c.dec_head_dim + 2) + c.dec_kv_heads;
    TRYH(dalloc(&b->apart, S * b->apart_n));
    TRYH(hipMalloc((void**)&b->slots, SLOT_BYTES));
    TRYH(hipMemset(b->slots, 0, SLOT_BYTES));
    TRYH(hipHostMalloc((void**)&b->hslots, SLOT_BYTES, hipHostMallocDefault));
    memset((void*)b->hslots, 0, SLOT_BYTES);
    if (model_frag(m)) return fail();
    TRYH(dalloc(&b->xp_d, (size_t)3 * S * D));  // [row block][3][16][K]
    TRYH(dalloc(&b->xp_q, (size_t)3 * S * c.dec_heads * c.dec_head_dim));
    TRYH(dalloc(&b->xp_h, (size_t)3 * S * c.dec_hidden));
#undef TRYH
    return b;
}

// the batched step's projections: k_skl, one burst of column groups per block
static hipError_t batch_gemm(const uint16_t* xs, int K, const void* Wf, const float* wscale, int N, int nb, float* part,
                             hipStream_t st, const float* ssq = nullptr, int nsl = 0, float eps = 0.f) {
    return launch_gemm_skl(xs, K, Wf, wscale, N, nb, part, st, ssq, nsl, eps, 1);
}

// one batched step over slots 0..nb-1 of the slot table (their input rows already in b->x)
static int batch_step(vox_hip_batch_t* b, int nb, int splits, int kv16) {
    vox_hip_model_t* m = b->m;
    const vox_hip_config_t& c = m->c;
    const int DD = c.dec_dim, H = c.dec_heads, KVH = c.dec_kv_heads, hd = c.dec_head_dim;
    const int DQ = H * hd, DKV = KVH * hd, DH = c.dec_hidden;
    const float scale = 1.0f / sqrtf((float)hd);
    const int cap = c.dec_window + DEC_SLACK;
    const size_t ring_layer = (size_t)cap * DKV * (kv16 ? 2 : 4);
    hipStream_t st = b->st;
    AttnPtrs ap;
    memset(&ap, 0, sizeof ap);
    ap.slots = b->slots;
    for (int i = 0; i < nb; i++) {
        ap.q[i] = b->q + (size_t)i * DQ;
        ap.part[i] = b->apart + (size_t)i * b->apart_n;
        ap.out[i] = b->att + (size_t)i * DQ;
    }
    const int Sres = skl_splits(DH, DD);  // slabs the previous layer's w2 left for the residual
    for (int l = 0; l < c.dec_layers; l++) {
        const DecLayerD& L = m->dec[l];
        const DecFragD& F = m->dfrag[l];
        ap.ring_off = (size_t)l * ring_layer;
        // skinny MFMA GEMMs over fragment-major weights: the slots are the 16-column B
        // operand, every weight byte read once per step; each projection leaves split-K slabs
        // in b->part that the next kernel sums (with the residual for wo / w2).
        // residual + RMSNorm as slice-parallel rows: x * w planes + slice sums of squares, the
        // inverse RMS applied by the projection
        CK(launch_resid_xw_fplanes(b->x, nb, DD, L.attn_norm, nullptr, b->xp_d, b->part, l ? Sres : 0, nullptr,
                                   b->ssq, st));
        CK(batch_gemm(b->xp_d, DD, F.wqkv, L.sqkv, DQ + 2 * DKV, nb, b->part, st, b->ssq, DD / 256, c.dec_eps));
        // RoPE + KV append + attention of every live slot, output into the wo planes (one
        // launch; past 256 keys the last key-range block of a kv head merges the partials)
        AttnFuse af;
        af.qkv = b->part; af.S = skl_splits(DD, DQ + 2 * DKV); af.N = DQ + 2 * DKV; af.rope = m->rope_dec; af.xs = b->xp_q;
        CK(launch_attn_batch_fused(hd, ap, af, nb, cap, c.dec_window, scale, H, KVH, splits, st, kv16));
        CK(batch_gemm(b->xp_q, DQ, F.wo, L.so, DD, nb, b->part, st));
        CK(launch_resid_xw_fplanes(b->x, nb, DD, L.ffn_norm, m->ada_scale + (size_t)l * DD, b->xp_d, b->part,
                                   skl_splits(DQ, DD), nullptr, b->ssq, st));
        if (!L.s13) {
            // W1|W3 with the SwiGLU folded in (k_sklx: the last block of each column slice
            // sums its slabs and writes the w2 planes)
            SklFused f;
            f.ssq_in = b->ssq; f.nsl = DD / 256; f.eps = c.dec_eps;
            f.part = b->part; f.ticket = b->ticket;
            f.planes = b->xp_h;
            CK(launch_gemm_sklx(SKX_PRO_SCALE, SKX_EPI_SWIGLU, b->xp_d, DD, F.w13, 2 * DH, nb, f, st));
        } else {
            // Q8: the int8 projection, then the SwiGLU rows
            CK(batch_gemm(b->xp_d, DD, F.w13, L.s13, 2 * DH, nb, b->part, st, b->ssq, DD / 256, c.dec_eps));
            CK(launch_swiglu_fplanes(b->part, skl_splits(DD, 2 * DH), DH, nb, b->xp_h, st));
        }
        CK(batch_gemm(b->xp_h, DH, F.w2, L.s2, DD, nb, b->part, st));
    }
    // final norm (after the last w2 residual) + LM head (tied embeddings) + per-slot argmax,
    // state, token log and next inputs (decoder.c:762-779)
    CK(launch_rmsnorm_fplanes(b->x, nb, DD, m->dec_norm, nullptr, c.dec_eps, b->xp_d, b->part, Sres, st));
    // 17..32 rows: both 16-row blocks in one k_skf launch (the embeddings read once;
    // VOX_HIP_SKF2=0: one launch per 16-row block)
    static int skf2 = -1;
    if (skf2 < 0) {
        const char* e = getenv("VOX_HIP_SKF2");
        skf2 = (e && atoi(e) == 0) ? 0 : 1;
    }
    if (skf2 && nb > SK_ROWS)
        CK(launch_gemm_skf2(b->xp_d, DD, m->lm_frag, m->tok_emb_s, c.vocab, nb, b->logits, c.vocab, st));
    else
        for (int r0 = 0; r0 < nb; r0 += SK_ROWS)
            CK(launch_gemm_skf(b->xp_d + (size_t)r0 * 3 * DD, DD, m->lm_frag, m->tok_emb_s, c.vocab,
                               std::min(SK_ROWS, nb - r0), b->logits + (size_t)r0 * c.vocab, c.vocab, st));
    CK(launch_argmax_batch(b->logits, nb, c.vocab, b->pval, b->pidx, b->palt, b->slots, TOKENS_CAP, slot_toklog(b->slots),
                           m->tok_emb, m->tok_emb_s, DD, b->x, st));
    return 0;
}

// slot bucket of n streams: 1, 2, 4, 8, 16 or 32 slots (graph g of the bucket)
static int slot_bucket(int n, int* g) {
    int k = 0;
    while ((1 << k) < n) k++;
    *g = k;
    return 1 << k;
}

// `steps` batched steps over slots 0..nb-1: replays of the bucket's step graph (captured the
// first time, and again only when the rope table moved), or eager launches
static int batch_run(vox_hip_batch_t* b, int nb, int gb, int gi, int splits, int kv16, int steps) {
    if (!use_graphs()) {
        for (int k = 0; k < steps; k++)
            if (batch_step(b, nb, splits, kv16)) return -1;
        b->n_replays += steps;
        return 0;
    }
    if (b->grope_gen != b->m->rope_gen) {
        batch_drop_graphs(b);
        b->grope_gen = b->m->rope_gen;
    }
    hipGraphExec_t& ge = b->gexec[kv16][gb][gi];
    if (!ge) {
        hipGraph_t g = nullptr;
        CK(hipStreamBeginCapture(b->st, hipStreamCaptureModeThreadLocal));
        const int rc = batch_step(b, nb, splits, kv16);
        hipError_t e = hipStreamEndCapture(b->st, &g);
        if (rc || e != hipSuccess) {
            if (g) hipGraphDestroy(g);
            return set_err("batch graph capture failed: %s", hipGetErrorString(e));
        }
        e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        hipGraphDestroy(g);
        if (e != hipSuccess) {
            ge = nullptr;
            return set_err("batch graph instantiate failed: %s", hipGetErrorString(e));
        }
        b->n_captures++;
    }
    for (int k = 0; k < steps; k++) CK(hipGraphLaunch(ge, b->st));
    b->n_replays += steps;
    return 0;
}

// host mirror after `produced` device steps of stream s (as vox_hip_stream_decode)
static void stream_steps_done(vox_hip_stream_t* s, int produced, int last_token) {
    s->n_generated += produced;
    s->h_state[0] += produced;
    s->h_state[1] += produced;
    if (produced) s->h_state[2] = last_token;
    s->h_state[3] = s->n_generated;
}

// The prompts of several new streams in one stacked prefill pass on the batch queue (the
// decoder prefill of voxtral.c:1036-1057 per stream; rows [b np, (b + 1) np) = stream b):
// RMSNorm and the projections over all rows (every weight byte read once for the group),
// RoPE + K/V append and the causal attention per stream against its own ring (the batched
// encoder's row-offset kernels), scratch of ss[0].  One stream, or 16-bit rings, take the
// single-stream prefill.  The member queues must be idle.
// bounded (vox_hip_batch_decode_rows): a single new stream takes the stacked path too, on the
// batch queue -- its own queue may be busy with an encoder pass the steps overlap; 16-bit rings and
// stacks past ENC_SUB rows still take the per-stream prefill on the member's own queue and
// wait there for any encoder pass queued on it (correct; the overlap is lost for them)
static int batch_prefill(vox_hip_batch_t* b, vox_hip_stream_t* const* ss, int B, bool bounded) {
    vox_hip_model_t* m = b->m;
    const vox_hip_config_t& c = m->c;
    const int np = 32 + m->delay_tokens;
    // more prompts than one pass holds (ENC_SUB rows: 26 prompts of 39 rows): stacked passes of
    // as many as fit
    const int per = std::max(1, ENC_SUB / np);
    if (B > per && !ss[0]->kv16) {
        for (int i0 = 0; i0 < B; i0 += per)
            if (batch_prefill(b, ss + i0, std::min(per, B - i0), bounded)) return -1;
        return 0;
    }
    if ((B == 1 && !bounded) || ss[0]->kv16 || B * np > ENC_SUB) {
        for (int i = 0; i < B; i++) {
            if (stream_prefill(ss[i])) return -1;
            CK(hipStreamSynchronize(ss[i]->st));
        }
        b->n_prefill_passes += B;
        b->n_prefilled += B;
        return 0;
    }
    const int DD = c.dec_dim, H = c.dec_heads, KVH = c.dec_kv_heads, hd = c.dec_head_dim;
    const int DQ = H * hd, DKV = KVH * hd, DH = c.dec_hidden;
    const float scale = 1.0f / sqrtf((float)hd);
    vox_hip_stream_t* lead = ss[0];
    const int N = B * np, cap = lead->dcap;
    hipStream_t st = b->st;
    if (stream_alloc_dec_rows(lead, N)) return -1;
    if (ensure_rope(lead, np + 2)) return -1;
    if (!b->pgws) CK(dalloc(&b->pgws, GEMM_WS_ELEMS));
    float* gws = b->pgws;
    const size_t gws_n = GEMM_WS_ELEMS;
    float* X = lead->xd;
    for (int i = 0; i < B; i++)
        CK(launch_embed_rows(ss[i]->adapter, m->tok_emb, m->tok_emb_s, 0, np, TOKEN_BOS, TOKEN_STREAMING_PAD, DD,
                             X + (size_t)i * np * DD, st));
    EncRows er;
    memset(&er, 0, sizeof er);
    er.B = B;
    for (int i = 0; i < B; i++) {
        er.off[i] = i * np;
        er.nr[i] = np;
        er.pos0[i] = 0;
    }
    if (dec_gemmf_ok(m, N)) {
        if (!b->gflags) CK(dalloc(&b->gflags, gemmf_flag_ints()));
        if (dec_layers_gemmf(lead, GemmfQ{st, gws, gws_n, b->gflags, &b->gepoch}, X, N, [&](int l) -> int {
                for (int i = 0; i < B; i++) {
                    er.Kc[i] = dec_ring(ss[i], ss[i]->dk, l);
                    er.Vc[i] = dec_ring(ss[i], ss[i]->dv, l);
                }
                CK(launch_rope_kv_rows(lead->qkvd, N, DQ, DKV, hd, m->rope_dec, er, lead->qd_, cap, st));
                CK(launch_attn_rows(hd, lead->qd_, er, N, cap, lead->attd, H, KVH, c.dec_window, scale, gws, gws_n, st,
                                    lead->dpa));
                return 0;
            }))
            return -1;
        for (int i = 0; i < B; i++)
            if (stream_prefilled(ss[i], st)) return -1;
        b->n_prefill_passes++;
        b->n_prefilled += B;
        return 0;
    }
    for (int l = 0; l < c.dec_layers; l++) {
        const DecLayerD& L = m->dec[l];
        for (int i = 0; i < B; i++) {
            er.Kc[i] = dec_ring(ss[i], ss[i]->dk, l);
            er.Vc[i] = dec_ring(ss[i], ss[i]->dv, l);
        }
        CK(launch_rmsnorm_rows(X, DD, lead->xnd, DD, L.attn_norm, nullptr, N, DD, c.dec_eps, st));
        CK(launch_gemm(EPI_STORE, 3, lead->xnd, DD, L.wqkv, L.sqkv, DD, N, DQ + 2 * DKV, nullptr, lead->qkvd, DQ + 2 * DKV,
                       st, gws, gws_n));
        CK(launch_rope_kv_rows(lead->qkvd, N, DQ, DKV, hd, m->rope_dec, er, lead->qd_, cap, st));
        CK(launch_attn_rows(hd, lead->qd_, er, N, cap, lead->attd, H, KVH, c.dec_window, scale, gws, gws_n,
                            st));
        CK(launch_gemm(EPI_RESID, 3, lead->attd, DQ, L.wo, L.so, DQ, N, DD, nullptr, X, DD, st, gws, gws_n));
        CK(launch_rmsnorm_rows(X, DD, lead->xnd, DD, L.ffn_norm, m->ada_scale + (size_t)l * DD, N, DD, c.dec_eps, st));
        CK(launch_gemm(EPI_SWIGLU, 3, lead->xnd, DD, L.w13, L.s13, DD, N, 2 * DH, nullptr, lead->gated, DH, st, gws, gws_n));
        CK(launch_gemm(EPI_RESID, 3, lead->gated, DH, L.w2, L.s2, DH, N, DD, nullptr, X, DD, st, gws, gws_n));
    }
    for (int i = 0; i < B; i++)
        if (stream_prefilled(ss[i], st)) return -1;
    b->n_prefill_passes++;
    b->n_prefilled += B;
    return 0;
}

// rows == null: every stream's adapter rows, its queue synchronised first (an async encoder
// pass finishes before the steps read its rows); rows[i]: only stream i's first rows[i] rows,
// which the caller guarantees complete, and the members' queues are left running (an encoder
// pass enqueued on them after those rows overlaps the steps)
// batch_begin enqueues the call's prefills, slot table and first chunk of steps and returns
// without waiting (0: steps in flight, 1: nothing to run); batch_finish waits for them, runs
// the remaining chunks and fills the outputs.  batch_decode = both.
static int batch_begin(vox_hip_batch_t* b, vox_hip_stream_t** streams, int n, const int* rows, int max_steps,
                       int stop_at_eos, int* tokens_out, int* counts_out) {
    if (!b || n < 1 || n > b->cap || max_steps < 0) return set_err("bad batch arguments");
    if (b->call.active) return set_err("batch: a begun call was not finished");
    vox_hip_model_t* m = b->m;
    const vox_hip_config_t& c = m->c;
    const int prompt_len = 1 + 32 + m->delay_tokens;
    for (int i = 0; i < n; i++) {
        if (!streams[i] || streams[i]->m != m) return set_err("batch streams must share the batch's model");
        if (streams[i]->kv16 != streams[0]->kv16)
            return set_err("batch streams must share the decoder KV element type (vox_hip_model_set_kv_fp16)");
        for (int j = 0; j < i; j++)
            if (streams[j] == streams[i]) return set_err("stream listed twice in a batch");
        counts_out[i] = 0;
    }
    const int kv16 = streams[0]->kv16;
    b->n_calls++;
    b->lnb = 0;
    // every member's queue is idle before the batch queue touches its buffers (adapter rows
    // of an async encoder pass, a realloc'ed adapter buffer) -- unless the caller bounded the
    // rows each stream may read
    int avail[VOX_MAX_BATCH];
    for (int i = 0; i < n; i++) {
        if (rows) {
            if (rows[i] < 0 || rows[i] > streams[i]->total_adapter) return set_err("batch rows[%d] out of range", i);
            avail[i] = rows[i];
        } else {
            CK(hipStreamSynchronize(streams[i]->st));
            avail[i] = streams[i]->total_adapter;
        }
    }
    if (max_steps == 0) return 1;
    // 1. streams whose prompt is complete and whose decoder has not started: their prefills
    //    in one stacked pass; they take their first token in the batched steps below
    {
        vox_hip_stream_t* pre[VOX_MAX_BATCH];
        int np = 0;
        for (int i = 0; i < n; i++) {
            vox_hip_stream_t* s = streams[i];
            if (!s->started && !s->eos_seen && avail[i] >= prompt_len) pre[np++] = s;
        }
        if (np && batch_prefill(b, pre, np, rows != nullptr)) return -1;
    }
    // 2. the slot table: slot i = streams[i], a step budget per slot, empty slots up to the
    //    bucket stopped
    int gb = 0;
    const int nb = slot_bucket(n, &gb);
    BatchSlot* hs = b->hslots;
    int K = 0, longest = 0;
    for (int i = 0; i < nb; i++) {
        memset(&hs[i], 0, sizeof hs[i]);
        hs[i].stop_tok = -1;
        if (i >= n) continue;
        vox_hip_stream_t* s = streams[i];
        int lim = 0;
        if (s->started && !s->eos_seen) lim = std::max(0, std::min(avail[i] - s->h_state[1], max_steps));
        hs[i].state = s->state;
        hs[i].tokens = s->tokens;
        hs[i].adapter = s->adapter;
        hs[i].Kc = reinterpret_cast<char*>(s->dk);
        hs[i].Vc = reinterpret_cast<char*>(s->dv);
        hs[i].alts = s->n_alt > 1 ? s->alts : nullptr;
        hs[i].adapter_rows = avail[i];
        hs[i].left = lim;
        hs[i].stop_tok = stop_at_eos ? TOKEN_EOS : -1;
        hs[i].live = lim > 0;
        hs[i].pos = s->h_state[0];
        hs[i].produced = 0;
        if (lim > 0) {
            K = std::max(K, lim);
            longest = std::max(longest, s->h_state[0] + lim);
            if (ensure_rope(s, (long long)s->h_state[0] + lim + 1)) return -1;
        }
    }
    if (K == 0) {
        CK(hipStreamSynchronize(b->st));
        return 1;
    }
    const int gi = graph_index(streams[0], std::min(longest, c.dec_window));
    const int splits = graph_splits(streams[0], gi);
    CK(hipMemcpyAsync(b->slots, hs, sizeof(BatchSlot) * nb, hipMemcpyHostToDevice, b->st));
    CK(launch_embed_batch(b->slots, nb, m->tok_emb, m->tok_emb_s, c.dec_dim, b->x, b->st));
    // 3. the steps, in chunks of STEP_BATCH replays: after each chunk one copy of the slot
    //    table + token log comes back; the call ends when no slot is live.  The first chunk
    //    goes out here, the rest in batch_finish.
    const int k = std::min(STEP_BATCH, K);
    if (batch_run(b, nb, gb, gi, splits, kv16, k)) return -1;
    CK(hipMemcpyAsync(hs, b->slots, SLOT_BYTES, hipMemcpyDeviceToHost, b->st));
    auto& cl = b->call;
    cl.active = 1;
    cl.n = n;
    for (int i = 0; i < n; i++) cl.streams[i] = streams[i];
    cl.max_steps = max_steps;
    cl.stop_at_eos = stop_at_eos;
    cl.K = K;
    cl.nb = nb;
    cl.gb = gb;
    cl.gi = gi;
    cl.splits = splits;
    cl.kv16 = kv16;
    cl.done = 0;
    cl.k = k;
    cl.tokens_out = tokens_out;
    cl.counts_out = counts_out;
    return 0;
}

static int batch_finish(vox_hip_batch_t* b) {
    auto& cl = b->call;
    if (!cl.active) return set_err("batch_finish: no begun call");
    cl.active = 0;
    const int n = cl.n, max_steps = cl.max_steps, K = cl.K;
    vox_hip_stream_t** streams = cl.streams;
    int* tokens_out = cl.tokens_out;
    int* counts_out = cl.counts_out;
    if (K == 0) {
        // a begun call with nothing to run (vox_hip_batch_begin_rows)
        for (int i = 0; i < n; i++) counts_out[i] = 0;
        b->lnb = 0;
        return 0;
    }
    BatchSlot* hs = b->hslots;
    int* htok = slot_toklog(hs);
    int got[VOX_MAX_BATCH] = {0};
    int done = 0, k = cl.k;
    for (;;) {
        // the chunk of k steps in flight (its slot table + token log copy queued behind it)
        CK(hipStreamSynchronize(b->st));
        done += k;
        bool any = false;
        for (int i = 0; i < n; i++) {
            const int p = hs[i].produced;
            for (int j = got[i]; j < p; j++) tokens_out[(size_t)i * max_steps + j] = htok[i * BATCH_TOKLOG + j % BATCH_TOKLOG];
            got[i] = p;
            any = any || hs[i].live;
        }
        if (!any || done >= K) break;
        k = std::min(STEP_BATCH, K - done);
        if (batch_run(b, cl.nb, cl.gb, cl.gi, cl.splits, cl.kv16, k)) return -1;
        CK(hipMemcpyAsync(hs, b->slots, SLOT_BYTES, hipMemcpyDeviceToHost, b->st));
    }
    // 4. host mirrors
    int total = 0;
    const int stop_at_eos = cl.stop_at_eos;
    for (int i = 0; i < n; i++) {
        vox_hip_stream_t* s = streams[i];
        const int p = got[i];
        counts_out[i] = p;
        total += p;
        b->luid[i] = s->uid;
        b->llive[i] = p > 0 && p == done;
        if (!p) continue;
        const int last = tokens_out[(size_t)i * max_steps + p - 1];
        stream_steps_done(s, p, last);
        if (stop_at_eos && last == TOKEN_EOS) s->eos_seen = 1;
    }
    b->lnb = n;
    b->n_rows += total;
    return total;
}

static int batch_decode(vox_hip_batch_t* b, vox_hip_stream_t** streams, int n, const int* rows, int max_steps,
                        int stop_at_eos, int* tokens_out, int* counts_out) {
    const int r = batch_begin(b, streams, n, rows, max_steps, stop_at_eos, tokens_out, counts_out);
    if (r < 0) return -1;
    return r ? 0 : batch_finish(b);
}

extern "C" int vox_hip_batch_decode(vox_hip_batch_t* b, vox_hip_stream_t** streams, int n, int max_steps,
                                    int stop_at_eos, int* tokens_out, int* counts_out) {
    return batch_decode(b, streams, n, nullptr, max_steps, stop_at_eos, tokens_out, counts_out);
}

extern "C" int vox_hip_batch_begin_rows(vox_hip_batch_t* b, vox_hip_stream_t** streams, int n, const int* rows,
                                        int max_steps, int stop_at_eos, int* tokens_out, int* counts_out) {
    if (!rows) return set_err("batch_begin_rows: null rows");
    const int r = batch_begin(b, streams, n, rows, max_steps, stop_at_eos, tokens_out, counts_out);
    if (r < 0) return -1;
    if (r) {
        // nothing to run: an empty call that batch_finish completes
        b->call = {};
        b->call.active = 1;
        b->call.n = n;
        for (int i = 0; i < n; i++) b->call.streams[i] = streams[i];
        b->call.max_steps = max_steps;
        b->call.tokens_out = tokens_out;
        b->call.counts_out = counts_out;
        b->call.K = 0;
        b->call.k = 0;
    }
    return 0;
}

extern "C" int vox_hip_batch_finish(vox_hip_batch_t* b) {
    if (!b) return set_err("batch_finish: null batch");
    return batch_finish(b);
}

extern "C" int vox_hip_batch_decode_rows(vox_hip_batch_t* b, vox_hip_stream_t** streams, int n, const int* rows,
                                         int max_steps, int stop_at_eos, int* tokens_out, int* counts_out) {
    if (!rows) return set_err("batch_decode_rows: null rows");
    return batch_decode(b, streams, n, rows, max_steps, stop_at_eos, tokens_out, counts_out);
}

extern "C" int vox_hip_batch_read_logits(vox_hip_batch_t* b, vox_hip_stream_t* s, float* out) {
    if (!b || !s || !out) return set_err("batch_read_logits: null argument");
    const int V = b->m->c.vocab;
    for (int i = 0; i < b->lnb; i++)
        if (b->luid[i] == s->uid && b->llive[i]) {
            CK(hipMemcpyAsync(out, b->logits + (size_t)i * V, (size_t)V * 4, hipMemcpyDeviceToHost, b->st));
            CK(hipStreamSynchronize(b->st));
            return 0;
        }
    return set_err("batch_read_logits: the stream was not advanced by the last batched step");
}

extern "C" int vox_hip_batch_stats(const vox_hip_batch_t* b, long long* out6) {
    if (!b || !out6) return set_err("batch_stats: null argument");
    out6[0] = b->n_calls;
    out6[1] = b->n_replays;
    out6[2] = b->n_rows;
    out6[3] = b->n_captures;
    out6[4] = b->n_prefill_passes;
    out6[5] = b->n_prefilled;
    return 0;
}
