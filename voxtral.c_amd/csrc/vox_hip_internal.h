// vox_hip_internal.h -- kernel launch interface shared by the engine and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vox {

enum { EPI_STORE = 0, EPI_RESID = 1, EPI_GELU = 2, EPI_GELU_ERF = 3, EPI_SWIGLU = 4, EPI_QKV = 5, EPI_LOGITS = 6,
       EPI_LOGITS_ALT = 7,
       EPI_PARTIAL = 8,      // split-K GEMM slice: raw f32 tile into a workspace, epilogue in k_splitk_reduce
       EPI_QKV_BIAS = 9 };   // EPI_QKV with the projection's bias added before RoPE (the encoder's)
constexpr int ALT_TEXT_MIN = 1000;   // TOKEN_TEXT_MIN (voxtral.c:399)
constexpr int ALT_PART = 10;         // per-block alt partial: m, s, 4 values, 4 ids
constexpr int ALT_REC = 8;           // per-step alt record: p_best, (id, p) x 3, pad
enum { PRO_NONE = 0, PRO_NORM = 1, PRO_NORM_ADA = 2 };

constexpr int GEMV_MAX_BLOCKS = 1024;  // 4 blocks of 256 threads per CU on 256 CUs

struct GemvArgs {
    const float* x;        // input vector [K] (device)
    int K;
    const void* W;         // bf16 [rows, K], or int8 [rows, K] when wscale is set
    const float* wscale;   // Q8 per-row scales (null: bf16 weights)
    int rows;              // output rows streamed (2*hidden for SWIGLU)
    const float* norm_w;   // PRO_NORM*: RMSNorm weight [K]
    const float* ada;      // PRO_NORM_ADA: ada_scale row [K]
    float eps;
    float* y;              // output
    const float* bias;     // optional bias (STORE / RESID)
    // EPI_QKV
    int qd, kvd, hd;
    const float* rope;     // rope table [pos][hd]
    const int* state;      // device state (state[0] = logical position) or null
    int pos;               // logical position when state == null
    float* Kc;             // decoder ring (f32, or IEEE half when kv16)
    float* Vc;
    int cap;
    int kv16 = 0;
    // EPI_LOGITS(_ALT)
    float* part_val;
    int* part_idx;
    float* part_alt;       // EPI_LOGITS_ALT: [blocks][ALT_PART]
};

constexpr int VOX_MAX_BATCH = 32;    // streams per batched decode step (two 16-row blocks of the MFMA B operand)

// One row of a batched decode step, in device memory (the batch's slot table).  The step
// graph's kernel arguments point at the table, never at a stream, so streams join and leave
// a batch without a graph capture: the host rewrites the table before a call, the step's
// last kernel (k_argmax_batch_final) advances it, and a slot whose `live` is 0 costs no
// attention, KV append, argmax or state change (its row still rides through the GEMMs).
struct BatchSlot {
    int* state;             // the stream's {kv logical pos, next adapter row, prev token, step}
    int* tokens;            // the stream's token ring (tokens_cap entries)
    const float* adapter;   // the stream's adapter rows
    char* Kc;               // layer-0 base of the stream's decoder K / V rings (bytes)
    char* Vc;
    float* alts;            // stream_fill_alts records (null: no alternatives for this slot)
    int adapter_rows;       // rows the slot may consume (the stream's adapter count at the call)
    int left;               // steps the slot may still take in this call
    int stop_tok;           // the slot stops after emitting this id (TOKEN_EOS, or -1)
    int live;               // the current step runs for this slot
    int pos;                // state[0] mirror: the attention starts without the state hop
    int produced;           // steps taken in this call (index into the batch's token log)
};
static_assert(sizeof(BatchSlot) == 72, "BatchSlot layout");
constexpr int BATCH_TOKLOG = 64;     // per-slot token log entries (>= the steps between reads)

// per-stream operands of one decode-attention launch (blockIdx.z = stream of a batch)
struct AttnPtrs {
    const float* q[VOX_MAX_BATCH];
    const float* Kc[VOX_MAX_BATCH];
    const float* Vc[VOX_MAX_BATCH];
    const int* state[VOX_MAX_BATCH];
    float* part[VOX_MAX_BATCH];
    float* out[VOX_MAX_BATCH];
    // batched step: Kc / Vc / position / liveness from the slot table (layer base + ring_off)
    const BatchSlot* slots = nullptr;
    size_t ring_off = 0;
};
// Kc / Vc of the decoder rings point at f32 elements, or at IEEE half ones in the 16-bit
// mode (the kv16 argument of the launchers, VOX_DECODER_KV_FP16)

// batched decode attention with the QKV epilogue folded in (k_attn_decode<.., FUSE = 1>):
// RoPE of q / k and the KV append read the QKV projection's split-K slabs, and the output
// goes straight into the wo input planes
struct AttnFuse {
    const float* qkv;      // [S][16][N] slabs, row z = stream z of the batch
    int S, N;              // slab count, row length (H*hd + 2*KVH*hd)
    const float* rope;     // [pos][hd] (cos, sin) table
    uint16_t* xs;          // [3][16][H*hd] fragment-major planes of the attention output
};

constexpr int ARGB = 64;                // argmax partial blocks per row

int gemv_grid(int rows);
bool gemv_ok(int rows, int K, int q8);  // shapes launch_gemv accepts (rows, K multiple of the chunk)
int attn_maxch(int window);      // decode-attention partials per head (64-key blocks)
int attn_maxsplits(int window);  // 256-key spans of a window (graph buckets)
hipError_t launch_rmsnorm_rows(const float* x, int ldx, float* y, int ldy, const float* w,
                               const float* ada, int M, int D, float eps, hipStream_t st);
// ws: f32 workspace for split-K partials (ws_elems floats; nullptr = no split)
hipError_t launch_gemm(int epi, int nsplit, const float* A, int lda, const void* W,
                       const float* wscale, int K, int M, int N, const float* bias, float* C,
                       int ldc, hipStream_t st, float* ws = nullptr, size_t ws_elems = 0);
hipError_t launch_rope_kv(const float* qkv, int M, int qd, int kvd, int hd, const float* rope,
                          int pos0, float* q, float* Kc, float* Vc, int cap, hipStream_t st, int kv16 = 0);
hipError_t launch_attn_rows_mf(int hd, const float* Q, int ldq, const float* Kc, const float* Vc,
                             int cap, float* O, int ldo, int M, int H, int KVH, int q_pos0,
                             int k_first, int window, float scale, hipStream_t st, float* ws = nullptr,
                             size_t ws_elems = 0, uint16_t* xs = nullptr, int kv16 = 0);
// xs: the output also (or only, through the combine kernel) as fragment-major planes
// the skinny encoder's QKV slabs (+ bias) -> RoPE'd q rows and the K/V ring slots (one pass)
hipError_t launch_slabs_rope_kv(const float* part, int S, int M, const float* bias, int qd, int kvd, int hd,
                                const float* rope, int pos0, float* q, float* Kc, float* Vc, int cap, hipStream_t st);
hipError_t launch_gemv(int pro, int epi, const GemvArgs& a, hipStream_t st);
const void* gemv_kernel(int pro, int epi, const GemvArgs& a);
hipError_t launch_gemv_timed(int pro, int epi, const GemvArgs& a, hipEvent_t start, hipEvent_t stop,
                             hipStream_t st);
int gemv_occupancy(const void* fn);
// part: H * attn_maxch(window) * (hd + 2) floats of partials, then KVH ints (zeroed before
// the first launch) that count the split blocks' arrivals
hipError_t launch_attn_decode(int hd, const float* q, const float* Kc, const float* Vc, int cap,
                              const int* state, int pos_host, int window, float scale, int H,
                              int KVH, float* part, float* out, int splits, hipStream_t st, int kv16 = 0);
// the same over nb streams at once (device state positions; pointers per stream)
hipError_t launch_attn_decode_batch(int hd, const AttnPtrs& p, int nb, int cap, int window, float scale,
                                    int H, int KVH, int splits, hipStream_t st, int kv16 = 0);
constexpr int ATT_BLOCK_KEYS = 256;  // keys one decode-attention block covers
// the batched step's attention: RoPE + KV append from the QKV slabs, output as planes
// (one block per stream x kv head x 256-key split; splits > 1 adds the combine kernel)
hipError_t launch_attn_batch_fused(int hd, const AttnPtrs& p, const AttnFuse& f, int nb, int cap, int window,
                                   float scale, int H, int KVH, int splits, hipStream_t st, int kv16 = 0);

// a batched encoder pass: rows [off[b], off[b] + nr[b]) of the stacked rows belong to stream
// b, at logical positions pos0[b] + i, with its own K/V ring (layer base)
struct EncRows {
    int B;
    int off[VOX_MAX_BATCH], nr[VOX_MAX_BATCH], pos0[VOX_MAX_BATCH];
    float* Kc[VOX_MAX_BATCH];
    float* Vc[VOX_MAX_BATCH];
};
// RoPE + K/V append of every stacked row into its stream's ring (k_rope_kv per row block)
hipError_t launch_rope_kv_rows(const float* qkv, int N, int qd, int kvd, int hd, const float* rope_table,
                               const EncRows& er, float* q, int cap, hipStream_t st);
// windowed attention of every stream's rows against its own ring, one launch (+ one combine):
// Q / O stacked [N, H*hd]
hipError_t launch_attn_rows(int hd, const float* Q, const EncRows& er, int N, int cap, float* O, int H, int KVH,
                            int window, float scale, float* ws, size_t ws_elems, hipStream_t st, uint16_t* xs = nullptr);
constexpr int STEP_GRAPHS = 8;       // step graphs by attention split count 1, 2, 4, ..., 128
hipError_t launch_attn_batch_dbg(const AttnPtrs& p, const AttnFuse& f, int nb, int cap, int window, float scale, int H,
                                 int KVH, int splits, hipStream_t st);
hipError_t launch_attn_dbg(int dbg, const float* q, const float* Kc, const float* Vc, int cap,
                           const int* state, float* part, float* out, hipStream_t st);
hipError_t launch_embed_step(const float* adapter, const void* emb, const float* esc, const int* state,
                             int D, float* x, hipStream_t st);
hipError_t launch_embed_rows(const float* adapter, const void* emb, const float* esc, int row0, int n,
                             int first_tok, int rest_tok, int D, float* x, hipStream_t st);
hipError_t launch_argmax_final(const float* pv, const int* pi, int n, int* state, int* tokens,
                               int cap, const float* adapter, int adapter_rows,
                               const void* emb, const float* esc, int D, float* x,
                               const float* part_alt, float* alts, hipStream_t st);
// batched step: x_i = adapter_i[state[1]] + tok_emb[state[2]] for every live slot, 0 otherwise
hipError_t launch_embed_batch(const BatchSlot* slots, int nb, const void* emb, const float* esc, int D, float* x,
                              hipStream_t st);
// batched step's end: per live slot the first-max argmax of its logits row, the token into the
// stream's ring and toklog[slot][produced % BATCH_TOKLOG], the stream state and the slot
// advanced (the slot stops at stop_tok, after `left` steps or at its last adapter row), the
// next input row (0 for a slot that stopped); slots with alts also get the step's
// stream_fill_alts record (palt: [nb][ARGB][ALT_PART] scratch)
hipError_t launch_argmax_batch(const float* logits, int nb, int V, float* pval, int* pidx, float* palt,
                               BatchSlot* slots, int tokens_cap, int* toklog, const void* emb, const float* esc, int D,
                               float* x, hipStream_t st);
// Batched decode GEMMs for M <= 16 rows held as three bf16 planes xs[3][16][K] (hi/mid/lo =
// the exact f32 rows) in MFMA fragment order; weights packed by launch_frag_pack.
// tools/kbench sweep knobs: variables in a kbench build (-DVOX_KBENCH), compile-time constants
// (the product's own choice) in the library
#ifdef VOX_KBENCH
#define VOX_KB_KNOB(name, v) int name = v
#else
#define VOX_KB_KNOB(name, v) constexpr int name = v
#endif
constexpr int SK_ROWS = 16;
constexpr int SK_MAX_ROWS = 96;  // rows of one skinny launch: up to 6 row blocks of 16
                                 // (planes [rb][3][16][K], slabs [rb][S][16][N])
constexpr int PLANE_MAX_ROWS = 1024;  // rows of a planes buffer (one encoder pass, ENC_SUB)
hipError_t launch_frag_pack(const void* src, int N, int K, int q8, void* dst, hipStream_t st);
// RMSNorm (+ ada) of nb rows into planes; S > 0: x += the S split slabs of part first
hipError_t launch_rmsnorm_fplanes(float* x, int nb, int D, const float* w, const float* ada, float eps,
                                  uint16_t* xs, const float* part, int S, hipStream_t st, const float* bias = nullptr);
// x[j] += the S slabs of row j (+ bias); out[j] = the S slabs of row j (+ bias)
hipError_t launch_resid_slabs(float* x, int nb, int D, const float* part, int S, const float* bias, hipStream_t st);
hipError_t launch_slabs_rows(const float* part, int S, int nb, int N, const float* bias, float* out, int ldo,
                             hipStream_t st);
hipError_t launch_split_fplanes(const float* x, int nb, int K, uint16_t* xs, hipStream_t st);
// silu(W1 x) * (W3 x) from the split W1|W3 slabs (N = 2H rows) into planes
hipError_t launch_swiglu_fplanes(const float* part, int S, int H, int nb, uint16_t* xs, hipStream_t st);
// C[j][n] = sum_k x_j[k] W[n][k] (LM head: k_skf)
hipError_t launch_gemm_skf(const uint16_t* xs, int K, const void* Wf, const float* wscale, int N, int nb, float* C,
                           int ldc, hipStream_t st);
// launch_gemm_skf for 17..32 rows (two 16-row blocks of planes, one weight read)
hipError_t launch_gemm_skf2(const uint16_t* xs, int K, const void* Wf, const float* wscale, int N, int nb, float* C,
                            int ldc, hipStream_t st);
// split-K slabs part[s][16][N], s < skl_splits(K, N) (projections: k_skl; k_sklx and the
// encoder's skinny chain use skl_splits(K))
int skl_splits(int K, int N = 0);
// ssq: RMSNorm applied to the results (planes from launch_resid_xw_fplanes, nsl slices per row)
constexpr int SKL_MAX_SLICES = 12;  // D <= 3072
// pair: 17..32 rows through k_skl2 (both row blocks in one block; same bits) where its
// configuration exists (the batched step)
hipError_t launch_gemm_skl(const uint16_t* xs, int K, const void* Wf, const float* wscale, int N, int nb,
                           float* part, hipStream_t st, const float* ssq = nullptr, int nsl = 0, float eps = 0.f,
                           int pair = 0);
hipError_t launch_gemm_skl_cfg(int nw, int ks, const uint16_t* xs, int K, const void* Wf, int N, int nb, float* part,
                               hipStream_t st);  // tools/kbench sweep
hipError_t launch_gemm_skl2_cfg(int nw, int ks, const uint16_t* xs, int K, const void* Wf, int N, int nb, float* part,
                                hipStream_t st);  // tools/kbench sweep: 17..32 rows, weights shared by both row blocks
// x += the S slabs (+ bias); planes of x * w (* (1 + ada)); the row's sums of squares per
// 256-column slice to ssq[row / 16][D / 256][row % 16] (the inverse RMS is applied by
// launch_gemm_skl)
hipError_t launch_resid_xw_fplanes(float* x, int nb, int D, const float* w, const float* ada, uint16_t* xs,
                                   const float* part, int S, const float* bias, float* ssq, hipStream_t st);
// k_sklx: k_skl with the neighbouring row kernels folded in (bf16 weights).  Inputs are
// always planes; SKX_PRO_SCALE planes hold x * w (* (1 + ada)) of an RMSNorm whose inverse RMS
// is applied to the MFMA results, computed from the row sums of squares that the producer left
// per column slice (ssq_in[rb][nsl][16], summed in slice order).  Epilogue: the slabs go out
// write-through and one ticket per (row block, column slice) counts them; the block that
// completes a slice sums its S slabs in split order (as psum) and finishes it: SKX_EPI_QKV =
// bias + RoPE + K/V ring append (k_slabs_rope_kv), SKX_EPI_RESID = x += slabs + bias, the
// slice's row sums of squares to ssq_out[rb][X][16] and (planes != null) the next
// projection's planes x * nw (* (1 + ada)), SKX_EPI_SWIGLU = silu(W1) * W3 into the next
// projection's planes (k_swiglu_fplanes).
enum { SKX_PRO_PLANES = 0, SKX_PRO_SCALE = 1 };
enum { SKX_EPI_QKV = 1, SKX_EPI_RESID = 2, SKX_EPI_SWIGLU = 3 };
struct SklFused {
    const float* ssq_in = nullptr;
    int nsl = 0;
    float eps = 0.f;
    float* part = nullptr;
    int* ticket = nullptr;  // zeroed once; every finishing block resets its own
    const float* bias = nullptr;
    float* x = nullptr;
    float* ssq_out = nullptr;
    uint16_t* planes = nullptr;
    const float* nw = nullptr;   // SKX_EPI_RESID planes: the next RMSNorm's weight (and ada)
    const float* ada = nullptr;
    const float* rope = nullptr;  // row of position pos0
    int qd = 0, kvd = 0, hd = 0, pos0 = 0, cap = 0;
    float* q = nullptr;
    float* Kc = nullptr;
    float* Vc = nullptr;
};
// column slices of a k_sklx launch (the ssq_out slices its consumer sums)
int sklx_slices(int N, int K);
constexpr int SKX_TICKETS = 4 * 1024;
hipError_t launch_gemm_sklx(int pro, int epi, const uint16_t* xs, int K, const void* Wf, int N, int nb,
                            const SklFused& f, hipStream_t st);
// k_gemmf (vox_hip_gemmf.hip): stream-K MFMA GEMM, planes x fragment-major bf16 weights;
// epi in {STORE, RESID, GELU, GELU_ERF, SWIGLU}; SWIGLU with xo writes the gate rows as
// planes [rb][3][16][N / 2].  ws: gemmf_ws_floats(gemmf_grid()) floats of partial tiles,
// flags: gemmf_grid() ints (zeroed once), epoch: > 0, new for every launch on the stream.
bool gemmf_ok(int M, int N, int K);
int gemmf_grid();
size_t gemmf_flag_ints();      // flags buffer: gemmf_grid() flags, then the recompute counter
int set_gemmf_wait(int ticks); // owner's wait per partial in 100 MHz ticks (< 0: always recompute); returns the old
size_t gemmf_ws_floats(int blocks);
hipError_t launch_gemmf(int epi, int np, const uint16_t* xs, int K, int M, const void* Wf, int N, const float* bias,
                        float* C, int ldc, uint16_t* xo, float* ws, size_t ws_floats, int* flags, int epoch,
                        hipStream_t st);
int gemm_planes_np();  // activation planes of the M > 1 GEMMs (2, or 3 with VOX_HIP_GEMM_PLANES=3)
int set_gemm_planes(int np);  // 2 or 3 (vox_hip_set_gemm_planes); -1 otherwise
hipError_t launch_im2col3(const float* src, int C, int T, int stride, int off, float* A,
                          hipStream_t st);
hipError_t launch_mel_tail(const float* melp, int n_new, int MB, float* tail, hipStream_t st);
// device log-mel (vox_hip_mel_*): nframes frames from samples[start0 + 160 f ..]; tables
// transposed: dcosT / dsinT [400][201], filtT [201][128]
hipError_t launch_mel_frames(const float* samples, long long start0, int nframes, const float* window,
                             const float* dcosT, const float* dsinT, const float* filtT, float log_min, float* mel,
                             hipStream_t st);
hipError_t launch_mel_reflect(float* buf, long long n, long long real_end, int len, hipStream_t st);

}  // namespace vox
