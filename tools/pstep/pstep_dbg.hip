// pstep_dbg.hip -- developer check of the persistent decode step (k_pstep) against the
// per-operation kernels, stage by stage (QKV+RoPE, attention, gate, residual x), and a
// timing of both.  Build: make -C tools pstep_dbg; run: tools/pstep_dbg [layers] [pos]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#include "vox_hip_pstep.h"

using namespace vox;
namespace vox { extern int g_pstep_d; }

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s (line %d)\n", #x, hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static uint32_t rs = 12345;
static float frand() { rs = rs * 1664525u + 1013904223u; return ((rs >> 8) & 0xffff) / 65536.0f - 0.5f; }
static uint16_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }

template <class T>
static T* up(const std::vector<T>& v) {
    T* p;
    CK(hipMalloc(&p, v.size() * sizeof(T)));
    CK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}
static std::vector<float> down(const float* p, size_t n) {
    std::vector<float> v(n);
    CK(hipMemcpy(v.data(), p, n * 4, hipMemcpyDeviceToHost));
    return v;
}
static double maxdiff(const std::vector<float>& a, const std::vector<float>& b, double* mag) {
    double d = 0, m = 0;
    for (size_t i = 0; i < a.size(); i++) {
        d = fmax(d, fabs((double)a[i] - b[i]));
        m = fmax(m, fabs((double)b[i]));
    }
    if (mag) *mag = m;
    return d;
}

int main(int argc, char** argv) {
    const int NL = argc > 1 ? atoi(argv[1]) : 1;
    const int LP = argc > 2 ? atoi(argv[2]) : 100;
    const int small = argc > 3 ? atoi(argv[3]) : 0;
    g_pstep_d = argc > 4 ? atoi(argv[4]) : 0;
    printf("ring depth knob %d\n", g_pstep_d);
    const int D = small ? 256 : 3072, H = small ? 4 : 32, KVH = small ? 2 : 8, HD = 128, DH = small ? 512 : 9216;
    const int DQ = H * HD, DKV = KVH * HD, NQKV = DQ + 2 * DKV, WIN = small ? 48 : 8192, CAP = WIN + 64;
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    printf("D %d H %d KVH %d DH %d layers %d pos %d CUs %d pstep_ok %d\n", D, H, KVH, DH, NL, LP, cus,
           (int)pstep_ok(D, H, KVH, HD, DH, cus));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    auto wmat = [&](size_t rows, size_t K, float sc) {
        std::vector<uint16_t> w(rows * K);
        for (auto& x : w) x = bf(frand() * sc);
        return up(w);
    };
    auto fvec = [&](size_t n, float base, float sc) {
        std::vector<float> v(n);
        for (auto& x : v) x = base + frand() * sc;
        return v;
    };
    std::vector<PLayer> tab(NL), tab2(NL);
    std::vector<float*> K1(NL), V1(NL), K2(NL), V2(NL);
    for (int l = 0; l < NL; l++) {
        tab[l].w[0] = (const uint8_t*)wmat(NQKV, D, 0.08f);
        tab[l].w[1] = (const uint8_t*)wmat(D, DQ, 0.05f);
        tab[l].w[2] = (const uint8_t*)wmat(2 * DH, D, 0.08f);
        tab[l].w[3] = (const uint8_t*)wmat(D, DH, 0.03f);
        tab[l].attn_norm = up(fvec(D, 1.0f, 0.2f));
        tab[l].ffn_norm = up(fvec(D, 1.0f, 0.2f));
        tab[l].ada = up(fvec(D, 0.0f, 0.2f));
        std::vector<float> kv = fvec((size_t)CAP * DKV, 0.f, 2.f);
        K1[l] = up(kv); K2[l] = up(kv);
        kv = fvec((size_t)CAP * DKV, 0.f, 2.f);
        V1[l] = up(kv); V2[l] = up(kv);
        tab2[l] = tab[l];
        tab[l].Kc = K2[l]; tab[l].Vc = V2[l];
    }
    std::vector<float> rope((size_t)(LP + 8) * HD);
    for (int p = 0; p < LP + 8; p++)
        for (int i = 0; i < HD / 2; i++) {
            const double f = p / pow(1e6, 2.0 * i / HD);
            rope[(size_t)p * HD + 2 * i] = (float)cos(f);
            rope[(size_t)p * HD + 2 * i + 1] = (float)sin(f);
        }
    float* drope = up(rope);
    std::vector<float> x0 = fvec(D, 0.f, 2.f);
    float* x1 = up(x0);
    float* x2 = up(x0);
    int st4[4] = {LP, 0, 0, 0};
    int* state = up(std::vector<int>(st4, st4 + 4));
    float *q, *att, *gate, *part;
    CK(hipMalloc(&q, DQ * 4));
    CK(hipMalloc(&att, DQ * 4));
    CK(hipMalloc(&gate, DH * 4));
    CK(hipMalloc(&part, (size_t)H * 256 * (HD + 2) * 4));
    // reference: the per-operation kernels
    auto ref_layer = [&](int l, float* x) {
        GemvArgs a;
        memset(&a, 0, sizeof a);
        a.x = x; a.K = D; a.W = tab2[l].w[0]; a.rows = NQKV; a.norm_w = tab2[l].attn_norm; a.eps = 1e-5f; a.y = q;
        a.qd = DQ; a.kvd = DKV; a.hd = HD; a.state = state; a.rope = drope; a.Kc = K1[l]; a.Vc = V1[l]; a.cap = CAP;
        CK(launch_gemv(PRO_NORM, EPI_QKV, a, st));
        const int splits = (std::min(LP + 1, WIN) + 255) / 256;
        int sp = 1;
        while (sp < splits) sp *= 2;
        CK(launch_attn_decode(HD, q, K1[l], V1[l], CAP, state, 0, WIN, 1.0f / sqrtf((float)HD), H, KVH, part, att, sp, st));
        memset(&a, 0, sizeof a);
        a.x = att; a.K = DQ; a.W = tab2[l].w[1]; a.rows = D; a.y = x;
        CK(launch_gemv(PRO_NONE, EPI_RESID, a, st));
        memset(&a, 0, sizeof a);
        a.x = x; a.K = D; a.W = tab2[l].w[2]; a.rows = 2 * DH; a.norm_w = tab2[l].ffn_norm; a.ada = tab2[l].ada; a.eps = 1e-5f;
        a.y = gate;
        CK(launch_gemv(PRO_NORM_ADA, EPI_SWIGLU, a, st));
        memset(&a, 0, sizeof a);
        a.x = gate; a.K = DH; a.W = tab2[l].w[3]; a.rows = D; a.y = x;
        CK(launch_gemv(PRO_NONE, EPI_RESID, a, st));
    };
    for (int l = 0; l < NL; l++) ref_layer(l, x1);
    CK(hipStreamSynchronize(st));
    // persistent
    PLayer* dtab = up(tab);
    uint2* gran;
    const size_t ng = (size_t)NQKV + DQ + D + DH;
    CK(hipMalloc(&gran, ng * 8));
    CK(hipMemset(gran, 0, ng * 8));
    int* ctl;
    CK(hipMalloc(&ctl, 16));
    CK(hipMemset(ctl, 0, 16));
    PStepArgs pa;
    memset(&pa, 0, sizeof pa);
    pa.layers = dtab; pa.nl = NL; pa.D = D; pa.H = H; pa.KVH = KVH; pa.DH = DH; pa.cap = CAP; pa.window = WIN;
    pa.eps = 1e-5f; pa.scale = 1.0f / sqrtf((float)HD); pa.state = state; pa.rope = drope; pa.x = x2;
    pa.gq = gran; pa.ga = gran + NQKV; pa.gx = pa.ga + DQ; pa.gg = pa.gx + D; pa.ctl = ctl;
    CK(launch_pstep(pa, cus, st));
    CK(hipStreamSynchronize(st));
    int hctl[4];
    CK(hipMemcpy(hctl, ctl, 16, hipMemcpyDeviceToHost));
    printf("ctl: epoch %d arrivals %d err %d\n", hctl[0], hctl[1], hctl[2]);
    // granules of the last layer vs the reference buffers
    std::vector<uint2> g(ng);
    CK(hipMemcpy(g.data(), gran, ng * 8, hipMemcpyDeviceToHost));
    auto gv = [&](size_t off, size_t n) {
        std::vector<float> v(n);
        for (size_t i = 0; i < n; i++) memcpy(&v[i], &g[off + i].x, 4);
        return v;
    };
    unsigned tag_bad = 0;
    for (size_t i = 0; i < (size_t)NQKV + DQ + DH; i++) {
        const size_t gi = i < (size_t)NQKV + DQ ? i : i + D;
        if ((g[gi].y & 0xff) == 0) tag_bad++;
    }
    printf("granules with tag 0: %u\n", tag_bad);
    double mag;
    const int slot = LP % CAP;
    std::vector<float> rq = down(q, DQ), pq = gv(0, DQ);
    printf("q (layer %d)       maxdiff %.3e (|ref| %.3e)\n", NL - 1, maxdiff(pq, rq, &mag), mag);
    std::vector<float> rk = down(K1[NL - 1] + (size_t)slot * DKV, DKV), pk = down(K2[NL - 1] + (size_t)slot * DKV, DKV);
    printf("k new (cache)     maxdiff %.3e (|ref| %.3e)\n", maxdiff(pk, rk, &mag), mag);
    printf("k new (granules)  maxdiff %.3e\n", maxdiff(gv(DQ, DKV), rk, &mag));
    std::vector<float> rv = down(V1[NL - 1] + (size_t)slot * DKV, DKV), pv = down(V2[NL - 1] + (size_t)slot * DKV, DKV);
    printf("v new (cache)     maxdiff %.3e (|ref| %.3e)\n", maxdiff(pv, rv, &mag), mag);
    std::vector<float> ra = down(att, DQ), pat = gv(NQKV, DQ);
    printf("attention out     maxdiff %.3e (|ref| %.3e)\n", maxdiff(pat, ra, &mag), mag);
    std::vector<float> rg = down(gate, DH), pg = gv((size_t)NQKV + DQ + D, DH);
    printf("gate              maxdiff %.3e (|ref| %.3e)\n", maxdiff(pg, rg, &mag), mag);
    std::vector<float> rx = down(x1, D), px = down(x2, D);
    printf("x out             maxdiff %.3e (|ref| %.3e)\n", maxdiff(px, rx, &mag), mag);
    {
        // per-phase timeline of one launch (tid 0 of every block, s_memrealtime 10 ns ticks)
        unsigned long long* stamps;
        const size_t nst = (size_t)NL * cus * 16;
        CK(hipMalloc(&stamps, nst * 8));
        CK(hipMemset(stamps, 0, nst * 8));
        PStepArgs pb = pa;
        pb.stamps = stamps;
        CK(launch_pstep(pb, cus, st));
        CK(hipStreamSynchronize(st));
        std::vector<unsigned long long> h(nst);
        CK(hipMemcpy(h.data(), stamps, nst * 8, hipMemcpyDeviceToHost));
        const char* names[10] = {"QKV stream", "QKV epi + q", "attention", "merge + att gather", "wo stream",
                                 "wo epi + x gather", "W13 stream", "W13 epi + gate", "W2 stream", "W2 epi + x gather"};
        double sum_med[10] = {0}, sum_max[10] = {0};
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int l = 0; l < NL; l++)
            for (int k = 0; k < 10; k++) {
                if (k == 9 && l + 1 == NL) continue;
                std::vector<double> d;
                for (int bb = 0; bb < cus; bb++) {
                    const unsigned long long* r = &h[((size_t)l * cus + bb) * 16];
                    const unsigned long long e = k < 9 ? r[k + 1] : h[((size_t)(l + 1) * cus + bb) * 16];
                    d.push_back((double)(e - r[k]) * 0.01);
                    t0 = std::min(t0, r[0]);
                    t1 = std::max(t1, r[9]);
                }
                std::sort(d.begin(), d.end());
                sum_med[k] += d[d.size() / 2];
                sum_max[k] += d.back();
            }
        printf("timeline per layer (median / max over blocks, us):\n");
        double tm = 0;
        for (int k = 0; k < 10; k++) {
            printf("  %-20s %7.2f %7.2f\n", names[k], sum_med[k] / NL, sum_max[k] / NL);
            tm += sum_med[k] / NL;
        }
        printf("  sum of medians %.2f us per layer; layer 0 QKV start -> last W2 stream end %.2f us\n", tm, (t1 - t0) * 0.01);
        // each hand-off: the producers' spread (last block's stream end - median block's) and the
        // latency after the LAST producer (median block's operand-ready time - last stream end)
        {
            const int pe[4] = {1, 5, 7, 9}, pr[4] = {4, 6, 8, 0};
            const char* en[4] = {"QKV -> wo (attention)", "wo -> W13", "W13 -> W2", "W2 -> next QKV"};
            for (int e = 0; e < 4; e++) {
                double sk = 0, la = 0;
                int n = 0;
                for (int l = 0; l < NL; l++) {
                    if (e == 3 && l + 1 == NL) continue;
                    std::vector<double> te, tr;
                    for (int bb = 0; bb < cus; bb++) {
                        te.push_back((double)h[((size_t)l * cus + bb) * 16 + pe[e]]);
                        tr.push_back((double)h[((size_t)(e == 3 ? l + 1 : l) * cus + bb) * 16 + pr[e]]);
                    }
                    std::sort(te.begin(), te.end());
                    std::sort(tr.begin(), tr.end());
                    sk += (te.back() - te[te.size() / 2]) * 0.01;
                    la += (tr[tr.size() / 2] - te.back()) * 0.01;
                    n++;
                }
                printf("  edge %-22s producer spread %5.2f us, after last producer %5.2f us\n", en[e], sk / n, la / n);
            }
        }
        // streamer wave 0 in the W1|W3 phase: 13 = released after the wo boundary, 10 = first slot
        // consumed, 11 = first slot of local row 3, 12 = last slot consumed (W1|W3 end)
        double dA = 0, dB = 0, dC = 0;
        int nn = 0;
        for (int l = 0; l < NL; l++)
            for (int bb = 0; bb < cus; bb++) {
                const unsigned long long* r = &h[((size_t)l * cus + bb) * 16];
                if (!r[13] || !r[10] || !r[11] || !r[12]) continue;
                dA += (double)(r[10] - r[13]) * 0.01;
                dB += (double)(r[11] - r[10]) * 0.01;
                dC += (double)(r[12] - r[11]) * 0.01;
                nn++;
            }
        if (nn) printf("  streamer W13: release -> 1st slot %.2f, 1st slot -> row 3 (9 slots) %.2f, row 3 -> end (45 slots) %.2f us\n",
                       dA / nn, dB / nn, dC / nn);
    }
    {
        // the weight stream alone: barriers only, no hand-offs (results garbage)
        PStepArgs pb = pa;
        pb.flags = 1;
        hipEvent_t f0, f1;
        CK(hipEventCreate(&f0));
        CK(hipEventCreate(&f1));
        CK(launch_pstep(pb, cus, st));
        CK(hipEventRecord(f0, st));
        for (int i = 0; i < 10; i++) CK(launch_pstep(pb, cus, st));
        CK(hipEventRecord(f1, st));
        CK(hipEventSynchronize(f1));
        float fm;
        CK(hipEventElapsedTime(&fm, f0, f1));
        const double lb = 2.0 * ((double)NQKV * D + (double)D * DQ + 2.0 * DH * D + (double)D * DH);
        printf("stream only (no hand-offs): %.2f us per layer, %.0f GB/s\n", fm * 100 / NL, lb * NL / (fm * 1e-4) / 1e9);
        pb.flags = 2;  // consume the first ring contents over and over: no weight traffic
        CK(launch_pstep(pb, cus, st));
        CK(hipEventRecord(f0, st));
        for (int i = 0; i < 10; i++) CK(launch_pstep(pb, cus, st));
        CK(hipEventRecord(f1, st));
        CK(hipEventSynchronize(f1));
        CK(hipEventElapsedTime(&fm, f0, f1));
        printf("consume only (no loads, no hand-offs): %.2f us per layer (%.0f GB/s equivalent)\n", fm * 100 / NL,
               lb * NL / (fm * 1e-4) / 1e9);
        for (int T : {100, 300, 500, 800}) {  // every hand-off replaced by a fixed wait of T x 10 ns
            pb.flags = 4 | (T << 8);
            CK(launch_pstep(pb, cus, st));
            CK(hipEventRecord(f0, st));
            for (int i = 0; i < 10; i++) CK(launch_pstep(pb, cus, st));
            CK(hipEventRecord(f1, st));
            CK(hipEventSynchronize(f1));
            CK(hipEventElapsedTime(&fm, f0, f1));
            printf("stream + 4 fixed %.1f us waits per layer: %.2f us per layer (stream + waits = %.2f)\n", T * 0.01,
                   fm * 100 / NL, 0.0);
        }
    }
    // timing (repeat launches; the inputs drift, values do not matter here)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int it = 20;
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < it; i++) CK(launch_pstep(pa, cus, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double lbytes = 2.0 * ((double)NQKV * D + (double)D * DQ + 2.0 * DH * D + (double)D * DH);
    printf("pstep:   %.2f us per launch, %.2f us per layer, %.0f GB/s\n", ms * 1000 / it, ms * 1000 / it / NL,
           lbytes * NL / (ms * 1e-3 / it) / 1e9);
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < it; i++)
        for (int l = 0; l < NL; l++) ref_layer(l, x1);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("per-op:  %.2f us per step, %.2f us per layer, %.0f GB/s\n", ms * 1000 / it, ms * 1000 / it / NL,
           lbytes * NL / (ms * 1e-3 / it) / 1e9);
    CK(hipMemcpy(hctl, ctl, 16, hipMemcpyDeviceToHost));
    printf("ctl after timing: epoch %d arrivals %d err %d\n", hctl[0], hctl[1], hctl[2]);
    return 0;
}
