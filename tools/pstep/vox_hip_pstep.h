// vox_hip_pstep.h -- developer-only persistent decode step (tools/pstep; not in the product
// library: measured slower than the per-operation graph).
#pragma once
#include "../../voxtral.c_amd/csrc/vox_hip_internal.h"

namespace vox {

// Persistent decode step (vox_hip_pstep.hip): every decoder layer of one single-stream step
// in one launch of G workgroups (one per CU).  Per-layer device table:
struct PLayer {
    const uint8_t* w[4];   // QKV [DQ+2DKV][D], wo [D][DQ], W1|W3 [2DH][D] (16-row interleave), W2 [D][DH]; bf16
    const float* attn_norm;
    const float* ffn_norm;
    const float* ada;      // ada_scale row of the layer [D]
    float* Kc;             // this stream's K / V rings of the layer [cap][DKV]
    float* Vc;
};
struct PStepArgs {
    const PLayer* layers;  // device [nl]
    int nl, D, H, KVH, DH, cap, window;
    float eps, scale;
    const int* state;      // state[0] = logical position of the step's token
    const float* rope;     // [pos][hd] (cos, sin)
    float* x;              // [D] step input (in) and final residual (out)
    uint2 *gq, *ga, *gx, *gg;  // hand-off granules {value, tag}: [DQ+2DKV], [DQ], [D], [DH]
    int* ctl;              // [0] launch epoch, [1] arrival count, [2] hand-off timeout flag
    unsigned long long* stamps;  // diagnostics (tools/pstep_dbg): per layer/block timeline, or null
    int flags;                   // diagnostics: 1 = barriers only, no hand-offs (results garbage)
};
bool pstep_ok(int D, int H, int KVH, int hd, int DH, int G);
int pstep_max_keys();
hipError_t launch_pstep(const PStepArgs& a, int G, hipStream_t st);
hipError_t launch_pstep_timed(const PStepArgs& a, int G, hipEvent_t start, hipEvent_t stop, hipStream_t st);

}  // namespace vox
