// Reproduction attempts for the rocprofv3 --kernel-trace crash on graph replays.
// mode 0: 2 trivial kernel nodes; 1: 131 nodes (a decode step's count); 2: 2 nodes whose
// kernel argument is an 832-byte struct (the batched attention's AttnPtrs + AttnFuse);
// 3: 131 nodes with 192-byte arguments (GemvArgs-sized); 4: six graphs of 131 nodes captured
// on one stream and replayed alternately (the decode step's split buckets).  Each graph is
// launched 10 times.  5: mode 3's graph, replayed after (and between) eager launches that
// carry dispatch-recorded events (hipExtLaunchKernel with start / stop), as the profiled
// decode batches interleave them.
//   rocprofv3 --kernel-trace --stats -d <dir> -- tools/graph_prof_repro <mode>
// Built with -DREPRO_LIB the same code is a shared library (repro_run) that
// graph_prof_repro_dl.c dlopen()s, as Python's ctypes loads libvoxtral_hip.so.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

struct Big { float* x; float v; int pad[206]; };   // 832 bytes
struct Mid { float* x; float v; int pad[44]; };    // 192 bytes

__global__ void k_add(float* x, float v) { x[threadIdx.x] += v; }
__global__ void k_add_big(const Big b) { b.x[threadIdx.x] += b.v + (float)b.pad[threadIdx.x & 127]; }
__global__ void k_add_mid(const Mid m) { m.x[threadIdx.x] += m.v + (float)m.pad[threadIdx.x & 31]; }

#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("%s: %s\n", #e, hipGetErrorString(r)); return 1; } } while (0)

#ifdef REPRO_LIB
extern "C" int repro_run(int mode) {
#else
int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
#endif
    const int nodes = (mode == 1 || mode == 3 || mode == 4 || mode == 5) ? 131 : 2;
    const int ngraphs = mode == 4 ? 6 : 1;
    float* x;
    CK(hipMalloc(&x, 256 * 4));
    CK(hipMemset(x, 0, 256 * 4));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipGraph_t g;
    hipGraphExec_t ges[6];
    Big b = {};
    Mid m = {};
    b.x = m.x = x;
    b.v = m.v = 1.0f;
    for (int gi = 0; gi < ngraphs; gi++) {
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < nodes; i++) {
            if (mode == 2) hipLaunchKernelGGL(k_add_big, dim3(1), dim3(256), 0, st, b);
            else if (mode >= 3) hipLaunchKernelGGL(k_add_mid, dim3(1), dim3(256), 0, st, m);
            else hipLaunchKernelGGL(k_add, dim3(1), dim3(256), 0, st, x, 1.0f);
        }
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ges[gi], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int extra = 0;
    for (int i = 0; i < 10 * ngraphs; i++) {
        CK(hipGraphLaunch(ges[i % ngraphs], st));
        if (mode == 5) {
            Mid mm = m;
            void* kargs[] = {&mm};
            CK(hipExtLaunchKernel(reinterpret_cast<const void*>(&k_add_mid), dim3(1), dim3(256), kargs, 0, st, e0, e1, 0));
            extra++;
        }
    }
    if (mode == 5) {
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
    }
    CK(hipStreamSynchronize(st));
    float h[1];
    CK(hipMemcpy(h, x, 4, hipMemcpyDeviceToHost));
    printf("mode %d: %d nodes x 10 replays ok: x[0] = %.1f (expected %.1f)\n", mode, nodes, h[0], 10.0f * nodes * ngraphs + extra);
    return 0;
}
