/* dlopen() driver for graph_prof_repro built as a shared library (-DREPRO_LIB): the kernels
 * and graphs live in a library loaded at run time, as libvoxtral_hip.so is under ctypes.
 *   rocprofv3 --kernel-trace --stats -d <dir> -- tools/graph_prof_repro_dl <mode> */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>

int main(int argc, char** argv) {
    void* h = dlopen("tools/libgraph_prof_repro.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 1;
    }
    int (*run)(int) = (int (*)(int))dlsym(h, "repro_run");
    if (!run) return 1;
    return run(argc > 1 ? atoi(argv[1]) : 0);
}
