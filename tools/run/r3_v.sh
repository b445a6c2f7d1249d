# Round 3: decode GEMV grid caps (bf16 and Q8); rocprofv3 graph repro: six graphs on one
# stream, and the kernels + graphs inside a dlopen()ed library
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=grid timeout -k 10 180 tools/kbench 200 > gpurun_out/r3v_grid.txt 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3v_prof4 -o r -- tools/graph_prof_repro 4 > gpurun_out/r3v_prof4.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3v_dl3 -o r -- tools/graph_prof_repro_dl 3 > gpurun_out/r3v_dl3.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3v_dl4 -o r -- tools/graph_prof_repro_dl 4 > gpurun_out/r3v_dl4.log 2>&1
echo rc=$?
