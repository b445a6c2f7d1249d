# Round 3: k_gemmf diagnostics -- full kernel, loads + barriers only (no MFMA), MFMA +
# barriers only (no DMA)
export TMPDIR=/tmp VOX_KB_ONLY=gemmf
mkdir -p gpurun_out
( timeout -k 5 120 tools/kbench 100 | grep gemmf ) > gpurun_out/r3e_full.log 2>&1 && \
( timeout -k 5 120 tools/kbench_gfd1 100 | grep gemmf ) > gpurun_out/r3e_nomfma.log 2>&1 && \
( timeout -k 5 120 tools/kbench_gfd2 100 | grep gemmf ) > gpurun_out/r3e_nodma.log 2>&1
echo rc=$?
