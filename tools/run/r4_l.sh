# Round 4: k_gemmf with 16 waves per block (4 row shares) against 8 (kbench)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 50 > gpurun_out/r4l_kb_gemmf.txt 2>&1 || { tail -20 gpurun_out/r4l_kb_gemmf.txt; exit 1; }
echo rc=0
