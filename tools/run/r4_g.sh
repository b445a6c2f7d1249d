# Round 4: k_gemmf tile shapes (4 column groups per wave: 32 x 64 / 64 x 64 per wave with 8
# waves) and the batched k_skl waves x split sweep (kbench only)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 50 > gpurun_out/r4g_kb_gemmf.txt 2>&1 || { tail -20 gpurun_out/r4g_kb_gemmf.txt; exit 1; }
VOX_KB_ONLY=sklks timeout -k 10 200 tools/kbench 100 > gpurun_out/r4g_kb_sklks.txt 2>&1 || { tail -20 gpurun_out/r4g_kb_sklks.txt; exit 1; }
echo rc=0
