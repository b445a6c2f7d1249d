# k_gemmf unit order A/B (row-tile-major vs column-tile-major), np3 and np2, M = 70 / 677 / 1024
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 20 > gpurun_out/r5d_kbench_gemmf.txt 2>&1 || { tail -20 gpurun_out/r5d_kbench_gemmf.txt; exit 1; }
grep gemmf gpurun_out/r5d_kbench_gemmf.txt
echo rc=0
