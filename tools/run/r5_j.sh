# k_gemmf / k_gemmw with XCD-contiguous logical block ids, both unit orders
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmfx timeout -k 10 400 tools/kbench 20 > gpurun_out/r5j_kbench_gemmfx.txt 2>&1 || { tail -20 gpurun_out/r5j_kbench_gemmfx.txt; exit 1; }
echo rc=0
