# decode GEMV prologue x epilogue combinations (tools/kbench VOX_KB_ONLY=gpe), run twice
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gpe timeout -k 10 200 tools/kbench 100 > gpurun_out/r5l_kbench_gpe.txt 2>&1 || { tail -20 gpurun_out/r5l_kbench_gpe.txt; exit 1; }
VOX_KB_ONLY=gpe timeout -k 10 200 tools/kbench 100 >> gpurun_out/r5l_kbench_gpe.txt 2>&1 || { tail -20 gpurun_out/r5l_kbench_gpe.txt; exit 1; }
grep "^gemv" gpurun_out/r5l_kbench_gpe.txt
echo rc=0
