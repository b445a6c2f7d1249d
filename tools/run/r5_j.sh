# wave-independent decode GEMV prototype against k_gemv (tools/kbench VOX_KB_ONLY=gw)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gw timeout -k 10 240 tools/kbench 100 > gpurun_out/r5j_kbench_gw.txt 2>&1 || { tail -20 gpurun_out/r5j_kbench_gw.txt; exit 1; }
grep -v occupancy gpurun_out/r5j_kbench_gw.txt
echo rc=0
