# k_gemmf tile order with XCD groups (order 3) vs auto / column / row (kbench)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 20 > gpurun_out/r5r_kbench_gemmf_xcdgrp.txt 2>&1 || { tail -20 gpurun_out/r5r_kbench_gemmf_xcdgrp.txt; exit 1; }
echo rc=0
