# wo's weights warmed into L2 beside the decode attention (kbench probe)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=l2pf timeout -k 10 300 tools/kbench 100 > gpurun_out/r5o_kbench_l2pf.txt 2>&1 || { tail -20 gpurun_out/r5o_kbench_l2pf.txt; exit 1; }
grep -E "l2pf|l2 touch|attn L" gpurun_out/r5o_kbench_l2pf.txt
echo rc=0
