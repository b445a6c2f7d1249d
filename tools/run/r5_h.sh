# the cost of a launch boundary between dependent weight streams (tools/kbench VOX_KB_ONLY=bar)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=bar timeout -k 10 180 tools/kbench 100 > gpurun_out/r5h_kbench_bar.txt 2>&1 || { tail -20 gpurun_out/r5h_kbench_bar.txt; exit 1; }
cat gpurun_out/r5h_kbench_bar.txt | grep -v occupancy
echo rc=0
