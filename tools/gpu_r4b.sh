# Chained GEMV launches (two streams, in-kernel wait/arrive) against one stream: tools/kbench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 150 tools/kbench 100 > gpurun_out/r4b_kb.log 2>&1
echo rc=$?
