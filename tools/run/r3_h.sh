# Round 3: k_gemmf tile shape / stream-K split sweep
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=gemmf timeout -k 5 200 tools/kbench 100 | grep gemmf ) > gpurun_out/r3h_sweep.log 2>&1
echo rc=$?
