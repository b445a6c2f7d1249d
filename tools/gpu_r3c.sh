export TMPDIR=/tmp
mkdir -p gpurun_out
( echo "== wide"; timeout -k 5 120 tools/kbench 50 | grep -E "^gemm" ; echo "== narrow"; VOX_HIP_GEMM_WIDE=0 timeout -k 5 120 tools/kbench 50 | grep -E "^gemm" ) > gpurun_out/r3c.log 2>&1
echo rc=$?
