export TMPDIR=/tmp
mkdir -p gpurun_out
for b in kbench kbench_g2d1 kbench_g2d2; do echo "== $b"; timeout -k 5 120 tools/$b 50 | grep -E "^gemm enc|^gemm pre" || exit 1; done > gpurun_out/r2z.log 2>&1
echo rc=$?
