# A/B on one box: three-wave GEMVs (auto) against four waves everywhere (VOX_HIP_GEMV_NW=4)
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  VOX_HIP_GEMV_NW=4 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4i_nw4_$r.json 2>> gpurun_out/r4i.err || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4i_auto_$r.json 2>> gpurun_out/r4i.err || exit 1
  VOX_HIP_GEMV_NW=4 timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r4i_q8nw4_$r.json 2>> gpurun_out/r4i.err || exit 1
  timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r4i_q8auto_$r.json 2>> gpurun_out/r4i.err || exit 1
done
echo rc=$?
