# decode GEMV grids with >= 3 groups per block (wo / W2: 768 -> 512 blocks) A/B, alternating on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5m_c2_base$k.json 2> gpurun_out/r5m_err.txt || { tail -20 gpurun_out/r5m_err.txt; exit 1; }
  VOX_HIP_GEMV_MIN_GROUPS=3 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5m_c2_mg3_$k.json 2> gpurun_out/r5m_err.txt || { tail -20 gpurun_out/r5m_err.txt; exit 1; }
done
VOX_HIP_GEMV_MIN_GROUPS=3 timeout -k 10 200 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r5m_q8_mg3.json 2> gpurun_out/r5m_err.txt || { tail -20 gpurun_out/r5m_err.txt; exit 1; }
timeout -k 10 200 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r5m_q8_base.json 2> gpurun_out/r5m_err.txt || { tail -20 gpurun_out/r5m_err.txt; exit 1; }
for f in gpurun_out/r5m_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('decoder_ms_per_token'))"; done
echo rc=0
