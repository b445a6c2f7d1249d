# Round 5 measurements: 16-stream A/B (this tree vs the round-4 library), eager kernel tables of
# the 16-stream step and the -I 0.5 streaming encoder, C2 with the ~70-row flush chunk on k_gemmf
export TMPDIR=/tmp
mkdir -p gpurun_out
export VOX_HIP_GEMM_PLANES=3
R4=build/ab/libvoxtral_hip_r4.so
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r5b_s16_new$k.json 2>gpurun_out/r5b_err.txt || exit 1
  VOX_HIP_LIB=$R4 timeout -k 10 200 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r5b_s16_r4_$k.json 2>gpurun_out/r5b_err.txt || exit 1
done
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5b_prof_s16 -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5b_prof_s16.log 2>&1 || exit 1
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5b_prof_stream -o run --output-format csv -- python3 bench.py --streaming --audio-seconds 30 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5b_prof_stream.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5b_c2_default.json 2>gpurun_out/r5b_err.txt || exit 1
VOX_HIP_ENC_SKINNY_ROWS=64 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5b_c2_sk64.json 2>gpurun_out/r5b_err.txt || exit 1
VOX_HIP_ENC_SKINNY_ROWS=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5b_c2_sk0.json 2>gpurun_out/r5b_err.txt || exit 1
for f in gpurun_out/r5b_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('decoder_ms_per_batched_step'))"; done
find gpurun_out/r5b_prof_s16 gpurun_out/r5b_prof_stream -name "*kernel_stats.csv"
echo rc=0
