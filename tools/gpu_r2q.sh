export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0 1 0; do
VOX_HIP_ENC_FUSED=$v timeout -k 10 300 python -u bench.py --streaming --audio-seconds 20 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2q_stream_$v.json 2>> gpurun_out/r2q.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r2q_stream_$v.json'));print('fused=$v', d['encoder_ms_per_chunk'], d['decoder_ms_per_token'])" >> gpurun_out/r2q.txt
done
for v in 1 0; do
VOX_HIP_ENC_FUSED=$v timeout -k 10 300 python -u bench.py --streams 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2q_s16_$v.json 2>> gpurun_out/r2q.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r2q_s16_$v.json'));print('s16 fused=$v', d['decoder_ms_per_batched_step'])" >> gpurun_out/r2q.txt
done
echo rc=$?
