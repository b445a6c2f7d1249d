# batched decode (16 / 8 pre-encoded streams) with the f32 KV and with the 16-bit KV (the
# reference's VOX_DECODER_KV_FP16), alternating on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5n_$n.json 2> gpurun_out/r5n_err.txt || { tail -20 gpurun_out/r5n_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5n_$n.json')); print('$n', d['value'], d.get('decoder_ms_per_batched_step'), d.get('kv_dtype'))"; }
for r in 1 2; do
b s16_f32_$r --streams 16 --no-cpu-baseline
b s16_kv16_$r --streams 16 --kv-fp16 --no-cpu-baseline
done
b s8_f32 --streams 8 --no-cpu-baseline
b s8_kv16 --streams 8 --kv-fp16 --no-cpu-baseline
echo rc=0
