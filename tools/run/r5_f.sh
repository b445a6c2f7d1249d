# k_sklx waves per block / 64-k blocks per split for the -I 0.5 encoder chain (VOX_HIP_SKLX_NW,
# VOX_HIP_SKLX_KS): parity under the two forced settings, then C3 (60 s) per setting, and a
# kernel trace of each (20 s) for the per-projection times
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "4 4" "8 8"; do set -- $cfg
VOX_HIP_SKLX_NW=$1 VOX_HIP_SKLX_KS=$2 timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_tiny.py -k "encode_chunks or streaming" > gpurun_out/r5f_test_$1$2.log 2>&1 || { tail -30 gpurun_out/r5f_test_$1$2.log; exit 1; }
tail -1 gpurun_out/r5f_test_$1$2.log
done
for cfg in "0 0" "4 4" "4 8" "8 4" "8 8"; do set -- $cfg
VOX_HIP_SKLX_NW=$1 VOX_HIP_SKLX_KS=$2 timeout -k 10 300 python -u bench.py --streaming --audio-seconds 60 --no-cpu-baseline > gpurun_out/r5f_stream60_$1$2.json 2> gpurun_out/r5f_err.txt || { tail -20 gpurun_out/r5f_err.txt; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5f_stream60_$1$2.json')); print('nw $1 ks $2', d['value'], d.get('encoder_ms_per_chunk'))"
VOX_HIP_SKLX_NW=$1 VOX_HIP_SKLX_KS=$2 VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r5f_prof_$1$2 -o run -- python3 bench.py --streaming --audio-seconds 20 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5f_prof_$1$2.log 2>&1 || { tail -20 gpurun_out/r5f_prof_$1$2.log; exit 1; }
done
echo rc=0
