export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0; do
VOX_HIP_ENC_FUSED=$v VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2r_prof$v -o run --output-format csv -- python3 bench.py --streaming --audio-seconds 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2r_$v.json 2>> gpurun_out/r2r.err || exit 1
done
echo rc=$?
