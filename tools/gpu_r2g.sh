# long-clip / long-stream parity (C2 59.75 s one-shot, C3 60 s -I 0.5), persistent-step parity,
# the long-clip and streaming bench lines, Q8 PMC traffic
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_pstep.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r2g_test.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --clip-seconds 59.75 --steps 1 --warmup 1 > gpurun_out/r2g_clip.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --streaming --audio-seconds 60 --steps 1 --warmup 1 > gpurun_out/r2g_stream.log 2>&1 &&
bash tools/pmc_q8.sh
echo rc=$?
