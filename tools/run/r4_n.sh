# Round 4: mel feeds through a pinned staging buffer (asynchronous host -> device copies):
# parity (mel, scheduler, tiny, host C), served 16 / 8 streams A/B against the pageable copy
# (VOX_HIP_MEL_PIN=0) on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mel.py tests/test_gpu_sched.py tests/test_gpu_tiny.py tests/test_host_c.py > gpurun_out/r4n_test.log 2>&1 || { tail -40 gpurun_out/r4n_test.log; exit 1; }
for p in 1 0 1 0 1 0; do VOX_HIP_MEL_PIN=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4n_serve16_pin$p.json 2>> gpurun_out/r4n.err || exit 1; echo "pin$p $(cat gpurun_out/r4n_serve16_pin$p.json)" >> gpurun_out/r4n_serve16_ab.txt; done
for p in 1 0; do VOX_HIP_MEL_PIN=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4n_serve8_pin$p.json 2>> gpurun_out/r4n.err || exit 1; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --streaming --audio-seconds 60 --steps 1 --warmup 1 > gpurun_out/r4n_stream60.json 2>> gpurun_out/r4n.err || exit 1
echo rc=0
