# Round 4: the scheduler's encoder pass left running when the run returns (default) vs
# completed inside the run (VOX_HIP_SCHED_OVERLAP=2): parity, served 16 / 8 streams A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sched.py > gpurun_out/r4k_test.log 2>&1 || { tail -40 gpurun_out/r4k_test.log; exit 1; }
for ov in 1 2 1 2 1 2; do VOX_HIP_SCHED_OVERLAP=$ov timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4k_serve16_ov$ov.json 2>> gpurun_out/r4k.err || exit 1; echo "ov$ov $(cat gpurun_out/r4k_serve16_ov$ov.json)" >> gpurun_out/r4k_serve16_ab.txt; done
for ov in 1 2; do VOX_HIP_SCHED_OVERLAP=$ov timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4k_serve8_ov$ov.json 2>> gpurun_out/r4k.err || exit 1; done
echo rc=0
