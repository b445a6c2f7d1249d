# Round 4: k_gemmf with 16 waves per block as the default: parity (planes, full-size, scheduler,
# twins) and the C2 line A/B against 8 waves (VOX_HIP_GEMMF_WR=2) on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_gemm_planes.py tests/test_gpu_full.py tests/test_gpu_sched.py tests/test_gpu_twins.py > gpurun_out/r4m_test.log 2>&1 || { tail -40 gpurun_out/r4m_test.log; exit 1; }
for w in 4 2 4 2; do VOX_HIP_GEMMF_WR=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r4m_c2_wr$w.json 2>> gpurun_out/r4m.err || exit 1; echo "wr$w $(cat gpurun_out/r4m_c2_wr$w.json)" >> gpurun_out/r4m_c2_ab.txt; done
for w in 4 2; do VOX_HIP_GEMMF_WR=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --clip-seconds 59.75 --steps 2 --warmup 1 > gpurun_out/r4m_clip59_wr$w.json 2>> gpurun_out/r4m.err || exit 1; done
echo rc=0
