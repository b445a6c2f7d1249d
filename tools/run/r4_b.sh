# Round 4: dynamic row-group claims in the decode GEMVs (A/B, kbench + bench), step-capped
# serving A/B, kernel stats of the served line (eager) and a graph-replay profile attempt
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_sched.py tests/test_gpu_q8.py tests/test_gpu_full.py::test_full_jfk_transcription > gpurun_out/r4b_test.log 2>&1 || { tail -40 gpurun_out/r4b_test.log; exit 1; }
VOX_KB_ONLY=drain timeout -k 10 120 tools/kbench 100 > gpurun_out/r4b_kb_drain.txt 2>&1 || { tail -20 gpurun_out/r4b_kb_drain.txt; exit 1; }
VOX_KB_ONLY=gemmf timeout -k 10 200 tools/kbench 50 > gpurun_out/r4b_kb_gemmf.txt 2>&1 || { tail -20 gpurun_out/r4b_kb_gemmf.txt; exit 1; }
VOX_KB_ONLY=attb timeout -k 10 200 tools/kbench 100 > gpurun_out/r4b_kb_attb.txt 2>&1 || { tail -20 gpurun_out/r4b_kb_attb.txt; exit 1; }
VOX_HIP_BATCH_SKLP=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py -k "not full_size" > gpurun_out/r4b_test_sklp.log 2>&1 || { tail -40 gpurun_out/r4b_test_sklp.log; exit 1; }
VOX_KB_ONLY=sklp timeout -k 10 120 tools/kbench 100 > gpurun_out/r4b_kb_sklp.txt 2>&1 || { tail -20 gpurun_out/r4b_kb_sklp.txt; exit 1; }
for d in 0 1 0 1; do VOX_HIP_GEMV_DRAIN=$d timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r4b_c2_d$d.json 2>> gpurun_out/r4b.err || exit 1; cat gpurun_out/r4b_c2_d$d.json >> gpurun_out/r4b_c2_ab.jsonl; done
for d in 0 1; do VOX_HIP_GEMV_DRAIN=$d timeout -k 10 200 python -u bench.py --no-cpu-baseline --q8 --steps 10 --warmup 2 > gpurun_out/r4b_q8_d$d.json 2>> gpurun_out/r4b.err || exit 1; done
# rocprofv3 on graph replays: which replay survives the profiler
for mode in plain batch prof; do
  VOX_GP_MAPS=gpurun_out/r4b_gp_maps_$mode.txt timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r4b_gp_$mode -o gp -- python3 -u tools/graph_prof_py.py $mode > gpurun_out/r4b_gp_$mode.log 2>&1 || { echo "graph profile $mode failed rc=$?"; tail -40 gpurun_out/r4b_gp_$mode.log; exit 1; }
  find /tmp/r4b_gp_$mode -name "*kernel_stats.csv" -exec cp {} gpurun_out/r4b_gp_${mode}_kernel_stats.csv \;
done
echo rc=0
