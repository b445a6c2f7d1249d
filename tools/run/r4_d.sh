# Round 4: batched adapter in the cross-stream encoder pass (tests + served lines, the
# common-end workload and the per-stream one), batched attention phase stamps, and the
# rocprofv3 crash hunt (full-shape profiled decode with maps; the C2 bench with maps last)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_sched.py tests/test_gpu_batch.py tests/test_gpu_full.py::test_full_encode_mel_batch_streaming_chunks > gpurun_out/r4d_test.log 2>&1 || { tail -40 gpurun_out/r4d_test.log; exit 1; }
VOX_KB_ONLY=attb timeout -k 10 200 tools/kbench 100 > gpurun_out/r4d_kb_attb.txt 2>&1 || { tail -20 gpurun_out/r4d_kb_attb.txt; exit 1; }
B="python -u bench.py --no-cpu-baseline"
timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4d_serve16.json 2>> gpurun_out/r4d.err || { tail -20 gpurun_out/r4d.err; exit 1; }
timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 --serve-end per-stream > gpurun_out/r4d_serve16_perstream.json 2>> gpurun_out/r4d.err || { tail -20 gpurun_out/r4d.err; exit 1; }
timeout -k 10 300 $B --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4d_serve8.json 2>> gpurun_out/r4d.err || { tail -20 gpurun_out/r4d.err; exit 1; }
VOX_GP_MAPS=gpurun_out/r4d_gp_maps_fullprof.txt timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r4d_gp -o gp -- python3 -u tools/graph_prof_py.py fullprof > gpurun_out/r4d_gp_fullprof.log 2>&1 || { echo "fullprof rc=$?"; grep -v "^W2026" gpurun_out/r4d_gp_fullprof.log | tail -40; exit 1; }
VOX_BENCH_MAPS=gpurun_out/r4d_c2_maps.txt timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r4d_c2 -o c2 -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r4d_c2_graphprof.json 2> gpurun_out/r4d_c2_graphprof.err || { echo "C2 graph profile rc=$?"; grep -v "^W2026" gpurun_out/r4d_c2_graphprof.err | tail -30; exit 1; }
echo rc=0
