# Round 4: served lines on the slot table (step cap, no cap, 8 streams, fp16 KV), the 2-rank
# served rehearsal on one GPU, pre-encoded 16 / 8 streams, eager kernel stats of the served
# line, then the graph-replay profiles (TINY + full shapes; the C2 bench under rocprofv3 last:
# a profiler crash ends the script)
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline"
timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4c_serve16.json 2>> gpurun_out/r4c.err || { tail -20 gpurun_out/r4c.err; exit 1; }
timeout -k 10 300 $B --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4c_serve8.json 2>> gpurun_out/r4c.err || { tail -20 gpurun_out/r4c.err; exit 1; }
timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 --serve-step-cap 0 > gpurun_out/r4c_serve16_nocap.json 2>> gpurun_out/r4c.err || { tail -20 gpurun_out/r4c.err; exit 1; }
timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 --kv-fp16 > gpurun_out/r4c_serve16_kv16.json 2>> gpurun_out/r4c.err || { tail -20 gpurun_out/r4c.err; exit 1; }
VOX_BENCH_SHARE_GPU=1 timeout -k 10 400 $B --gpus 2 --stagger --streams 8 --steps 1 --warmup 1 --serve-seconds 30 > gpurun_out/r4c_gpus2_serve8.json 2> gpurun_out/r4c_gpus2.err || { tail -20 gpurun_out/r4c_gpus2.err; exit 1; }
timeout -k 10 200 $B --streams 16 > gpurun_out/r4c_s16.json 2>> gpurun_out/r4c.err || { tail -20 gpurun_out/r4c.err; exit 1; }
timeout -k 10 200 $B --streams 8 > gpurun_out/r4c_s8.json 2>> gpurun_out/r4c.err || { tail -20 gpurun_out/r4c.err; exit 1; }
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/r4c_prof -o serve -- python3 -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 40 > gpurun_out/r4c_prof_serve16.json 2> gpurun_out/r4c_prof.err || { tail -20 gpurun_out/r4c_prof.err; exit 1; }
python3 tools/db_stats.py /tmp/r4c_prof/serve_results.db 45 > gpurun_out/r4c_serve16_kernel_stats.txt || exit 1
rm -rf /tmp/r4c_prof
for mode in plain batch full; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r4c_gp_$mode -o gp -- python3 -u tools/graph_prof_py.py $mode > gpurun_out/r4c_gp_$mode.log 2>&1 || { echo "graph profile $mode failed rc=$?"; tail -40 gpurun_out/r4c_gp_$mode.log; exit 1; }
  python3 tools/db_stats.py /tmp/r4c_gp_$mode/gp_results.db 40 gaps > gpurun_out/r4c_gp_${mode}_stats.txt || exit 1
done
# the C2 bench itself, graph replays, under the profiler
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r4c_c2 -o c2 -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r4c_c2_graphprof.json 2> gpurun_out/r4c_c2_graphprof.err || { echo "C2 graph profile rc=$?"; tail -30 gpurun_out/r4c_c2_graphprof.err; exit 1; }
python3 tools/db_stats.py /tmp/r4c_c2/c2_results.db 40 gaps > gpurun_out/r4c_c2_graph_kernel_stats.txt || exit 1
echo rc=0
