# Round 4 closing bench lines on the final tree (every config of BASELINE.json), and the
# kernel statistics of the C2 line (eager launches) summarised on the box
export TMPDIR=/tmp
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py"
$B > gpurun_out/r4y_bench.json 2> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --q8 > gpurun_out/r4y_q8.json 2>> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --streams 16 > gpurun_out/r4y_s16.json 2>> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --streams 8 > gpurun_out/r4y_s8.json 2>> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4y_serve16.json 2>> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4y_serve8.json 2>> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --streaming --audio-seconds 60 --steps 1 --warmup 1 > gpurun_out/r4y_stream60.json 2>> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --clip-seconds 59.75 --steps 2 --warmup 1 > gpurun_out/r4y_clip59.json 2>> gpurun_out/r4y.err || exit 1
$B --no-cpu-baseline --long-context 8192 --steps 1 --warmup 1 > gpurun_out/r4y_long8192.json 2>> gpurun_out/r4y.err || exit 1
# the C2 decode path's graph replays under the profiler (full shapes), dispatch gaps included
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r4y_gp -o gp -- python3 -u tools/graph_prof_py.py full > gpurun_out/r4y_gp_full.log 2>&1 || exit 1
python3 tools/db_stats.py /tmp/r4y_gp/gp_results.db 40 gaps > gpurun_out/r4y_graph_replay_stats.txt || exit 1
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r4y_prof -o c2 -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r4y_prof_c2.json 2> gpurun_out/r4y_prof.err || exit 1
python3 tools/db_stats.py /tmp/r4y_prof/c2_results.db 40 > gpurun_out/r4y_c2_kernel_stats.txt || exit 1
# W1|W3 HBM bytes per launch (PMC, separate passes)
bash tools/pmc.sh > gpurun_out/r4y_pmc.log 2>&1 || exit 1
echo rc=0
