# Round 3: kernel statistics of the served 16-stream line (eager launches); the trace
# database is summarised on the box and removed (it exceeds what gpurun returns)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/r3ak_prof -o serve -- python3 -u bench.py --streams 16 --stagger --steps 1 --warmup 1 --serve-seconds 30 > gpurun_out/r3ak_serve.json 2> gpurun_out/r3ak.err || exit 1
python3 tools/db_stats.py /tmp/r3ak_prof/serve_results.db 40 > gpurun_out/r3ak_stats.txt
echo rc=$?
