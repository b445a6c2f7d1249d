# Round 4 (second half of r4_b): batched projections A/B (k_skl vs k_sklp), served lines,
# kernel stats of the served line (eager)
export TMPDIR=/tmp
mkdir -p gpurun_out
for sp in 0 1 0 1; do VOX_HIP_BATCH_SKLP=$sp timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r4b_s16_sklp$sp.json 2>> gpurun_out/r4b.err || exit 1; cat gpurun_out/r4b_s16_sklp$sp.json >> gpurun_out/r4b_s16_sklp_ab.jsonl; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4b_serve16.json 2>> gpurun_out/r4b.err || { tail -20 gpurun_out/r4b.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 --serve-step-cap 0 > gpurun_out/r4b_serve16_nocap.json 2>> gpurun_out/r4b.err || { tail -20 gpurun_out/r4b.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4b_serve8.json 2>> gpurun_out/r4b.err || { tail -20 gpurun_out/r4b.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 --kv-fp16 > gpurun_out/r4b_serve16_kv16.json 2>> gpurun_out/r4b.err || { tail -20 gpurun_out/r4b.err; exit 1; }
VOX_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --gpus 2 --stagger --streams 8 --steps 1 --warmup 1 --serve-seconds 30 > gpurun_out/r4c_gpus2_serve8.json 2> gpurun_out/r4c_gpus2.err || { tail -20 gpurun_out/r4c_gpus2.err; exit 1; }
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/r4b_prof -o serve -- python3 -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 40 > gpurun_out/r4b_prof_serve16.json 2> gpurun_out/r4b_prof.err || { tail -20 gpurun_out/r4b_prof.err; exit 1; }
python3 tools/db_stats.py /tmp/r4b_prof/serve_results.db 45 > gpurun_out/r4b_serve16_kernel_stats.txt
echo rc_stats=$?
echo rc=0
