# Round 4: where the served tick's wall goes outside the scheduler run (feed / run / collect
# split; a cProfile of the same command)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4o_serve16.json 2>> gpurun_out/r4o.err || exit 1
timeout -k 10 400 python -u -m cProfile -o /tmp/r4o.prof bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4o_serve16_cprof.json 2>> gpurun_out/r4o.err || exit 1
python3 -c "import pstats; pstats.Stats('/tmp/r4o.prof').sort_stats('tottime').print_stats(30)" > gpurun_out/r4o_cprofile.txt || exit 1
echo rc=0
