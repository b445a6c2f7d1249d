# Round 4: served streams reused per slot through vh_stream_reset (default) against a fresh
# vh_stream per clip (--serve-fresh-streams): parity (scheduler incl. the reuse test, mel,
# tiny), served 16 / 8 streams A/B on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sched.py tests/test_gpu_mel.py tests/test_gpu_tiny.py > gpurun_out/r4p_test.log 2>&1 || { tail -40 gpurun_out/r4p_test.log; exit 1; }
B="python -u bench.py --no-cpu-baseline --stagger --steps 1 --warmup 1"
for v in reuse fresh reuse fresh reuse fresh; do A=""; [ $v = fresh ] && A="--serve-fresh-streams"; timeout -k 10 300 $B --streams 16 $A > gpurun_out/r4p_serve16_$v.json 2>> gpurun_out/r4p.err || exit 1; echo "$v $(cat gpurun_out/r4p_serve16_$v.json)" >> gpurun_out/r4p_serve16_ab.txt; done
for v in reuse fresh; do A=""; [ $v = fresh ] && A="--serve-fresh-streams"; timeout -k 10 300 $B --streams 8 $A > gpurun_out/r4p_serve8_$v.json 2>> gpurun_out/r4p.err || exit 1; done
echo rc=0
