# Round 6 call B: (1) sanity of this round's library changes (tiny, attention incl. the 70-row
# max-split case, batch); (2) served 8-stream A/B: HEAD vs HEAD with 2 planes vs HEAD with the
# k_gemm2 prefill vs round 4's libvoxtral_hip.so (tools/ab/r4, HEAD's host lib and bench.py),
# alternated twice; (3) served 16 / 8 eager kernel traces for the tick decomposition
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_attention.py tests/test_gpu_batch.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
R4=/tmp/r4tree; rm -rf $R4; mkdir -p $R4
cp -r bench.py voxtral.c_amd oracle tests $R4/ && cp tools/ab/r4/libvoxtral_hip.so $R4/voxtral.c_amd/libvoxtral_hip.so
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for r in 1 2; do
  b s8_head_$r --stagger --streams 8 --no-cpu-baseline
  VOX_HIP_GEMM_PLANES=2 b s8_p2_$r --stagger --streams 8 --no-cpu-baseline
  VOX_HIP_PREFILL_GEMMF=0 b s8_pf0_$r --stagger --streams 8 --no-cpu-baseline
  ( cd $R4 && timeout -k 10 300 python -u bench.py --stagger --streams 8 --no-cpu-baseline > /root/repo/$O/s8_r4_$r.json 2> /root/repo/$O/s8_r4_$r.err ) || { tail -20 $O/s8_r4_$r.err; exit 1; }
done
for f in $O/s8_*.json; do python3 -c "import json; d=json.load(open('$f')); bd=d['batched_decode']; print('$f', d['value'], round(bd['ms']/bd['steps'],3), bd['rows_per_step'])"; done
export VOX_HIP_GRAPH=0
b s16_eager --stagger --streams 16 --no-cpu-baseline
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/tr16 -o run --output-format csv -- python3 bench.py --stagger --streams 16 --steps 1 --warmup 0 --no-cpu-baseline > $O/tr16.log 2>&1 || { tail -20 $O/tr16.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/tr8 -o run --output-format csv -- python3 bench.py --stagger --streams 8 --steps 1 --warmup 0 --no-cpu-baseline > $O/tr8.log 2>&1 || { tail -20 $O/tr8.log; exit 1; }
python3 tools/serve_timeline.py $(find $O/tr16 -name "*kernel_trace.csv" | head -1) > $O/timeline16.txt 2>&1; cat $O/timeline16.txt
python3 tools/serve_timeline.py $(find $O/tr8 -name "*kernel_trace.csv" | head -1) > $O/timeline8.txt 2>&1; cat $O/timeline8.txt

VOX_KB_ONLY=sknb timeout -k 10 200 tools/kb_run 100 > $O/kb_sknb.txt 2>&1 || { tail -20 $O/kb_sknb.txt; exit 1; }
cat $O/kb_sknb.txt
echo rc=0
