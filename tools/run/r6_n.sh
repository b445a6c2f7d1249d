# Round 6 call N: k_gemmf with one barrier per PAIR of 64-deep stages on a 4-slot ring
# (gf_stages_pair) against one per stage on 3 slots.  tools/kbench VOX_KB_ONLY=pair (bits
# compared), the gemmf parity tests, then C2 alternated VOX_HIP_GEMMF_PAIR=0 / 1 on one box
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
VOX_KB_ONLY=pair timeout -k 10 300 tools/kb_run 100 > $O/kb_pair.txt 2>&1 || { tail -20 $O/kb_pair.txt; exit 1; }
grep -E "^pair" $O/kb_pair.txt
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm_planes.py tests/test_gpu_full.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
for i in 1 2; do
  for r in 0 1; do
    VOX_HIP_GEMMF_PAIR=$r timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_p${r}_$i.json 2> $O/c2_p${r}_$i.err || { tail -20 $O/c2_p${r}_$i.err; exit 1; }
  done
done
for f in $O/c2_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d.get('encoder_rtf'), d.get('encoder_rtf_2plane'), d.get('encoder_roofline', {}).get('frac'))"; done
echo rc=0
