# Round 6 call L: k_gemmf with a 4-slot LDS ring (3 stages in flight) against 3 slots -- the
# encoder GEMM's fetch is latency-bound.  tools/kbench VOX_KB_ONLY=ring (both
# rings, bits compared), the gemmf parity tests, then C2 / C2 two-plane / C3 stream alternated
# VOX_HIP_GEMMF_RING=3 / 4 on one box (tools/kb_run = a copy of tools/kbench)
export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
VOX_KB_ONLY=ring timeout -k 10 300 tools/kb_run 100 > $O/kb_ring.txt 2>&1 || { tail -20 $O/kb_ring.txt; exit 1; }
grep -E "^ring" $O/kb_ring.txt
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm_planes.py tests/test_gpu_full.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
for i in 1 2; do
  for r in 3 4; do
    VOX_HIP_GEMMF_RING=$r timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_r${r}_$i.json 2> $O/c2_r${r}_$i.err || { tail -20 $O/c2_r${r}_$i.err; exit 1; }
  done
done
for r in 3 4; do
  VOX_HIP_GEMMF_RING=$r timeout -k 10 300 python -u bench.py --clip-seconds 59.75 --no-cpu-baseline > $O/clip_r$r.json 2> $O/clip_r$r.err || { tail -20 $O/clip_r$r.err; exit 1; }
done
for f in $O/c2_*.json $O/clip_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d.get('encoder_rtf'), d.get('encoder_rtf_2plane'), d.get('encoder_roofline', {}).get('frac'))"; done
echo rc=0
