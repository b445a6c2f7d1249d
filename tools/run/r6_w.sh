# Round 6 call W (r6_r again, table loads batched 40 / 67 ahead): k_mel_frames with 1 / 2 / 4 / 8 frames per block (tools/kbench VOX_KB_ONLY=mel,
# bits compared), then the mel parity tests on the library's default (4)
export TMPDIR=/tmp
O=gpurun_out/r6w; mkdir -p $O
VOX_KB_ONLY=mel timeout -k 10 200 tools/kb_run 100 > $O/kb_mel.txt 2>&1 || { tail -20 $O/kb_mel.txt; exit 1; }
grep -E "^mel" $O/kb_mel.txt
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_mel.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
echo rc=0
