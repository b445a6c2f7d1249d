# Round 3: L2 prefetch probe for the decode GEMVs, batched-attention split A/B (+ its tests),
# every config's bench line and the batched step's kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=pf timeout -k 5 120 tools/kbench 200 | grep pf ) > gpurun_out/r3o_pf.log 2>&1 && \
VOX_HIP_ATT_BSPLIT=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_batch.py "tests/test_gpu_ring.py::test_batch_decode_through_ring_wrap" > gpurun_out/r3o_test_bsplit.log 2>&1 && \
VOX_HIP_ATT_BSPLIT=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r3o_s16_bsplit.json 2> gpurun_out/r3o.err && \
VOX_HIP_ATT_BSPLIT=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 8 > gpurun_out/r3o_s8_bsplit.json 2>> gpurun_out/r3o.err && \
bash tools/run/r3_n.sh
