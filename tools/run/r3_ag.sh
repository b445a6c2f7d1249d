# Round 3: cross-stream batched encoder pass (vox_hip_stream_encode_mel_batch) -- TINY and
# full-size parity vs the oracle, plus the existing encoder tests on the refactored path
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py "tests/test_gpu_full.py::test_full_jfk_transcription" "tests/test_gpu_full.py::test_full_encode_mel_batch_streaming_chunks" tests/test_gpu_sched.py > gpurun_out/r3ag_test.log 2>&1
echo rc=$?
