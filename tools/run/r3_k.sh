# Round 3: long-context decode attention over 26 layers' rings (f32 / half), kernel split
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=attn timeout -k 5 120 tools/kbench 100 | grep attn ) > gpurun_out/r3k_attn.log 2>&1 && \
VOX_KB_ONLY=attn timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k_prof -o r3k -- tools/kbench 100 > gpurun_out/r3k_prof.log 2>&1
echo rc=$?
