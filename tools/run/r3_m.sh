# Round 3: long-context decode attention block-size sweep (26 layers' rings)
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=attn timeout -k 5 120 tools/kbench 100 | grep attn ) > gpurun_out/r3m_attn.log 2>&1
echo rc=$?
