# Round 3: L2 prefetch probe for the decode GEMVs, then every config's bench line and the
# batched step's kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=pf timeout -k 5 120 tools/kbench 200 | grep pf ) > gpurun_out/r3o_pf.log 2>&1 && \
bash tools/run/r3_n.sh
