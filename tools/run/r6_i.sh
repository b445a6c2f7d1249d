# Round 6 call I: k_gemmf XCD rounds (VOX_HIP_GEMMF_ORDER=3: an XCD's blocks on their own
# column tiles, the row tiles in rounds) against the default unit order, encoder and stacked-
# prefill shapes (tools/kbench VOX_KB_ONLY=gemmfx, tools/kb_run = a copy of tools/kbench)
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
VOX_KB_ONLY=gemmfx timeout -k 10 300 tools/kb_run 100 > $O/kb_gemmfx.txt 2>&1 || { tail -20 $O/kb_gemmfx.txt; exit 1; }
grep -E "^gemmfx" $O/kb_gemmfx.txt
echo rc=0
