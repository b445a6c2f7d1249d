# Round 6 call F: k_skl2 (both 16-row blocks of a 32-row batch in one block, weights shared)
# against k_skl's two-block grid, every decode shape (tools/kbench VOX_KB_ONLY=sknb)
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
VOX_KB_ONLY=sknb timeout -k 10 200 tools/kb_run 100 > $O/kb_sknb.txt 2>&1 || { tail -20 $O/kb_sknb.txt; exit 1; }
grep -E "^skl|^skf" $O/kb_sknb.txt
echo rc=0
