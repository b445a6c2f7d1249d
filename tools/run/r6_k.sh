# Round 6 call K: where the fused QKV + attention launch loses time.  Graph-replayed C2 decode
# kernel tables for: unfused, fused with the arrival polls 1 / 8 / 32 sleep rounds apart, and
# two diagnostic builds of the wait (1: attention blocks do not wait; 2: and the GEMV blocks
# do not count) -- diagnostics give wrong ids, only their timing is read
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
run() { tag=$1; shift; env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p_$tag -o run --output-format csv -- python3 tools/graph_prof_py.py full > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 tools/kstats.py /tmp/p_$tag/run_kernel_stats.csv > $O/$tag.txt 2>&1; echo "== $tag"; head -6 $O/$tag.txt; }
run unfused VOX_HIP_ATT_FUSE=0
run poll1 VOX_HIP_ATT_POLL=1
run poll8 VOX_HIP_ATT_POLL=8
run poll32 VOX_HIP_ATT_POLL=32
run diag1 VOX_HIP_ATT_DIAG=1
run diag2 VOX_HIP_ATT_DIAG=2
echo rc=0
