# Round 6 call O: where the served C4 loop's idle device time sits (tools/serve_timeline.py
# idle-gap attribution) and the encoder pass's full kernel list, 16 streams, eager trace
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/trn -o run --output-format csv -- python3 bench.py --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 20 --no-cpu-baseline > $O/trn.log 2>&1 || { tail -20 $O/trn.log; exit 1; }
python3 tools/serve_timeline.py $(find /tmp/trn -name "*kernel_trace.csv" | head -1) --top 30 > $O/timeline.txt 2>&1; cat $O/timeline.txt
echo rc=0
