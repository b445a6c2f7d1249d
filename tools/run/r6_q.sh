# Round 6 call Q: what the host does while the device idles in served C4 (16 streams, eager):
# kernel + HIP API traces, tools/serve_gaps.py
export TMPDIR=/tmp
O=gpurun_out/r6q; mkdir -p $O
export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace -d /tmp/trh -o run --output-format csv -- python3 bench.py --stagger --streams 16 --steps 1 --warmup 1 --serve-seconds 20 --no-cpu-baseline > $O/trh.log 2>&1 || { tail -20 $O/trh.log; exit 1; }
python3 tools/serve_gaps.py /tmp/trh --after-setup > $O/gaps.txt 2>&1; cat $O/gaps.txt
echo rc=0
