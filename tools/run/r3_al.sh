# Round 3 final tree: the config-3 streaming line (60 s at -I 0.5) after the encode_mel split
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu-baseline --streaming --audio-seconds 60 --steps 1 --warmup 1 > gpurun_out/r3al_stream60.json 2> gpurun_out/r3al.err
echo rc=$?
