# Round 4: served 16 streams with the overlap, the encoder's stream-K grid at 256 (one block
# per CU, default) / 192 / 128 blocks (VOX_HIP_GEMMF_BLOCKS) so the batched steps keep CUs
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline"
for g in 0 128 192 0 128 192; do VOX_HIP_GEMMF_BLOCKS=$g timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4i_serve16_g$g.json 2>> gpurun_out/r4i.err || exit 1; echo "g$g $(cat gpurun_out/r4i_serve16_g$g.json)" >> gpurun_out/r4i_serve16_ab.txt; done
echo rc=0
