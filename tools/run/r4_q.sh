# Round 4: served 16 streams with the encoder's k_gemmf on 64-row tiles everywhere
# (VOX_HIP_GEMMF_RB=4: 96 KB LDS ring, room for the batched steps' blocks beside it) vs by shape
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1"
for v in 4 0 4 0 4 0; do VOX_HIP_GEMMF_RB=$v timeout -k 10 300 $B > gpurun_out/r4q_serve16_rb$v.json 2>> gpurun_out/r4q.err || exit 1; echo "rb$v $(cat gpurun_out/r4q_serve16_rb$v.json)" >> gpurun_out/r4q_serve16_ab.txt; done
echo rc=0
