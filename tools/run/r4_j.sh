# Round 4: served 16 streams with the overlap: encoder projections on k_gemm2 (short-lived
# tiles, VOX_HIP_GEMMF=0) against k_gemmf, and step caps 6 / 7 / 8
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1"
for v in gf0 gf1 cap7 cap6 gf0 gf1 cap7; do
  case $v in gf0) E="VOX_HIP_GEMMF=0"; A="";; gf1) E="VOX_HIP_GEMMF=1"; A="";; cap7) E="VOX_HIP_GEMMF=1"; A="--serve-step-cap 7";; cap6) E="VOX_HIP_GEMMF=1"; A="--serve-step-cap 6";; esac
  env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 $A > gpurun_out/r4j_serve16_$v.json 2>> gpurun_out/r4j.err || exit 1
  echo "$v $(cat gpurun_out/r4j_serve16_$v.json)" >> gpurun_out/r4j_serve16_ab.txt
done
echo rc=0
