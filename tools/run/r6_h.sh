# Round 6 call H: the encoder k_gemmf's L2-miss traffic -- C2 bench with
# the decoder prefill off k_gemmf (every k_gemmf launch an M = 677 encoder projection),
# FETCH_SIZE and TCC_HIT_sum / TCC_MISS_sum in separate passes, column-major unit order
# (default) vs row-major (VOX_HIP_GEMMF_ORDER=2); tools/pmc_gemmf.py per projection
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
export VOX_HIP_GRAPH=0 VOX_HIP_PREFILL_GEMMF=0
for ord in 1 2; do
  for pc in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $pc | cut -c1-5)
    VOX_HIP_GEMMF_ORDER=$ord timeout -k 10 300 rocprofv3 --pmc $pc -d /tmp/pmc_${ord}_$tag -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_${ord}_$tag.log 2>&1 || { tail -20 $O/pmc_${ord}_$tag.log; exit 1; }
  done
  echo "== order $ord (1 = column-tile-major, 2 = row-tile-major)"
  python3 tools/pmc_gemmf.py 677 /tmp/pmc_${ord}_FETCH /tmp/pmc_${ord}_TCC_H | tee $O/gemmf_order$ord.txt
done
echo rc=0
