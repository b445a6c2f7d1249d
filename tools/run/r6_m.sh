# Round 6 call M: where the encoder k_gemmf's cycles go (M = 677 encoder launches only, as
# r6_h.sh): SQ wave-state counters in one pass (8 SQ counters), summarised per projection by
# tools/pmc_gemmf.py
export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
export VOX_HIP_GRAPH=0 VOX_HIP_PREFILL_GEMMF=0
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d /tmp/pmc_sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 1; }
python3 tools/pmc_gemmf.py 677 /tmp/pmc_sq | tee $O/gemmf_sq.txt
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA -d /tmp/pmc_sq2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_sq2.log 2>&1 || { tail -20 $O/pmc_sq2.log; exit 1; }
python3 tools/pmc_gemmf.py 677 /tmp/pmc_sq2 | tee $O/gemmf_sq2.txt
echo rc=0
