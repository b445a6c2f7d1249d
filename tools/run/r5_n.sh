# encoder attention: two query tiles per block / key splits rounded up (kbench)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=attnmf timeout -k 10 300 tools/kbench 50 > gpurun_out/r5n_kbench_attnmf.txt 2>&1 || { tail -20 gpurun_out/r5n_kbench_attnmf.txt; exit 1; }
grep attnmf gpurun_out/r5n_kbench_attnmf.txt
echo rc=0
