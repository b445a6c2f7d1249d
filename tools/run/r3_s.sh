# Round 3: rocprofv3 + hipGraph reproduction attempts, one profiler run per mode
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 2 3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3s_prof$m -o r -- tools/graph_prof_repro $m > gpurun_out/r3s_prof$m.log 2>&1 || { echo "mode $m rc=$?"; exit 1; }
done
echo rc=0
