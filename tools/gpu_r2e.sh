export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 60 tools/pstep_dbg 26 150 0 8 && timeout -k 5 60 tools/pstep_dbg 26 150 0 16 ) > gpurun_out/r2e_dbg.log 2>&1
echo rc=$?
