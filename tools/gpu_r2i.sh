export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 60 tools/pstep_dbg 26 150 0 16 | grep -vE "maxdiff" ) > gpurun_out/r2i_dbg.log 2>&1
echo rc=$?
