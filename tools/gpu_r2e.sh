export TMPDIR=/tmp
mkdir -p gpurun_out
( for d in 8 16; do timeout -k 5 60 tools/pstep_dbg 26 150 0 $d || exit 1; done ) > gpurun_out/r2e_dbg.log 2>&1
echo rc=$?
