#!/bin/bash
# Round-4: host API trace of the storm bench (where the refresh's host time goes)
A="--steps 8 --warmup 5 --no-cpu --spot 0 --trajectory 0"
mkdir -p gpurun_out/s23
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s23/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/gpurun_out/s23/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/s23/err.log
rc=$?
echo "rc=$rc"
cd $GRAFT_REPO_ROOT
for f in $(find gpurun_out/s23/prof -name "*.csv"); do gzip -c $f > gpurun_out/s23/$(basename $f).gz; done
rm -rf gpurun_out/s23/prof
ls -la gpurun_out/s23
exit $rc
