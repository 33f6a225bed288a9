# kernel trace of a short bench run (default storm 125k = the per-GPU share at 8 GPUs) and
# the timeline of one step: bash tools/trace_gaps.sh [scenarios] -> gpurun_out/gaps/
set -e
NS=${1:-125000}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gaps/t -o run --output-format csv -- python3 bench.py --scenarios $NS --steps 2 --warmup 1 --no-cpu "$@" > gpurun_out/gaps/bench.json 2> gpurun_out/gaps/err.log
python3 tools/trace_timeline.py gpurun_out/gaps > gpurun_out/gaps/timeline.txt
tail -45 gpurun_out/gaps/timeline.txt
