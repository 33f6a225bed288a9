mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-600
