#!/bin/bash
# Round-6 GPU pass L: where the fp32 argmax waits -- the cut alone (storm 1M at x_EV, |V| = 4096) under
# one PMC pass of LDS / MFMA / wait counters, and its timing.
set -u
mkdir -p gpurun_out/r06l
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/cut_speed.py 1000000 4096 5 || exit 1
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cut.py > gpurun_out/r06l_tests.log 2>&1 || { tail -20 gpurun_out/r06l_tests.log; exit 1; }
tail -1 gpurun_out/r06l_tests.log
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES -d gpurun_out/r06l/p1 -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 2 > gpurun_out/r06l/p1.json 2> gpurun_out/r06l/p1.err || { tail -5 gpurun_out/r06l/p1.err; exit 1; }
python3 tools/prof_reduce.py gpurun_out/r06l/p1 gpurun_out/r06l/p1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM -d gpurun_out/r06l/p2 -o run --output-format csv -- python3 tools/cut_speed.py 1000000 4096 2 > gpurun_out/r06l/p2.json 2> gpurun_out/r06l/p2.err || { tail -5 gpurun_out/r06l/p2.err; exit 1; }
python3 tools/prof_reduce.py gpurun_out/r06l/p2 gpurun_out/r06l/p2
