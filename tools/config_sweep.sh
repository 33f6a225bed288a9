# SURVEY §8(d) configs C2-C5 on one GPU (bench.py lines without the CPU leg):
#   bash tools/config_sweep.sh  -> gpurun_out/configs.jsonl
set -e
mkdir -p gpurun_out
OUT=gpurun_out/configs.jsonl
: > $OUT
run() { timeout -k 10 240 python bench.py --no-cpu --steps 3 --warmup 1 "$@" 2>> gpurun_out/configs.err | tail -1 >> $OUT; tail -1 $OUT | cut -c1-200; }
run --instance lands --scenarios 10000 --vertices 64
for v in 64 1024 16384 65536; do run --instance ssn --scenarios 100000 --vertices $v; done
for v in 64 512 4096; do run --instance storm --scenarios 1000000 --vertices $v; done
run --instance transship --scenarios 1000000 --epigraphs 4 --importance-scale 1.5 --vertices 4096
echo done
