#!/bin/bash
# Round-4 A/B: cut_argmax2_kernel fragment-group sizes (KG) and the pipelined variant (PF), storm
A="--steps 20 --warmup 5 --no-cpu --spot 0 --trajectory 0"
steps=("base|150|python bench.py $A > gpurun_out/s25/base.json")
for v in kg3 kg5 kg10 kg15 pf; do steps+=("$v|150|TWOSD_LIB=$v python bench.py $A > gpurun_out/s25/$v.json"); done
steps+=("base2|150|python bench.py $A > gpurun_out/s25/base2.json")
bash tools/gpu_session.sh gpurun_out/s25 "${steps[@]}"
