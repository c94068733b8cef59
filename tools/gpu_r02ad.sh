#!/bin/bash
# Round 2: single-reduction CG grid sizes: update (prologue reads 2 G partials) and (w,u) partial launch
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02ad
export TMPDIR=/tmp
V='[{},{"upd_blocks":512},{"upd_blocks":1024},{"dot_blocks":512},{"upd_blocks":512,"dot_blocks":512},{"upd_blocks":1024,"dot_blocks":512}]'
step ab_full 500 python tools/cg_ab.py "$V" --reps 5 --its 200 || exit 1
cp gpurun_out/ab_full.log gpurun_out/r02ad/grids_full.jsonl
step ab_eighth 400 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 5 --its 500 || exit 1
cp gpurun_out/ab_eighth.log gpurun_out/r02ad/grids_eighth.jsonl
echo done
