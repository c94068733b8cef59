#!/bin/bash
# Round 2: reserved CUs for the comm stream (KLE_RESERVE_CUS) x {cg, pipecg}, 1/8 slab and full size
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/r02j
export TMPDIR=/tmp
V='[{"_ksp":"cg"},{"_ksp":"pipecg"}]'
for k in 0 1 8 32; do
  KLE_RESERVE_CUS=$k step cgab_eighth_r$k 300 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 4 --its 1000 || exit 1
  tail -n 1 gpurun_out/cgab_eighth_r$k.log
  KLE_RESERVE_CUS=$k step cgab_full_r$k 300 python tools/cg_ab.py "$V" --reps 4 --its 200 || exit 1
  tail -n 1 gpurun_out/cgab_full_r$k.log
done
echo done
