# In-process A/B of the CG loop knobs (tools/cg_ab.py): config 2 and its 1/8 slab
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
V='[{"cg_rowdot":1,"cg_finish":0},{"cg_rowdot":0,"cg_finish":0},{"cg_rowdot":1,"cg_finish":2},{"cg_rowdot":0,"cg_finish":2}]'
step cgab_full 400 python tools/cg_ab.py "$V" --reps 8 --its 200 || exit 1
step cgab_eighth 300 python tools/cg_ab.py "$V" --nelem 20,16,2 --reps 8 --its 1000 || exit 1
tail -n 1 gpurun_out/cgab_full.log gpurun_out/cgab_eighth.log
