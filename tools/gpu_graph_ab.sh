# hipGraph A/B of the single-rank CG loop + setup phase timings (config 2, its 1/8 slab, config 4)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export KLE_TIMING=1
step gab_cfg2 300 python -u tools/graph_ab.py 20,16,16 5 || exit 1
step gab_cfg2_hostpat 300 env KLE_HOST_PATTERN=1 python -u tools/graph_ab.py 20,16,16 5 || exit 1
step gab_eighth 300 python -u tools/graph_ab.py 20,16,2 5 || exit 1
step gab_cfg4 600 python -u tools/graph_ab.py 18,18,18 7 || exit 1
grep -h "^{" gpurun_out/gab_*.log
