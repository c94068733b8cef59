# k_element_mfma register budget A/B (2 vs 3 waves/SIMD, 16-point chunks) at config 4 (p = 6) and config 2
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step elem_tests 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 150 --timeout-method thread -k "element_kernel or batched" || exit 1
for w in 2 3; do
KLE_TIMING=1 KLE_ELEMENT_WAVES=$w step gab_cfg4_w$w 600 python -u tools/graph_ab.py 18,18,18 7 || exit 1
KLE_TIMING=1 KLE_ELEMENT_WAVES=$w step gab_cfg2_w$w 600 python -u tools/graph_ab.py 20,16,16 5 || exit 1
done
grep -h "element batches\|elements + gathers" gpurun_out/gab_cfg*_w*.log
