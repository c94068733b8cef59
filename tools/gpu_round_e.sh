# element kernel (LDS-staged index math) parity + timing; stream-copy variants
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
step elem_tests 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 150 --timeout-method thread -k "element_kernel or batched or assembly_matches" || exit 1
KLE_TIMING=1 step gab_cfg4 600 python -u tools/graph_ab.py 18,18,18 7 || exit 1
KLE_TIMING=1 KLE_ELEMENT_VALU=1 step gab_cfg4_valu 600 python -u tools/graph_ab.py 18,18,18 7 || exit 1
step stream 120 python -c "
import pynama_amd as pa
c = pa.get_ctx()
import ctypes as C
from pynama_amd._lib import call
for mode in (0, 4, 1):
    for nb in (1 << 30, 1 << 32):
        g = C.c_double(); call('kle_stream_bench', c.h, nb, 20, mode, C.byref(g)); print('mode', mode, 'bytes', nb, 'GB/s', round(g.value, 1))
" || exit 1
cat gpurun_out/stream.log
grep -h "k_element\|^{" gpurun_out/gab_cfg4*.log | cut -c1-200
