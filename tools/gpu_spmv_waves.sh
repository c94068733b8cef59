# Waves per workgroup of the default SpMV kernel (KLE_SPMV_WAVES 1/2/4/8/16): config 2, its 1/8
# slab, the unstructured 1M mesh; alternating runs.  Usage: bash tools/gpu_spmv_waves.sh "4 8 16" 3
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
WS=${1:-"4 1 2 8 16"}
REPS=${2:-2}
for r in $(seq 1 $REPS); do
for w in $WS; do
KLE_SPMV_WAVES=$w step wv_full_${w}_$r 300 python bench.py --steps 1000 --no-cpu-baseline --no-solve || exit 1
KLE_SPMV_WAVES=$w step wv_eighth_${w}_$r 300 python bench.py --nelem 20,16,2 --steps 2000 --no-cpu-baseline --no-solve || exit 1
KLE_SPMV_WAVES=$w step wv_umesh_${w}_$r 300 python bench.py --mesh unstructured --steps 1000 --no-cpu-baseline --no-solve || exit 1
done
done
for f in gpurun_out/wv_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["avg_launch_ms"],5))')"; done
