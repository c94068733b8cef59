# 4 vs 8 waves per workgroup on the mid-size parts (1/4 and 1/2 of config 2): where the default switches
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
for r in 1 2 3; do
for w in 4 8; do
KLE_SPMV_WAVES=$w step wvm_quarter_${w}_$r 300 python bench.py --nelem 20,16,4 --steps 2000 --no-cpu-baseline --no-solve || exit 1
KLE_SPMV_WAVES=$w step wvm_half_${w}_$r 300 python bench.py --nelem 20,16,8 --steps 1000 --no-cpu-baseline --no-solve || exit 1
done
done
for f in gpurun_out/wvm_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["avg_launch_ms"],5))')"; done
