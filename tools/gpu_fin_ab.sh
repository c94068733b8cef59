# A/B of the dot-finish kernel shape (KLE_FIN 0..3), alternating, config 2, 400 steps
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt gpurun_out/fin_ab.jsonl
for rep in 1 2; do
for f in 0 1 2 3; do
  KLE_FIN=$f step fin_${f}_${rep} 300 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-solve || exit 1
  echo "{\"fin\": $f, \"rep\": $rep, \"line\": $(tail -n 1 gpurun_out/fin_${f}_${rep}.log)}" >> gpurun_out/fin_ab.jsonl
done
done
KLE_FIN=0 step prof_fin0 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof0 -o p --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --no-solve || exit 1
KLE_FIN=2 step prof_fin2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof2 -o p --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --no-solve || exit 1
echo done
