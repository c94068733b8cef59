# A/B: SpMV row-dot epilogue (KLE_ROWDOT=1) vs unrolled (u, w) pass in the finish kernel (0); finish shapes 0 / 2
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt gpurun_out/rowdot_ab.jsonl
for rep in 1 2; do
for rd in 1 0; do
for f in 0 2; do
  KLE_ROWDOT=$rd KLE_FIN=$f step rd_${rd}_${f}_${rep} 300 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-solve || exit 1
  echo "{\"rowdot\": $rd, \"fin\": $f, \"rep\": $rep, \"line\": $(tail -n 1 gpurun_out/rd_${rd}_${f}_${rep}.log)}" >> gpurun_out/rowdot_ab.jsonl
done
done
done
KLE_ROWDOT=0 KLE_FIN=0 step prof_rd0 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rd_prof0 -o p --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --no-solve || exit 1
KLE_ROWDOT=0 KLE_FIN=2 step prof_rd0f2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rd_prof0f2 -o p --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline --no-solve || exit 1
echo done
