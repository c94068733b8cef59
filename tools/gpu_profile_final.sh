# Round profiling pass: smoke, default bench (+aij, +ops), rocprofv3 kernel stats of
# the bench command, PMC FETCH/WRITE passes (traffic), config 4 / config-5-size /
# 1/8-slab / unstructured-1M benches.  Outputs under gpurun_out/final/.
#   gpurun --timeout 2400 -- 'bash tools/gpu_profile_final.sh'
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
mkdir -p gpurun_out/final
export TMPDIR=/tmp
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default 600 python bench.py --aij --ops || exit 1
tail -n 1 gpurun_out/bench_default.log > gpurun_out/final/bench_default.json
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof_bench -o bench --output-format csv -- python3 bench.py --steps 200 --no-cpu-baseline || exit 1
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/final/pmc_fetch -o f --output-format csv -- python3 bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/final/pmc_write -o w --output-format csv -- python3 bench.py --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
step bench_cfg4 900 python bench.py --nelem 18,18,18 --ngl 7 --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
tail -n 1 gpurun_out/bench_cfg4.log > gpurun_out/final/bench_cfg4.json
step bench_cfg5 900 python bench.py --mesh unstructured --nelem 40,32,32 --steps 50 --warmup 5 --cpu-seconds 10 || exit 1
tail -n 1 gpurun_out/bench_cfg5.log > gpurun_out/final/bench_cfg5_umesh.json
step bench_eighth 300 python bench.py --nelem 20,16,2 --steps 400 --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/bench_eighth.log > gpurun_out/final/bench_eighth_slab.json
step bench_umesh 600 python bench.py --mesh unstructured --ops --no-cpu-baseline || exit 1
tail -n 1 gpurun_out/bench_umesh.log > gpurun_out/final/bench_umesh.json
echo done
