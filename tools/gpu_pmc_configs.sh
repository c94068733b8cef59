# PMC HBM traffic of the default SpMV kernel on config 4 (p = 6) and the config-5-size
# unstructured mesh (FETCH_SIZE / WRITE_SIZE passes, one counter group per run)
source tools/gpu_steps.sh
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
step pmc_f_cfg4 400 timeout -s KILL 380 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_cfg4 -o f --output-format csv -- python3 bench.py --nelem 18,18,18 --ngl 7 --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
step pmc_w_cfg4 400 timeout -s KILL 380 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_cfg4 -o w --output-format csv -- python3 bench.py --nelem 18,18,18 --ngl 7 --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
step pmc_f_cfg5 400 timeout -s KILL 380 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f_cfg5 -o f --output-format csv -- python3 bench.py --mesh unstructured --nelem 40,32,32 --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
step pmc_w_cfg5 400 timeout -s KILL 380 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w_cfg5 -o w --output-format csv -- python3 bench.py --mesh unstructured --nelem 40,32,32 --steps 10 --warmup 0 --no-solve --no-cpu-baseline || exit 1
echo done
