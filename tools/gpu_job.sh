#!/bin/bash
# One parametrised GPU job (replaces the per-experiment gpu_r02*.sh scripts).
#   gpurun --timeout 1200 -- 'TAG=r03a bash tools/gpu_job.sh "tests:tests/test_gpu_sym.py" "ab:[{},{\"spmv_sym\":0}]"'
# Each argument is one step "recipe:args", run in order; a fault, abort or
# timeout ends the job (tools/gpu_steps.sh).  Recipes:
#   tests:<pytest args>     GPU tests (one process, per-test timeout)
#   ab:<json> [cg_ab args]  in-process CG A/B of tuning knobs (tools/cg_ab.py)
#   spmv:<json> [args]      in-process SpMV A/B of tuning knobs (tools/spmv_ab.py)
#   bench:<bench.py args>   one bench line -> $OUT/bench_<n>.json
#   prof:<bench.py args>    rocprofv3 kernel trace + stats of a bench run
#   pmc:<bench.py args>     PMC FETCH_SIZE and WRITE_SIZE passes (separate runs)
#   sprof:<spmv_ab.py args> rocprofv3 kernel trace + stats of an in-process SpMV A/B
#   sq:<spmv_ab.py args>    one PMC pass of 8 SQ counters (wave cycles, waits, active VALU/SALU/LDS) over tools/spmv_ab.py
#   cmd:<command>           any command (env assignments allowed: cmd:KLE_TRANSPORT=host python bench.py --gpus 2)
#   smoke:                  __graft_entry__.smoke()
#   suite:                  the whole GPU suite + smoke
# Outputs: gpurun_out/$TAG/ (logs, json lines, rocprof csv).
source tools/gpu_steps.sh
TAG=${TAG:-job}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
rm -f gpurun_out/steps.txt
export TMPDIR=/tmp
n=0
for spec in "$@"; do
  n=$((n + 1))
  recipe=${spec%%:*}
  args=${spec#*:}
  [ "$args" = "$spec" ] && args=""
  name="${TAG}_${n}_${recipe}"
  case $recipe in
    tests)
      step $name 900 python -u -m pytest $args -m gpu -x -v --timeout 240 --timeout-method thread || exit 1
      grep -E "passed|failed|PASSED|FAILED|ERROR" "gpurun_out/$name.log" > "$OUT/${n}_tests.txt" ;;
    ab)
      step $name 900 python -u tools/cg_ab.py $args || exit 1
      grep '^{' "gpurun_out/$name.log" > "$OUT/${n}_ab.jsonl" ;;
    spmv)
      step $name 900 python -u tools/spmv_ab.py $args || exit 1
      grep '^{' "gpurun_out/$name.log" > "$OUT/${n}_spmv.jsonl" ;;
    bench)
      step $name 900 python -u bench.py $args || exit 1
      tail -n 1 "gpurun_out/$name.log" > "$OUT/${n}_bench.json" ;;
    prof)
      step $name 900 rocprofv3 --kernel-trace --stats -d $OUT/${n}_prof -o prof --output-format csv -- python3 bench.py $args || exit 1
      grep '^{' "gpurun_out/$name.log" | tail -n 1 > "$OUT/${n}_prof_bench.json" ;;
    pmc)
      step ${name}_f 400 timeout -s KILL 380 rocprofv3 --pmc FETCH_SIZE -d $OUT/${n}_pmc_f -o f --output-format csv -- python3 bench.py $args || exit 1
      step ${name}_w 400 timeout -s KILL 380 rocprofv3 --pmc WRITE_SIZE -d $OUT/${n}_pmc_w -o w --output-format csv -- python3 bench.py $args || exit 1
      # per-launch HBM bytes of the kernel that ran, with its algorithmic bytes (bench line of the FETCH pass)
      grep '^{' "gpurun_out/${name}_f.log" | tail -n 1 > "$OUT/${n}_pmc_bench.json"
      step ${name}_t 60 python tools/pmc_traffic.py $OUT/${n}_pmc_f $OUT/${n}_pmc_w $OUT/${n}_pmc_bench.json auto $OUT/${n}_traffic.json || exit 1 ;;
    sq)
      step $name 400 timeout -s KILL 380 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d $OUT/${n}_sq -o sq --output-format csv -- python3 tools/spmv_ab.py $args || exit 1 ;;
    sprof)
      step $name 600 rocprofv3 --kernel-trace --stats -d $OUT/${n}_sprof -o prof --output-format csv -- python3 tools/spmv_ab.py $args || exit 1
      grep '^{' "gpurun_out/$name.log" > "$OUT/${n}_sprof.jsonl" || true ;;
    cmd)
      step $name 900 env $args || exit 1
      grep '^{' "gpurun_out/$name.log" > "$OUT/${n}_cmd.jsonl" || true ;;
    smoke)
      step $name 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
      tail -n 3 "gpurun_out/$name.log" > "$OUT/${n}_smoke.txt" ;;
    suite)
      step $name 1500 python -u -m pytest tests -m gpu -x -v --durations=80 --timeout 240 --timeout-method thread || exit 1
      grep -E "passed|failed|PASSED|FAILED|ERROR" "gpurun_out/$name.log" > "$OUT/${n}_suite.txt"
      step ${name}_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    *)
      echo "unknown recipe '$recipe'"; exit 2 ;;
  esac
done
echo "job $TAG done"
