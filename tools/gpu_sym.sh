# Prototype runs of tools/sym_proto2 (symmetric position-class SpMV, uniform class lattices)
source tools/gpu_steps.sh
step sym2_check 120 tools/sym_proto2 6 5 4 4 0 1 1 1 5 4 4 || exit 1
# args: full check nt order reps split B
for cfg in "0 0 1 1 200 4 4" "0 0 0 1 200 4 4" "0 0 1 1 200 2 4" "0 0 1 0 200 4 4" "0 0 1 1 200 4 2" "1 0 1 1 200 4 4" "1 0 0 1 200 4 4"; do
  n=$(echo $cfg | tr ' ' '_')
  step sym2_$n 120 tools/sym_proto2 20 16 16 4 $cfg || exit 1
done
cat gpurun_out/sym2_*.log
