set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "group_fixpoint or bf16_encode or lowp" > gpurun_out/fg_test.log 2>&1
for n in 10000 20000 30000; do
 for m in 0 1; do
  SRNN_FIX_GROUP=$m timeout -k 10 120 python -u bench/configs.py --only 2 --n2 $n --reps 20 >> gpurun_out/fg_bench.log 2>&1
  echo "n=$n mode=$m" >> gpurun_out/fg_bench.log
 done
done
