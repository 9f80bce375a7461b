set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r03c/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -30 gpurun_out/r03c/pytest_gpu.log
for c in C2 C3 C5; do
  [ -f gpurun_out/fullbatch_${c}_worst.npz ] || continue
  for v in . _ab/base; do
    timeout -k 10 120 python tools/eval_rows.py $v gpurun_out/fullbatch_${c}_worst.npz $c fast || exit $?
    timeout -k 10 120 python tools/eval_rows.py $v gpurun_out/fullbatch_${c}_worst.npz $c precise || exit $?
  done
done
bash tools/ab_bench.sh r03c_ab "C5 dense:C2 C2" base cur
