set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py tests/test_gpu_partition.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "4]" > gpurun_out/t_band.log 2>&1
rc=$?; tail -3 gpurun_out/t_band.log; [ $rc -ne 0 ] && exit $rc
for T in 0 1 2; do
  echo "== tile $T"; SEM_BAND_TILE=$T timeout -k 10 120 python tools/kbench.py --algo 4 --meshes 8:64,12:128,8:256,8:1024 --reps 200 || exit $?
done
