set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_pmemo.py > gpurun_out/pm_tests.log 2>&1
rc=$?
tail -25 gpurun_out/pm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --run-mode 6 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pm_bench.log 2>&1
rc=$?
tail -3 gpurun_out/pm_bench.log
exit $rc
