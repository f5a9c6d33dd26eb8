set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests -m gpu > gpurun_out/r6_l64_tests.log 2>&1 || { tail -30 gpurun_out/r6_l64_tests.log; exit 1; }
tail -2 gpurun_out/r6_l64_tests.log
timeout -k 10 600 python3 -u scripts/dev/sweep_r6.py --quick > gpurun_out/r6_l64_sweep.log 2>&1 || { tail -5 gpurun_out/r6_l64_sweep.log; exit 1; }
tail -1 gpurun_out/r6_l64_sweep.log
