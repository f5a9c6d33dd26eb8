set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_faults.py > gpurun_out/r6_bxpure_tests.log 2>&1 || { tail -40 gpurun_out/r6_bxpure_tests.log; exit 1; }
tail -3 gpurun_out/r6_bxpure_tests.log
timeout -k 10 500 python3 bench.py --gpus 1 --path samplesort --no-cpu-baseline --legs c4 > gpurun_out/r6_bench_ss_bxpure.json 2> gpurun_out/r6_bench_ss_bxpure.err || { tail -20 gpurun_out/r6_bench_ss_bxpure.err; exit 1; }
tail -c 1500 gpurun_out/r6_bench_ss_bxpure.json
