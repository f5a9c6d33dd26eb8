cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for d in uniform byte ref100 few; do
  timeout -k 10 120 python3 -u scripts/dev/ktime.py --dist $d --reps 5 >> gpurun_out/r5_start_ktime.log 2>&1 || exit $?
done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/r5_start_bench.json 2> gpurun_out/r5_start_bench.err || exit $?
echo done
