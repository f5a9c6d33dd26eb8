cd $GRAFT_REPO_ROOT
for v in mw16 mw8 mw16 mw8; do DSORT_LIB=build_variants/$v/libdsort.so timeout -k 10 120 python scripts/dev/ktime.py --reps 6 || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_bucket.py -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/t_mw8.log 2>&1; echo "tests $?"; tail -3 gpurun_out/t_mw8.log
