cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/sbsA -o run -- python3 $R/scripts/dev/ktime.py --reps 4 > $R/gpurun_out/sbsA.log 2>&1 || exit 1
DSORT_LIB=$R/build_variants/base/libdsort.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/sbsB -o run -- python3 $R/scripts/dev/ktime.py --reps 4 > $R/gpurun_out/sbsB.log 2>&1 || exit 1
grep -h sb_scan $R/gpurun_out/sbsA/*stats.csv $R/gpurun_out/sbsB/*stats.csv | cut -c1-160
