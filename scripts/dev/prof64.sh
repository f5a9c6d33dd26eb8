cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/p64 -o run -- python3 $R/scripts/dev/ktime.py --dtype i64 --dist zipf --keys "2**30" --reps 2
