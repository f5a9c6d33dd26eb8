#!/bin/bash
# rocprofv3 kernel-trace summary of scripts/dev/ktime.py (2^30 uniform int32, default path)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/pb -o run -- python3 $R/scripts/dev/ktime.py --reps 2
