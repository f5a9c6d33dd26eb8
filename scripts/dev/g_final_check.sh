cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/tests_final.log 2>&1 || { tail -20 gpurun_out/tests_final.log; exit 1; }
tail -2 gpurun_out/tests_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/torchrun_final.log 2>&1 || { tail -20 gpurun_out/torchrun_final.log; exit 1; }
grep -o '"value": [0-9.]*, "ms_per_step": [0-9.]*' gpurun_out/torchrun_final.log
