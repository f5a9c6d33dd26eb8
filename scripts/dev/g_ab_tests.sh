cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -x -m gpu --timeout 170 --timeout-method thread > gpurun_out/tests.log 2>&1
st=$?; echo "tests exit $st"; tail -4 gpurun_out/tests.log
[ $st -ne 0 ] && exit $st
VS="csw0" bash scripts/dev/ab_multi.sh > gpurun_out/ab.log 2>&1 || exit $?
cat gpurun_out/ab.log | grep -v amdgpu.ids
