set -o pipefail
mkdir -p gpurun_out
( for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --codec --keys 2**28 --steps 5 --warmup 2 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', {k: d[k] for k in d if 'ms' in k or k=='value'}, d.get('roofline',{}).get('stages',''))" || exit $?
  DSORT_LIB=$PWD/build_variants/textnt/libdsort.so timeout -k 10 200 python3 bench.py --codec --keys 2**28 --steps 5 --warmup 2 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('textnt', {k: d[k] for k in d if 'ms' in k or k=='value'}, d.get('roofline',{}).get('stages',''))" || exit $?
done ) > gpurun_out/r6_ab_text_nt.log 2>&1
